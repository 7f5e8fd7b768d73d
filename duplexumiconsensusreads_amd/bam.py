"""Minimal BAM (BGZF) reader/writer for the host side.

The reference streams BAM through pysam/htslib (DuplexUMIConsensusReads.py:1476,
:1494-1502, :1519, :1526, :1551, :1594).  pysam is absent from this image, so
the host carries its own codec for the SAM spec v1.6 BAM layout: BGZF blocks
(RFC1952 members with the BC extra field), the binary header, and records with
typed aux fields.  Throughput-critical ingest of very large files is a later
native item.  The BGZF layer runs natively when
``libdcr_bgzf.so`` (csrc/dcr_bgzf.cpp, include/dcr_bgzf.h) is built: blocks are
inflated / deflated on a pool of host threads, and the written files are
byte-identical to the Python writer's.  The Python BGZF classes below stay as
the portable codec (``DCR_BGZF=python`` forces them).
"""
from __future__ import annotations

import array
import ctypes
import os
import struct
import zlib

import numpy as np

from .records import AlignedSegment, array_subtype

_SEQ_ALPHA = "=ACMGRSVTWYHKDBN"
_SEQ_CODE = {c: i for i, c in enumerate(_SEQ_ALPHA)}
_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
_MAX_BLOCK = 0xff00

# decode table: byte -> two bases
_SEQ_PAIR = [(_SEQ_ALPHA[b >> 4] + _SEQ_ALPHA[b & 15]) for b in range(256)]
_SEQ_PAIR_NP = np.array([p.encode() for p in _SEQ_PAIR], dtype="S2")
# encode table: ASCII (either case) -> 4-bit code; '=' is 0, unknown letters 15
_SEQ_CODE_NP = np.full(256, 15, np.uint8)
for _c, _i in _SEQ_CODE.items():
    _SEQ_CODE_NP[ord(_c)] = _SEQ_CODE_NP[ord(_c.lower())] = _i


def reg2bin(beg: int, end: int) -> int:
    """SAM spec §5.3 bin of the 0-based half-open interval [beg, end)."""
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


_NATIVE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdcr_bgzf.so")
_native_lib = None


def native_bgzf():
    """The native codec library, or None when it is not built (or disabled)."""
    global _native_lib
    if _native_lib is None:
        if os.environ.get("DCR_BGZF", "") == "python" or not os.path.exists(_NATIVE_PATH):
            return None
        lib = ctypes.CDLL(_NATIVE_PATH)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.dcr_bgzf_open_read.restype = vp
        lib.dcr_bgzf_open_read.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.dcr_bgzf_read.restype = i64
        lib.dcr_bgzf_read.argtypes = [vp, vp, i64]
        lib.dcr_bgzf_close_read.restype = None
        lib.dcr_bgzf_close_read.argtypes = [vp]
        lib.dcr_bgzf_open_write.restype = vp
        lib.dcr_bgzf_open_write.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        lib.dcr_bgzf_write.restype = ctypes.c_int
        lib.dcr_bgzf_write.argtypes = [vp, ctypes.c_char_p, i64]
        lib.dcr_bgzf_close_write.restype = ctypes.c_int
        lib.dcr_bgzf_close_write.argtypes = [vp]
        lib.dcr_bgzf_last_error.restype = ctypes.c_char_p
        lib.dcr_bgzf_last_error.argtypes = []
        _native_lib = lib
    return _native_lib


def _native_error(lib, what):
    return OSError(f"{what}: {lib.dcr_bgzf_last_error().decode()}")


class NativeBGZFReader:
    """BGZF decompressed stream from csrc/dcr_bgzf.cpp (threaded inflate)."""

    def __init__(self, path, n_threads=0):
        self._lib = native_bgzf()
        self._h = self._lib.dcr_bgzf_open_read(os.fsencode(path), n_threads)
        if not self._h:
            raise _native_error(self._lib, "BGZF open")

    def read(self, n):
        buf = ctypes.create_string_buffer(n)
        got = self._lib.dcr_bgzf_read(self._h, buf, n)
        if got < 0:
            raise ValueError(self._lib.dcr_bgzf_last_error().decode())
        return buf.raw[:got]

    def close(self):
        if self._h:
            self._lib.dcr_bgzf_close_read(self._h)
            self._h = None


class NativeBGZFWriter:
    """BGZF writer from csrc/dcr_bgzf.cpp (threaded deflate, same bytes as BGZFWriter)."""

    def __init__(self, path, level=6, n_threads=0):
        self._lib = native_bgzf()
        self._h = self._lib.dcr_bgzf_open_write(os.fsencode(path), level, n_threads)
        if not self._h:
            raise _native_error(self._lib, "BGZF open")
        self._buf = bytearray()

    def write(self, data):
        self._buf += data
        if len(self._buf) >= 1 << 20:
            self._push()

    def _push(self):
        if self._buf:
            if self._lib.dcr_bgzf_write(self._h, bytes(self._buf), len(self._buf)) != 0:
                raise _native_error(self._lib, "BGZF write")
            self._buf = bytearray()

    def close(self):
        if self._h:
            self._push()
            rc = self._lib.dcr_bgzf_close_write(self._h)
            self._h = None
            if rc != 0:
                raise _native_error(self._lib, "BGZF close")


def open_bgzf_reader(path):
    return NativeBGZFReader(path) if native_bgzf() is not None else BGZFReader(path)


def bgzf_stream(path):
    """The whole decompressed byte stream of a BGZF file."""
    r = open_bgzf_reader(path)
    out = bytearray()
    while True:
        chunk = r.read(1 << 22)
        if not chunk:
            break
        out += chunk
    r.close()
    return bytes(out)


def open_bgzf_writer(path, level=6):
    return NativeBGZFWriter(path, level) if native_bgzf() is not None else BGZFWriter(path, level)


class BGZFReader:
    def __init__(self, path):
        self._f = open(path, "rb")
        self._buf = b""
        self._pos = 0
        self._eof = False

    def _fill(self):
        hdr = self._f.read(18)
        if len(hdr) < 18:
            self._eof = True
            return False
        if hdr[:4] != b"\x1f\x8b\x08\x04":
            raise ValueError("not a BGZF file")
        xlen = struct.unpack_from("<H", hdr, 10)[0]
        extra = hdr[12:18] + self._f.read(xlen - 6)
        bsize = None
        i = 0
        while i < len(extra):
            si1, si2, slen = extra[i], extra[i + 1], struct.unpack_from("<H", extra, i + 2)[0]
            if si1 == 66 and si2 == 67:
                bsize = struct.unpack_from("<H", extra, i + 4)[0]
            i += 4 + slen
        if bsize is None:
            raise ValueError("BGZF block without BC field")
        rest = self._f.read(bsize - xlen - 19 + 8)
        if len(rest) != bsize - xlen - 19 + 8:
            raise ValueError("truncated BGZF block")
        cdata = rest[:-8]
        crc, isize = struct.unpack("<II", rest[-8:])
        data = zlib.decompress(cdata, -15)
        if len(data) != isize or (zlib.crc32(data) & 0xffffffff) != crc:
            raise ValueError("BGZF block CRC32 / ISIZE mismatch")
        self._buf = self._buf[self._pos:] + data
        self._pos = 0
        return True

    def read(self, n):
        while len(self._buf) - self._pos < n:
            if not self._fill():
                break
        out = self._buf[self._pos:self._pos + n]
        self._pos += len(out)
        return out

    def close(self):
        self._f.close()


class BGZFWriter:
    def __init__(self, path, level=6):
        self._f = open(path, "wb")
        self._buf = bytearray()
        self._level = level

    def write(self, data):
        self._buf += data
        while len(self._buf) >= _MAX_BLOCK:
            self._flush_block(bytes(self._buf[:_MAX_BLOCK]))
            del self._buf[:_MAX_BLOCK]

    def _flush_block(self, data):
        co = zlib.compressobj(self._level, zlib.DEFLATED, -15)
        cdata = co.compress(data) + co.flush()
        bsize = len(cdata) + 25
        hdr = struct.pack("<4BIBBHBBHH", 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6, 66, 67, 2, bsize)
        self._f.write(hdr + cdata + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data)))

    def close(self):
        if self._buf:
            self._flush_block(bytes(self._buf))
            self._buf = bytearray()
        self._f.write(_BGZF_EOF)
        self._f.close()


class BamHeader:
    def __init__(self, text="", references=(), lengths=()):
        self.text = text
        self.references = list(references)
        self.lengths = list(lengths)

    def encode(self):
        t = self.text.encode()
        out = bytearray(b"BAM\x01" + struct.pack("<i", len(t)) + t)
        out += struct.pack("<i", len(self.references))
        for name, ln in zip(self.references, self.lengths):
            nb = name.encode() + b"\x00"
            out += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
        return bytes(out)


def _decode_tags(buf, off, end):
    tags = []
    while off < end:
        tag = buf[off:off + 2].decode()
        t = chr(buf[off + 2])
        off += 3
        if t == "A":
            v = chr(buf[off]); off += 1
        elif t in "cCsSiI":
            fmt = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}[t]
            v = struct.unpack_from(fmt, buf, off)[0]; off += struct.calcsize(fmt)
        elif t == "f":
            v = struct.unpack_from("<f", buf, off)[0]; off += 4
        elif t == "d":
            v = struct.unpack_from("<d", buf, off)[0]; off += 8
        elif t in "ZH":
            e = buf.index(b"\x00", off)
            v = buf[off:e].decode(); off = e + 1
        elif t == "B":
            sub = chr(buf[off]); n = struct.unpack_from("<i", buf, off + 1)[0]; off += 5
            code = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}[sub]
            a = array.array(code)
            a.frombytes(bytes(buf[off:off + n * a.itemsize])); off += n * a.itemsize
            v = a
        else:
            raise ValueError(f"bad tag type {t}")
        tags.append([tag, t, v])
    return tags


def decode_record(buf: bytes) -> AlignedSegment:
    (tid, pos, l_rn, mapq, _bin, n_cig, flag, l_seq, ntid, npos, tlen) = struct.unpack_from(
        "<iiBBHHHiiii", buf, 0)
    off = 32
    r = AlignedSegment()
    r.query_name = buf[off:off + l_rn - 1].decode(); off += l_rn
    cig = struct.unpack_from(f"<{n_cig}I", buf, off); off += 4 * n_cig
    r._cigar = [(c & 15, c >> 4) for c in cig] or None
    nb = (l_seq + 1) // 2
    seq = _SEQ_PAIR_NP[np.frombuffer(buf, np.uint8, nb, off)].tobytes()[:l_seq].decode() if nb else ""
    off += nb
    qual = buf[off:off + l_seq]; off += l_seq
    r._seq = seq or None
    if l_seq and qual[0] != 0xff:
        r._qual = array.array("B", qual)
    else:
        r._qual = None
    r.reference_id, r.reference_start, r._mapq, r.flag = tid, pos, mapq, flag
    r.next_reference_id, r.next_reference_start, r.template_length = ntid, npos, tlen
    r._tags = _decode_tags(buf, off, len(buf))
    return r


def _encode_tag(tag, code, v):
    out = bytearray(tag.encode())
    if code == "A":
        out += b"A" + v.encode()[:1]
    elif code in "cCsSiI":
        fmt = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}[code]
        out += code.encode() + struct.pack(fmt, v)
    elif code == "f":
        out += b"f" + struct.pack("<f", v)
    elif code == "d":
        out += b"d" + struct.pack("<d", v)
    elif code in "ZH":
        out += code.encode() + str(v).encode() + b"\x00"
    elif code == "B":
        sub = array_subtype(v)
        acode = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}[sub]
        a = v if isinstance(v, array.array) and v.typecode == acode else array.array(acode, v)
        out += b"B" + sub.encode() + struct.pack("<i", len(a)) + a.tobytes()
    else:
        raise ValueError(code)
    return bytes(out)


def encode_record(r: AlignedSegment) -> bytes:
    name = (r.query_name or "*").encode() + b"\x00"
    cig = r._cigar or []
    seq = r._seq or ""
    l_seq = len(seq)
    if r.reference_start >= 0:
        rl = sum(n for op, n in cig if op in (0, 2, 3, 7, 8))
        end = r.reference_start + (rl if rl > 0 else 1)
        bin_ = reg2bin(r.reference_start, end)
    else:
        bin_ = 4680
    core = struct.pack("<iiBBHHHiiii", r.reference_id, r.reference_start, len(name), r._mapq & 0xff,
                       bin_, len(cig), r.flag, l_seq, r.next_reference_id,
                       r.next_reference_start, r.template_length)
    cigb = struct.pack(f"<{len(cig)}I", *[(n << 4) | op for op, n in cig])
    if l_seq:
        codes = _SEQ_CODE_NP[np.frombuffer(seq.encode("latin-1"), np.uint8)]
        if l_seq & 1:
            codes = np.append(codes, np.uint8(0))
        seqb = ((codes[0::2] << 4) | codes[1::2]).tobytes()
    else:
        seqb = b""
    qualb = bytes(r._qual) if r._qual is not None else b"\xff" * l_seq
    tagb = b"".join(_encode_tag(t, c, v) for t, c, v in r._tags)
    body = core + name + cigb + seqb + qualb + tagb
    return struct.pack("<i", len(body)) + body


class AlignmentFile:
    """``pysam.AlignmentFile`` subset: 'rb' iteration and 'wb' with template."""

    def __init__(self, path, mode="rb", template=None, header=None):
        self.mode = mode
        if mode.startswith("r"):
            self._r = open_bgzf_reader(path)
            magic = self._r.read(4)
            if magic != b"BAM\x01":
                raise ValueError(f"{path}: not a BAM file")
            l_text = struct.unpack("<i", self._r.read(4))[0]
            text = self._r.read(l_text).rstrip(b"\x00").decode()
            n_ref = struct.unpack("<i", self._r.read(4))[0]
            refs, lens = [], []
            for _ in range(n_ref):
                ln = struct.unpack("<i", self._r.read(4))[0]
                refs.append(self._r.read(ln)[:-1].decode())
                lens.append(struct.unpack("<i", self._r.read(4))[0])
            self.header = BamHeader(text, refs, lens)
        else:
            if template is not None:
                self.header = template.header
            elif isinstance(header, BamHeader):
                self.header = header
            else:
                self.header = BamHeader()
            self._w = open_bgzf_writer(path)
            self._w.write(self.header.encode())

    def __iter__(self):
        # records are cut from 1 MiB reads of the decompressed stream
        buf, pos = b"", 0
        unpack = struct.unpack_from
        while True:
            if len(buf) - pos < 4 or len(buf) - pos < 4 + unpack("<i", buf, pos)[0]:
                more = self._r.read(1 << 20)
                if not more:
                    if len(buf) > pos:
                        raise ValueError("truncated BAM record at the end of the file")
                    return
                buf, pos = buf[pos:] + more, 0
                continue
            n = unpack("<i", buf, pos)[0]
            yield decode_record(buf[pos + 4:pos + 4 + n])
            pos += 4 + n

    def fetch_all(self):
        return list(self)

    def write(self, r):
        self._w.write(encode_record(r))

    def close(self):
        if self.mode.startswith("r"):
            self._r.close()
        else:
            self._w.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
