"""Test helpers: BGZF files of arbitrary block sizes and a digest of what the
native ingest packs from a file (or a range of it)."""
import gzip
import hashlib
import random
import struct
import zlib


def bgzf_block(data: bytes, level=1) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    cdata = c.compress(data) + c.flush()
    bsize = 12 + 6 + len(cdata) + 8
    head = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize - 1)
    return head + cdata + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def reblock(src: str, dst: str, lo: int, hi: int, seed: int = 0, level: int = 1) -> int:
    """Rewrite a BGZF file with blocks of lo..hi uncompressed bytes (BGZF allows
    any size up to 64 KiB); returns the block count."""
    raw = gzip.decompress(open(src, "rb").read())
    rng = random.Random(seed)
    n = 0
    with open(dst, "wb") as f:
        p = 0
        while p < len(raw):
            k = rng.randint(lo, hi)
            f.write(bgzf_block(raw[p:p + k], level))
            p += k
            n += 1
        f.write(bgzf_block(b""))
    return n


def ingest_digest(path, start_voff=0, end_voff=-1, reads=1 << 18):
    """sha256 over every batch the ingest packs from [start_voff, end_voff)
    (the dcr_batch arrays, the family table and both side-record streams),
    plus the counters."""
    from duplexumiconsensusreads_amd import native_io
    ing = native_io.Ingest(path, start_voff=start_voff, end_voff=end_voff)
    hb = native_io.HostBatch(reads=reads)
    h = hashlib.sha256()
    n = 0
    while True:
        ing.next(hb)
        n += 1
        pb = hb.packed()
        for k in sorted(vars(pb)):
            v = getattr(pb, k)
            if hasattr(v, "tobytes"):
                h.update(v.tobytes())
        h.update(repr(hb.table()).encode())
        h.update(hb.side("exc").tobytes())
        h.update(hb.side("filt").tobytes())
        h.update(struct.pack("<ii", hb.end_kind, hb.s.err_kind))
        if hb.end_kind != native_io.END_FULL:
            break
    c = ing.counters()
    gpu = ing.gpu_inflate
    ing.close()
    return h.hexdigest(), n, c, gpu
