"""Native BGZF codec (csrc/dcr_bgzf.cpp, include/dcr_bgzf.h) against the
portable Python codec in bam.py: same decompressed stream on read, same bytes
on write, the reference's own e2e input BAM decoded record for record, and
the failure modes (truncation, CRC, non-BGZF input).  Host code only."""
import ctypes
import os
import re
import random
import zlib

import pytest

from duplexumiconsensusreads_amd import bam

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dcr_bgzf.h")
GOLDEN_BAM = os.path.join(ROOT, "tests", "golden", "e2e_c1_small.bam")


@pytest.fixture(scope="module")
def lib():
    if bam.native_bgzf() is None:
        import __graft_entry__
        __graft_entry__.build()
    lib = bam.native_bgzf()
    assert lib is not None, "libdcr_bgzf.so not built"
    return lib


def _payload(n, seed):
    rng = random.Random(seed)
    # BAM-like: repetitive text mixed with random bytes (compressible and not)
    parts = []
    while sum(map(len, parts)) < n:
        if rng.random() < 0.5:
            parts.append(bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 3000))))
        else:
            parts.append(b"ACGT" * rng.randint(1, 5000))
    return b"".join(parts)[:n]


def test_header_functions_exported(lib):
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    names = set(re.findall(r"\b(dcr_\w+)\s*\(", txt))
    assert {"dcr_bgzf_open_read", "dcr_bgzf_write", "dcr_bam_index_records"} <= names
    raw = ctypes.CDLL(bam._NATIVE_PATH)
    for n in names:
        assert hasattr(raw, n), n


@pytest.mark.parametrize("n", [0, 1, 0xff00 - 1, 0xff00, 0xff00 + 1, 3_000_000])
def test_writer_bytes_identical_and_roundtrip(lib, tmp_path, n):
    data = _payload(n, n)
    p_py, p_nat = tmp_path / "py.gz", tmp_path / "nat.gz"
    w = bam.BGZFWriter(str(p_py))
    for i in range(0, len(data), 7777):                 # ragged writes
        w.write(data[i:i + 7777])
    w.close()
    w = bam.NativeBGZFWriter(str(p_nat))
    for i in range(0, len(data), 100_003):
        w.write(data[i:i + 100_003])
    w.close()
    assert p_py.read_bytes() == p_nat.read_bytes()
    r = bam.NativeBGZFReader(str(p_py))
    got = b"".join(iter(lambda: r.read(65_537), b""))
    r.close()
    assert got == data
    r = bam.BGZFReader(str(p_nat))
    assert r.read(len(data) + 10) == data
    r.close()


def test_reader_many_threads_small_reads(lib, tmp_path):
    data = _payload(2_000_000, 7)
    p = tmp_path / "x.gz"
    w = bam.BGZFWriter(str(p))
    w.write(data)
    w.close()
    for nt in (1, 3, 16):
        r = bam.NativeBGZFReader(str(p), n_threads=nt)
        chunks, k = [], 1
        while True:
            c = r.read(k)
            if not c:
                break
            chunks.append(c)
            k = k * 3 % 70_001 + 1
        r.close()
        assert b"".join(chunks) == data


def test_golden_bam_decodes_identically(lib, monkeypatch):
    nat = [rec.to_dict() for rec in bam.AlignmentFile(GOLDEN_BAM, "rb")]
    monkeypatch.setenv("DCR_BGZF", "python")
    monkeypatch.setattr(bam, "_native_lib", None)
    py = [rec.to_dict() for rec in bam.AlignmentFile(GOLDEN_BAM, "rb")]
    assert len(nat) == len(py) > 100
    assert nat == py


def test_bam_roundtrip_through_native_writer(lib, tmp_path):
    src = bam.AlignmentFile(GOLDEN_BAM, "rb")
    recs = list(src)
    out = tmp_path / "o.bam"
    w = bam.AlignmentFile(str(out), "wb", template=src)
    assert isinstance(w._w, bam.NativeBGZFWriter)
    for rec in recs:
        w.write(rec)
    w.close()
    back = [rec.to_dict() for rec in bam.AlignmentFile(str(out), "rb")]
    assert back == [rec.to_dict() for rec in recs]


def test_index_records(lib):
    body = [b"x" * k for k in (0, 5, 40, 3)]
    buf = b"".join(len(b).to_bytes(4, "little") + b for b in body) + b"\x10\x00"
    offs = (ctypes.c_int64 * 8)()
    used = ctypes.c_int64()
    f = lib.dcr_bam_index_records
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    n = f(buf, len(buf), offs, 8, ctypes.byref(used))
    assert n == 4 and list(offs[:4]) == [0, 4, 13, 57] and used.value == len(buf) - 2
    assert f(buf, len(buf), offs, 2, ctypes.byref(used)) == 2 and used.value == 13
    assert f(b"\xff\xff\xff\xff", 4, offs, 8, ctypes.byref(used)) == -1


def test_errors(lib, tmp_path):
    data = _payload(300_000, 3)
    p = tmp_path / "x.gz"
    w = bam.NativeBGZFWriter(str(p))
    w.write(data)
    w.close()
    raw = p.read_bytes()
    (tmp_path / "trunc.gz").write_bytes(raw[:len(raw) // 2])
    r = bam.NativeBGZFReader(str(tmp_path / "trunc.gz"))
    with pytest.raises(ValueError, match="truncated"):
        r.read(len(data))
    r.close()
    bad = bytearray(raw)
    first_len = int.from_bytes(raw[16:18], "little") + 1
    bad[first_len - 8] ^= 0xff                           # CRC of the first block
    (tmp_path / "crc.gz").write_bytes(bytes(bad))
    r = bam.NativeBGZFReader(str(tmp_path / "crc.gz"))
    with pytest.raises(ValueError, match="CRC"):
        r.read(10)
    r.close()
    (tmp_path / "plain.gz").write_bytes(zlib.compress(data))
    r = bam.NativeBGZFReader(str(tmp_path / "plain.gz"))
    with pytest.raises(ValueError, match="BGZF"):
        r.read(10)
    r.close()
    with pytest.raises(OSError):
        bam.NativeBGZFReader(str(tmp_path / "missing.gz"))
