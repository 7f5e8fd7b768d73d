"""The GPU BGZF block compressor's algorithm (csrc/dcr_deflate.h), run lane
by lane on the host (dcr_deflate_emulate): every block must be one valid
BGZF member (SAM spec v1.6 §4.1: BC extra field, BSIZE, CRC32, ISIZE) that
zlib inflates back to the input, for compressible record text, random bytes
(stored-block fallback), runs, tiny and full-size blocks.  The kernel runs
the same phase code (tests/test_gpu_writer.py checks its stream)."""
import struct
import zlib

import numpy as np
import pytest

from duplexumiconsensusreads_amd import native_io


def check_member(blob, data):
    assert blob[:4] == b"\x1f\x8b\x08\x04"
    assert blob[10:16] == b"\x06\x00BC\x02\x00"
    bsize = struct.unpack_from("<H", blob, 16)[0] + 1
    assert bsize == len(blob)
    crc, isize = struct.unpack_from("<II", blob, len(blob) - 8)
    out = zlib.decompress(blob[18:-8], -15)
    assert out == data
    assert isize == len(data) and crc == zlib.crc32(data)


def record_text(n, seed):
    rng = np.random.default_rng(seed)
    parts = []
    while sum(map(len, parts)) < n:
        L = int(rng.integers(60, 160))
        seq = "".join(rng.choice(list("ACGT"), L))
        qual = bytes(rng.integers(20, 41, L) + 33).decode()
        d = ", ".join(str(int(x)) for x in rng.integers(1, 9, L))
        parts.append(f"consensus_family{int(rng.integers(1e6))}_paired-end1\0{seq}\0{qual}\0[{d}]\0".encode())
    return b"".join(parts)[:n]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 64, 255, 256, 257, 1000, 32768, 40000, 0xff00])
def test_record_text_blocks(n):
    data = record_text(n, n)
    check_member(native_io.deflate_emulate(data), data)


@pytest.mark.parametrize("n", [1, 100, 5000, 0xff00])
def test_random_bytes_take_the_stored_block(n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    blob = native_io.deflate_emulate(data)
    check_member(blob, data)
    if n > 1000:
        assert len(blob) == n + 5 + 26          # stored: BFINAL/BTYPE, LEN, NLEN
        assert blob[18] == 1


@pytest.mark.parametrize("pattern", [b"\0", b"A", b"AC", b"ACG", b"1, ", b"ACGTACGTAC"])
def test_runs(pattern):
    data = (pattern * (0xff00 // len(pattern) + 1))[:0xff00]
    blob = native_io.deflate_emulate(data)
    check_member(blob, data)
    assert len(blob) < 0xff00 // 20


def test_mixed_runs_and_noise():
    rng = np.random.default_rng(3)
    chunks = []
    while sum(map(len, chunks)) < 0xff00:
        if rng.random() < 0.5:
            chunks.append(bytes([int(rng.integers(256))]) * int(rng.integers(1, 600)))
        else:
            chunks.append(rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes())
    data = b"".join(chunks)[:0xff00]
    check_member(native_io.deflate_emulate(data), data)


def test_bad_sizes_rejected():
    with pytest.raises(Exception):
        native_io.deflate_emulate(b"")
    with pytest.raises(Exception):
        native_io.deflate_emulate(b"x" * (0xff00 + 1))


@pytest.mark.parametrize("mode", ["flat", "wide", "skewed"])
def test_batched_code_lengths_equal_plain(mode):
    """The kernel's Huffman code lengths (mr_counts: LDS loads batched, counts
    per depth) equal the plain in-place minimum-redundancy algorithm's, codes
    per length after the 15-bit limit, on random alphabets of 2..288 symbols."""
    lib = native_io.load()
    rng = np.random.default_rng({"flat": 1, "wide": 2, "skewed": 3}[mode])
    a = np.zeros(33, np.uint32)
    b = np.zeros(33, np.uint32)
    for _ in range(400):
        m = int(rng.integers(2, 289))
        if mode == "flat":
            f = rng.integers(1, 6, m)
        elif mode == "wide":
            f = rng.integers(1, 100000, m)
        else:
            f = np.where(rng.random(m) < 0.9, rng.integers(1, 4, m), rng.integers(1, 60000, m))
        f = np.sort(f).astype(np.uint32)
        assert lib.dcr_deflate_lengths_ab(f.ctypes.data, m, a.ctypes.data, b.ctypes.data) == 0
        assert (a == b).all(), (m, a, b)
        assert sum(int(a[k]) << (15 - k) for k in range(1, 16)) == 1 << 15   # complete code
