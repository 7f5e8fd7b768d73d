"""The device BGZF inflater (csrc/dcr_inflate.hip, include/dcr_inflate.h)
against zlib on the same members: every block type (stored, fixed, dynamic),
several blocks per member and sync-flush stored blocks between them,
distances beyond the kernel's 8 KiB LDS history, periods below a wave,
65,536-byte and empty members, output offsets that are not dword aligned, the
native writer's BAMs at levels 1 and 6; and corrupted members reported by
index without touching memory outside the batch (reference: the BAM read
under ``samfile.fetch`` DuplexUMIConsensusReads.py:1476, :1519)."""
import os
import struct
import zlib

import numpy as np
import pytest

from duplexumiconsensusreads_amd import synth

pytestmark = pytest.mark.gpu


def member(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem_level=8, sync_at=()):
    co = zlib.compressobj(level, zlib.DEFLATED, -15, mem_level, strategy)
    parts, p = [], 0
    for cut in list(sync_at) + [len(data)]:
        parts.append(co.compress(data[p:cut]))
        if cut != len(data):
            parts.append(co.flush(zlib.Z_SYNC_FLUSH))
        p = cut
    parts.append(co.flush())
    cdata = b"".join(parts)
    bsize = 18 + len(cdata) + 8
    assert bsize <= 65536
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize - 1)
    return hdr + cdata + struct.pack("<II", zlib.crc32(data), len(data))


def inflate_all(inf, blob):
    from duplexumiconsensusreads_amd import _lib
    m, total = _lib.bgzf_members(blob)
    rc, out = inf.run(np.frombuffer(blob, np.uint8), m, total)
    if rc:
        print("inflate:", _lib.load().dcr_last_error().decode())
    return rc, out.tobytes(), m


@pytest.fixture(scope="module")
def inf():
    from duplexumiconsensusreads_amd import _lib
    h = _lib.Inflater(0)
    yield h
    h.close()


def test_inflate_smallest_members(inf):
    for d in (b"", b"A", b"ACGT" * 3 + b"N", b"ab" * 200):
        for level in (0, 1, 6):
            b = member(d, level=level)
            rc, out, _ = inflate_all(inf, b)
            assert rc == 0, (d[:8], level)
            assert out == d, (d[:8], level)


def test_inflate_block_types_and_edges(inf):
    rng = np.random.default_rng(1)
    rnd = rng.integers(0, 256, 30_000, dtype=np.uint8).tobytes()
    text = b"".join(b"read%07d\tMI:Z:%d/A\tRX:Z:ACGT-TTGA\n" % (i, i // 8) for i in range(1200))
    cases = [
        text[:60_000], rnd[:20_000],                                     # dynamic / stored (incompressible)
        member_data := text[:40_000],
        rnd[:9_000] * 4,                                                 # distances > 8 KiB
        b"ab" * 20_000, b"xyz0123456789" * 3000,                        # periods below 64, length-258 runs
        bytes(65536),                                                    # a full 64 KiB member
        b"", b"A", b"ACGT" * 3 + b"N",
        text[:33_333],                                                   # odd sizes: unaligned output offsets
        rnd[:777] + text[:5_000],
    ]
    blobs = []
    for i, d in enumerate(cases):
        blobs.append(member(d, level=6))
        blobs.append(member(d, level=1))
        if len(d) < 65000:
            blobs.append(member(d, level=0))                             # stored blocks
        blobs.append(member(d, level=6, strategy=zlib.Z_FIXED))
        blobs.append(member(d, level=6, strategy=zlib.Z_HUFFMAN_ONLY))
        blobs.append(member(d, level=6, strategy=zlib.Z_RLE))
        blobs.append(member(d, level=9, mem_level=1))                   # many small blocks
        if len(d) > 100:
            blobs.append(member(d, level=6, sync_at=(len(d) // 3, len(d) // 2)))   # empty stored blocks
    blob = b"".join(blobs)
    # one member per launch first (a failure names its case), then all at once
    for k, b in enumerate(blobs):
        rc, out, m = inflate_all(inf, b)
        assert rc == 0, (k, k // 8)
        assert out == zlib.decompress(b[int(m[0]["in_off"]):int(m[0]["in_off"] + m[0]["in_len"])], -15), k
    rc, out, m = inflate_all(inf, blob)
    assert rc == 0
    want = b"".join(zlib.decompress(blob[int(x["in_off"]):int(x["in_off"] + x["in_len"])], -15) for x in m)
    assert len(out) == len(want)
    assert out == want
    assert member_data in want


@pytest.mark.parametrize("level", [1, 6])
def test_inflate_native_writer_bam(inf, tmp_path, level):
    path = str(tmp_path / "c2.bam")
    synth.write_packed_bam(path, synth.packed_fixed_size(20_000, seed=3), seed=3, level=level)
    blob = open(path, "rb").read()
    rc, out, m = inflate_all(inf, blob)
    assert rc == 0
    from duplexumiconsensusreads_amd.bam import bgzf_stream
    assert out == bgzf_stream(path)
    ms, n = inf.last()
    assert n == len(m) and ms > 0


def test_inflate_reports_corrupt_members(inf):
    good = [member(b"ACGTN" * 4000 + bytes([i]) * 100, level=6) for i in range(6)]
    ref = b"".join(good)
    # a wrong CRC32 in member 2
    bad = bytearray(good[2])
    bad[-8] ^= 0x55
    rc, _, _ = inflate_all(inf, b"".join(good[:2] + [bytes(bad)] + good[3:]))
    assert rc == 3
    # a wrong ISIZE in member 4 (inside the batch's output)
    bad = bytearray(good[4])
    struct.pack_into("<I", bad, len(bad) - 4, 20_050)
    rc, _, _ = inflate_all(inf, b"".join(good[:4] + [bytes(bad)] + good[5:]))
    assert rc == 5
    # garbage in the compressed data of member 1: reported, nothing else written out of place
    rng = np.random.default_rng(5)
    for trial in range(20):
        bad = bytearray(good[1])
        k = int(rng.integers(18, len(bad) - 8))
        bad[k:k + 4] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        rc, out, _ = inflate_all(inf, b"".join(good[:1] + [bytes(bad)] + good[2:]))
        assert rc in (0, 2), trial          # member 1 fails (index + 1 = 2) unless the bytes changed nothing
        if rc == 0:
            assert zlib.decompress(bytes(bad[18:-8]), -15) == zlib.decompress(good[1][18:-8], -15)
    rc, out, _ = inflate_all(inf, ref)
    assert rc == 0
    assert out == b"".join(zlib.decompress(g[18:-8], -15) for g in good)


def _cli(inp, out, env_gpu_inflate):
    import contextlib
    import io
    import random

    from duplexumiconsensusreads_amd import cli
    old = os.environ.get("DCR_GPU_INFLATE")
    if env_gpu_inflate is None:
        os.environ.pop("DCR_GPU_INFLATE", None)
    else:
        os.environ["DCR_GPU_INFLATE"] = env_gpu_inflate
    try:
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            assert cli.main(["-i", inp, "-o", out, "--batch_reads", "200000"], rng=random.Random(4)) == 0
        return buf.getvalue()
    finally:
        if old is None:
            os.environ.pop("DCR_GPU_INFLATE", None)
        else:
            os.environ["DCR_GPU_INFLATE"] = old


@pytest.mark.parametrize("level", [1, 6])
def test_ingest_gpu_inflate_same_outputs_as_host_inflate(tmp_path, level):
    """The whole CLI over a C5-shape BAM (several chunks of members) reads
    the same records with the device inflater as with the host pool."""
    from duplexumiconsensusreads_amd import bam, cli, native_io
    inp = str(tmp_path / "in.bam")
    synth.write_packed_bam(inp, synth.packed_config(synth.CONFIGS["C5"], 60_000, seed=5), seed=5, level=level)
    os.environ["DCR_GPU_INFLATE"] = "1"
    try:
        cli.gpu_inflate(0)
    finally:
        os.environ.pop("DCR_GPU_INFLATE", None)
    ing = native_io.Ingest(inp)
    assert ing.gpu_inflate
    ing.close()
    so_gpu = _cli(inp, str(tmp_path / "g.bam"), "1")
    so_host = _cli(inp, str(tmp_path / "h.bam"), "0")
    assert so_gpu == so_host
    for suf in (".bam", "_filteredreads.bam", "_filteredfamilies.bam"):
        assert bam.bgzf_stream(str(tmp_path / ("g" + suf))) == bam.bgzf_stream(str(tmp_path / ("h" + suf)))


def test_ingest_gpu_inflate_corrupt_block(tmp_path):
    """A damaged member in the middle of the file stops the ingest with the
    host path's message."""
    from duplexumiconsensusreads_amd import cli, native_io
    inp = str(tmp_path / "in.bam")
    synth.write_packed_bam(inp, synth.packed_fixed_size(30_000, seed=9), seed=9, level=6)
    blob = bytearray(open(inp, "rb").read())
    from duplexumiconsensusreads_amd import _lib
    m, _ = _lib.bgzf_members(bytes(blob))
    x = m[len(m) // 2]
    blob[int(x["in_off"]) + 100] ^= 0xff
    open(inp, "wb").write(bytes(blob))
    os.environ["DCR_GPU_INFLATE"] = "1"
    try:
        cli.gpu_inflate(0)
    finally:
        os.environ.pop("DCR_GPU_INFLATE", None)
    ing = native_io.Ingest(inp)
    assert ing.gpu_inflate
    hb = native_io.HostBatch(reads=1 << 20)
    with pytest.raises(Exception, match="inflate|CRC"):
        while True:
            ing.next(hb)
            if hb.end_kind != native_io.END_FULL:
                if hb.end_kind == native_io.END_ERROR:
                    raise RuntimeError(hb.error()[1])
                break
    ing.close()


def _with_gpu_inflate(flag, fn):
    from duplexumiconsensusreads_amd import cli
    old = os.environ.get("DCR_GPU_INFLATE")
    os.environ["DCR_GPU_INFLATE"] = flag
    try:
        cli.gpu_inflate(0)
        return fn()
    finally:
        if old is None:
            os.environ.pop("DCR_GPU_INFLATE", None)
        else:
            os.environ["DCR_GPU_INFLATE"] = old
        cli.gpu_inflate(0)


def test_stream_small_bgzf_blocks_same_outputs_as_host_inflate(tmp_path):
    """Blocks of 0.5-4 KiB of data (any size is valid BGZF): one 64 MiB ingest
    chunk then covers more than the stream's four slots of spans, the case the
    per-span `fetched` mark fixes (csrc/dcr_span_stream.h).  CLI outputs and
    stdout equal the host pool's."""
    from duplexumiconsensusreads_amd import bam
    from .bgzf_util import reblock
    big = str(tmp_path / "big.bam")
    synth.write_packed_bam(big, synth.packed_fixed_size(8000, seed=13), seed=13, level=1)
    inp = str(tmp_path / "small.bam")
    assert reblock(big, inp, 512, 4096, seed=2) > 25_000
    so_gpu = _cli(inp, str(tmp_path / "g.bam"), "1")
    so_host = _cli(inp, str(tmp_path / "h.bam"), "0")
    assert so_gpu == so_host
    for suf in (".bam", "_filteredreads.bam", "_filteredfamilies.bam"):
        assert bam.bgzf_stream(str(tmp_path / ("g" + suf))) == bam.bgzf_stream(str(tmp_path / ("h" + suf)))


def test_stream_ranged_ingest_same_batches_as_host_inflate(tmp_path):
    """The sharded CLI's ranged ingests (dcr_split_points, start/end virtual
    offsets) through the device stream pack the same batches, family table and
    side records as through the host pool, part by part."""
    from duplexumiconsensusreads_amd import native_io
    from duplexumiconsensusreads_amd.params import ConsensusParams
    from .bgzf_util import ingest_digest
    inp = str(tmp_path / "in.bam")
    synth.write_packed_bam(inp, synth.packed_config(synth.CONFIGS["C5"], 40_000, seed=6), seed=6, level=6)
    pts = native_io.split_points(inp, 3, ConsensusParams())
    assert all(p > 0 for p in pts)
    bounds = list(zip([0] + pts, pts + [-1]))
    for lo, hi in bounds:
        g = _with_gpu_inflate("1", lambda: ingest_digest(inp, lo, hi))
        h = _with_gpu_inflate("0", lambda: ingest_digest(inp, lo, hi))
        assert g[3] and not h[3]
        assert g[:3] == h[:3], (lo, hi)
