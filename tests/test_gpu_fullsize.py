"""The product path at production size: ``cli.main`` with the device record
writer (dcr_submit_write: k_famfail -> k_fmt_* -> k_deflate -> k_compact) on
the whole 10 M-read C2 bench input at the CLI's default batch of 524,288
reads, against the same CLI driven by the C oracle (oracle/dcr_oracle.c, 16
threads) through the host record formatter (csrc/dcr_format.cpp) on the same
input.  The decompressed consensus stream, both side files and stdout must be
byte-identical.  This is the path the bench's whole-node ``value`` times
(reference: DuplexUMIConsensusReads.py:1352-1419 record fields,
:1593-1594 ``consensusbam.write``).

The second case is SURVEY.md §8d's C4 sub-run: the deep-panel shape at the
default ``--max_reads 100`` with ``random.seed(4)``, so every subfamily is
downsampled by CPython's ``random.sample`` (:157-188, :186) before the GPU
sees it; the GPU CLI and the oracle-backend CLI must write the same files and
leave the caller's generator in the same state."""
import contextlib
import functools
import io
import os
import random
import time

import numpy as np
import pytest

from duplexumiconsensusreads_amd import bam, cli, synth
from oracle import dcr_oracle_c

pytestmark = pytest.mark.gpu

SUFFIXES = (".bam", "_filteredreads.bam", "_filteredfamilies.bam")


def _run(inp, out, backend, rng, extra=()):
    buf = io.StringIO()
    stats = {}
    with contextlib.redirect_stdout(buf):
        rc = cli.main(["-i", inp, "-o", out, *extra], backend=backend, rng=rng, stats=stats)
    assert rc == 0
    return buf.getvalue(), stats


def _progress(capsys, msg):
    """A line on the real terminal while pytest captures output (the long
    cases would otherwise be silent for minutes)."""
    with capsys.disabled():
        print(msg, flush=True)


def _compare(out_gpu, out_cpu):
    for suf in SUFFIXES:
        a = bam.bgzf_stream(out_gpu[:-4] + suf)
        b = bam.bgzf_stream(out_cpu[:-4] + suf)
        if a != b:
            # a small message: pytest's own diff of two streams of hundreds
            # of MB would not finish
            n = min(len(a), len(b))
            ne = np.frombuffer(a, np.uint8, n) != np.frombuffer(b, np.uint8, n)
            k = int(ne.argmax()) if ne.any() else n
            pytest.fail(f"{suf}: lengths {len(a)} / {len(b)}, first difference at byte {k}: "
                        f"gpu {a[max(0, k - 16):k + 16].hex()} cpu {b[max(0, k - 16):k + 16].hex()}")


def test_cli_device_writer_full_c2_input(tmp_path):
    inp = str(tmp_path / "c2.bam")
    packed = synth.packed_fixed_size(312_500, seed=2)
    synth.write_packed_bam(inp, packed, seed=2, level=6)
    n_fam = packed.n_fam
    del packed
    from duplexumiconsensusreads_amd.params import ConsensusParams
    be = cli.default_backend(ConsensusParams())
    assert be.device_writer
    out_gpu = str(tmp_path / "gpu.bam")
    out_cpu = str(tmp_path / "cpu.bam")
    so_gpu, st_gpu = _run(inp, out_gpu, be, random.Random(4))       # default --batch_reads 524,288
    assert st_gpu["batches"] >= 19
    assert st_gpu["consensus_records"] == 2 * n_fam
    oracle = functools.partial(dcr_oracle_c.run, n_threads=min(16, os.cpu_count() or 1))
    so_cpu, st_cpu = _run(inp, out_cpu, oracle, random.Random(4))
    assert so_gpu == so_cpu
    assert st_gpu["consensus_bases"] == st_cpu["consensus_bases"]
    _compare(out_gpu, out_cpu)


def test_cli_c4_default_max_reads_downsampled(tmp_path):
    inp = str(tmp_path / "c4.bam")
    cfg = synth.CONFIGS["C4"]
    packed = synth.packed_config(cfg, 1_000, seed=4)                 # subfamilies of 100..1,000 reads
    assert int((packed.sub_off[1:] - packed.sub_off[:-1]).max()) > 100
    synth.write_packed_bam(inp, packed, seed=4, level=6)
    del packed
    from duplexumiconsensusreads_amd.params import ConsensusParams
    be = cli.default_backend(ConsensusParams())
    rng_gpu, rng_cpu = random.Random(4), random.Random(4)
    so_gpu, _ = _run(inp, str(tmp_path / "gpu.bam"), be, rng_gpu, ("--verbose",))
    so_cpu, _ = _run(inp, str(tmp_path / "cpu.bam"),
                     functools.partial(dcr_oracle_c.run, n_threads=min(16, os.cpu_count() or 1)), rng_cpu,
                     ("--verbose",))
    assert "randomly downsampled to 100 reads" in so_gpu
    assert so_gpu == so_cpu
    assert rng_gpu.getstate() == rng_cpu.getstate()
    _compare(str(tmp_path / "gpu.bam"), str(tmp_path / "cpu.bam"))


def test_cli_device_writer_c3_shard(tmp_path, capsys):
    """One GPU's share of C3 (100 M reads over 8 GPUs: 400 k families, ~12.3 M
    reads) with its insertion layouts, deletions, soft clips and Zipf(1.5)
    subfamily sizes 1..100, at BGZF level 6 and the CLI's default batch: the
    general and exact kernels, the device writer and the device inflate all
    on the product path, byte-compared with the oracle-backend CLI
    (reference :473-545 insertion columns, :191-265 clips, :1519-1631)."""
    t0 = time.perf_counter()
    inp = str(tmp_path / "c3.bam")
    packed = synth.packed_config(synth.CONFIGS["C3"], 400_000, seed=3)
    synth.write_packed_bam(inp, packed, seed=3, level=6)
    n_fam = packed.n_fam
    del packed
    _progress(capsys, f"c3 shard: input written in {time.perf_counter() - t0:.1f} s")
    from duplexumiconsensusreads_amd.params import ConsensusParams
    be = cli.default_backend(ConsensusParams())
    assert be.device_writer
    out_gpu = str(tmp_path / "gpu.bam")
    out_cpu = str(tmp_path / "cpu.bam")
    t0 = time.perf_counter()
    so_gpu, st_gpu = _run(inp, out_gpu, be, random.Random(4))
    _progress(capsys, f"c3 shard: GPU CLI {time.perf_counter() - t0:.1f} s, {st_gpu['batches']} batches")
    assert st_gpu["batches"] >= 20
    assert st_gpu["consensus_records"] == 2 * n_fam
    oracle = functools.partial(dcr_oracle_c.run, n_threads=min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    so_cpu, st_cpu = _run(inp, out_cpu, oracle, random.Random(4))
    _progress(capsys, f"c3 shard: oracle CLI {time.perf_counter() - t0:.1f} s")
    assert so_gpu == so_cpu
    assert st_gpu["consensus_bases"] == st_cpu["consensus_bases"]
    _compare(out_gpu, out_cpu)
