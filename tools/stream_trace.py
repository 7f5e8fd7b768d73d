"""One CLI pass over a C5-shaped BAM (subfamilies Poisson(4)+1, 2x150bp) of
several streaming batches, for a rocprofv3 kernel + memory-copy trace
(tools/overlap.py computes the copy/compute overlap from it).
usage: python tools/stream_trace.py <workdir> [families] [batch_reads]"""
import contextlib
import io
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from duplexumiconsensusreads_amd import cli, synth  # noqa: E402


def main():
    wd = sys.argv[1]
    fams = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    batch = sys.argv[3] if len(sys.argv) > 3 else str(1 << 22)
    os.makedirs(wd, exist_ok=True)
    path = os.path.join(wd, "c5.bam")
    t = time.time()
    packed = synth.packed_config(synth.CONFIGS["C5"], fams, seed=5)
    synth.write_packed_bam(path, packed, seed=5, level=1)
    print(f"{packed.n_reads} reads, {os.path.getsize(path) / 1e6:.0f} MB BAM in {time.time() - t:.1f} s", flush=True)
    del packed
    out = os.path.join(wd, "cons.bam")
    for k in range(2):
        stats = {}
        t = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            cli.main(["-i", path, "-o", out, "--batch_reads", batch], stats=stats)
        dt = time.perf_counter() - t
        print(f"pass {k}: {dt:.3f} s, {stats['consensus_bases'] / dt / 1e6:.1f} M consensus bases/s, "
              f"{stats['batches']} batches; " + ", ".join(f"{a} {b:.3f}" for a, b in stats.items() if a.endswith("_s")),
              flush=True)


if __name__ == "__main__":
    main()
