"""Host ingest throughput of the native BAM reader (libdcr_io.so) over the
C2 bench BAM at several thread counts, with per-stage times
(DCR_INGEST_PROF=1): run on the GPU box's host cores.

    python3 tools/ingest_profile.py BAM [gpu] [threads ...]

``gpu``: the device inflate hook set first (cli.gpu_inflate), as the CLI
runs it; the ingest alone, no consensus or writer."""
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCR_INGEST_PROF", "1")
from duplexumiconsensusreads_amd import native_io, synth  # noqa: E402


def main():
    path = sys.argv[1]
    if not os.path.exists(path):
        t = time.time()
        synth.write_packed_bam(path, synth.packed_fixed_size(312_500, seed=2), seed=2, level=1)
        print(f"wrote {os.path.getsize(path) / 1e6:.0f} MB in {time.time() - t:.1f} s", flush=True)
    rest = sys.argv[2:]
    if rest and rest[0] == "gpu":
        from duplexumiconsensusreads_amd import cli
        cli.gpu_inflate(0)
        rest = rest[1:]
    for th in [int(a) for a in rest] or [16]:
        hbs = [native_io.HostBatch(reads=1 << 19) for _ in range(2)]
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        ing = native_io.Ingest(path, n_threads=th)
        k = 0
        while True:
            hb = hbs[k % 2]
            k += 1
            ing.next(hb)
            if hb.end_kind != native_io.END_FULL:
                break
        ing.close()
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        t1 = time.perf_counter()
        print(f"threads {th}: wall {t1 - t0:.3f} s, user {r1.ru_utime - r0.ru_utime:.2f} s, "
              f"sys {r1.ru_stime - r0.ru_stime:.2f} s", flush=True)


if __name__ == "__main__":
    main()
