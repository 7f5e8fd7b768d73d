"""Host BGZF throughput: the Python codec (bam.BGZFReader/BGZFWriter) against
the native threaded one (csrc/dcr_bgzf.cpp) on a BAM-like stream built by
repeating the records of tests/golden/e2e_c1_small.bam.

    python tools/bench_bgzf.py [MiB] [threads]
"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from duplexumiconsensusreads_amd import bam  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    recs = b"".join(bam.encode_record(r) for r in bam.AlignmentFile(os.path.join(ROOT, "tests/golden/e2e_c1_small.bam")))
    data = (recs * (mib * (1 << 20) // len(recs) + 1))[:mib << 20]
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name, wcls, rcls in (("python", bam.BGZFWriter, bam.BGZFReader),
                                 ("native", lambda p: bam.NativeBGZFWriter(p, 6, nt),
                                  lambda p: bam.NativeBGZFReader(p, nt))):
            p = os.path.join(d, name + ".bam")
            t0 = time.perf_counter()
            w = wcls(p)
            for i in range(0, len(data), 1 << 20):
                w.write(data[i:i + (1 << 20)])
            w.close()
            t1 = time.perf_counter()
            r = rcls(p)
            n = 0
            while True:
                c = r.read(1 << 20)
                if not c:
                    break
                n += len(c)
            r.close()
            t2 = time.perf_counter()
            assert n == len(data)
            out[name] = (len(data) / (t1 - t0) / 1e6, len(data) / (t2 - t1) / 1e6, os.path.getsize(p))
    for k, (wr, rd, sz) in out.items():
        print(f"{k:7s} deflate {wr:8.1f} MB/s  inflate {rd:8.1f} MB/s  (uncompressed MB/s; file {sz / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
