"""Times the REFERENCE main() (DuplexUMIConsensusReads.py:1426-1650) on a
synthetic config-1 BAM in this container (the dev container: the reference is
not on the GPU box), for the CPU side of BASELINE's metric.

The reference runs as tests/golden/make_golden.py loads it: imported from
/root/reference with the pysam shim (tests/golden/pysam_shim.py: pure-Python
BAM I/O standing in for pysam, which this image lacks), so the time includes
the shim's record codec.  Prints one JSON line.

    python3 tools/time_reference_c1.py [n_families] [out.json]
"""
import contextlib
import io
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)

import make_golden  # noqa: E402
from duplexumiconsensusreads_amd import bam, synth  # noqa: E402


def main():
    n_fam = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    ref = make_golden.load_reference()
    inp, outp = "/tmp/time_ref_c1.bam", "/tmp/time_ref_c1_cons.bam"
    synth.write_config_bam(inp, synth.CONFIGS["C1"], n_families=n_fam, seed=21)
    argv = sys.argv
    sys.argv = ["DuplexUMIConsensusReads.py", "-i", inp, "-o", outp]
    random.seed(7)
    t0 = time.perf_counter()
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            ref.main()
    finally:
        sys.argv = argv
    dt = time.perf_counter() - t0
    n_reads, bases, n_cons = 0, 0, 0
    with bam.AlignmentFile(inp, "rb") as f:
        n_reads = sum(1 for _ in f)
    with bam.AlignmentFile(outp, "rb") as f:
        for r in f:
            n_cons += 1
            bases += len(r.query_sequence or "")
    line = {"what": "reference main() on a synthetic C1 BAM, this container, 1 core (pysam shim I/O)",
            "families": n_fam, "reads": n_reads, "consensus_records": n_cons, "consensus_bases": bases,
            "seconds": round(dt, 3), "ms_per_family": round(1e3 * dt / n_fam, 2),
            "consensus_bases_per_s": round(bases / dt, 1)}
    print(json.dumps(line))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
