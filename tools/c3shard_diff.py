"""Diagnostic: the C3-shard CLI case of tests/test_gpu_fullsize.py, GPU CLI
vs oracle-backend CLI, reporting where the outputs first differ (record
index, the two records decoded) instead of pytest's byte diff.

    python3 tools/c3shard_diff.py [families] [level] [batch_reads]
"""
import contextlib
import functools
import io
import os
import random
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from duplexumiconsensusreads_amd import bam, cli, synth  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams  # noqa: E402
from oracle import dcr_oracle_c  # noqa: E402


def run(inp, out, backend, extra):
    buf, st = io.StringIO(), {}
    with contextlib.redirect_stdout(buf):
        cli.main(["-i", inp, "-o", out, *extra], backend=backend, rng=random.Random(4), stats=st)
    return buf.getvalue(), st


def records(path):
    with bam.AlignmentFile(path, "rb") as f:
        for r in f:
            yield r.to_dict()


def main():
    fams = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    level = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    extra = ["--batch_reads", sys.argv[3]] if len(sys.argv) > 3 else []
    d = tempfile.mkdtemp()
    inp = os.path.join(d, "c3.bam")
    t0 = time.perf_counter()
    synth.write_packed_bam(inp, synth.packed_config(synth.CONFIGS["C3"], fams, seed=3), seed=3, level=level)
    print(f"input {time.perf_counter() - t0:.1f} s", flush=True)
    be = cli.default_backend(ConsensusParams())
    so_g, st_g = run(inp, os.path.join(d, "gpu.bam"), be, extra)
    print("gpu", {k: st_g.get(k) for k in ("batches", "consensus_records", "consensus_bases")}, flush=True)
    oracle = functools.partial(dcr_oracle_c.run, n_threads=min(16, os.cpu_count() or 1))
    so_c, st_c = run(inp, os.path.join(d, "cpu.bam"), oracle, extra)
    print("cpu", {k: st_c.get(k) for k in ("batches", "consensus_records", "consensus_bases")}, flush=True)
    print("stdout equal", so_g == so_c, flush=True)
    bad = 0
    for suf in (".bam", "_filteredreads.bam", "_filteredfamilies.bam"):
        a = bam.bgzf_stream(os.path.join(d, "gpu" + suf))
        b = bam.bgzf_stream(os.path.join(d, "cpu" + suf))
        same = a == b
        print(suf, len(a), len(b), "equal" if same else "DIFFER", flush=True)
        if same:
            continue
        bad += 1
        n = min(len(a), len(b))
        ne = np.frombuffer(a, np.uint8, n) != np.frombuffer(b, np.uint8, n)
        k = int(ne.argmax()) if ne.any() else n
        print("  first differing byte", k, flush=True)
        # the record holding byte k: walk the block_size chain (after the header)
        import struct
        hl = 12 + struct.unpack_from("<i", a, 4)[0]
        nref = struct.unpack_from("<i", a, hl - 4)[0]
        p = hl
        for _ in range(nref):
            p += 8 + struct.unpack_from("<i", a, p)[0]
        idx = 0
        while p + 4 <= k:
            q = p + 4 + struct.unpack_from("<i", a, p)[0]
            if q > k:
                break
            p, idx = q, idx + 1
        print(f"  in record {idx} at byte {p} (offset {k - p} into it)", flush=True)
        n = 0
        for ra, rb in zip(records(os.path.join(d, "gpu" + suf)), records(os.path.join(d, "cpu" + suf))):
            if n < idx:
                n += 1
                continue
            if ra != rb:
                print("  record", n, flush=True)
                for key in sorted(set(ra) | set(rb)):
                    if ra.get(key) == rb.get(key):
                        continue
                    if key == "tags":
                        for ta, tb in zip(ra[key], rb[key]):
                            if ta == tb:
                                continue
                            print(f"    tag {ta[0]} / {tb[0]} type {ta[1]} / {tb[1]}", flush=True)
                            va, vb = ta[2], tb[2]
                            if isinstance(va, str) and va.startswith("["):
                                va, vb = eval(va), eval(vb)   # noqa: S307 - our own list tags
                            if isinstance(va, (list, str)) and isinstance(vb, (list, str)):
                                ks = [i for i in range(min(len(va), len(vb))) if va[i] != vb[i]]
                                print(f"      lengths {len(va)} / {len(vb)}, {len(ks)} differ, first at {ks[:10]}",
                                      flush=True)
                                for i in ks[:5]:
                                    print(f"      [{i}] gpu {va[max(0, i - 3):i + 4]} cpu {vb[max(0, i - 3):i + 4]}",
                                          flush=True)
                            else:
                                print(f"      gpu {str(va)[:200]} cpu {str(vb)[:200]}", flush=True)
                    else:
                        print(f"    {key}: gpu={str(ra.get(key))[:300]}", flush=True)
                        print(f"    {key}: cpu={str(rb.get(key))[:300]}", flush=True)
                print(f"    gpu record: pos {ra.get('reference_start', ra.get('pos'))} "
                      f"seq {str(ra.get('query_sequence', ra.get('seq')))[:200]}", flush=True)
                print(f"    cpu record: pos {rb.get('reference_start', rb.get('pos'))} "
                      f"seq {str(rb.get('query_sequence', rb.get('seq')))[:200]}", flush=True)
                break
            n += 1
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
