"""Per-pass breakdown of the whole-node pipeline from a rocprofv3
--kernel-trace --memory-copy-trace run of bench.py: the busy time of the
stream that runs the batch kernels (consensus + record writer), its kernels,
and the other streams' work (inflate, runtime copy kernels) over the same
span; plus which host<->device copies ran on a copy engine (memory-copy
trace) and which as __amd_rocclr_copyBuffer kernels on the CUs.
usage: python tools/pipe_trace.py DIR   (DIR holds *_kernel_trace.csv, *_memory_copy_trace.csv)"""
import collections
import csv
import glob
import os
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    kt = load(d, "*kernel_trace.csv")
    mc = load(d, "*memory_copy_trace.csv")
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], name(r)) for r in kt)
    # the batch stream: the one that runs k_deflate
    bs = collections.Counter(e[2] for e in ev if e[3].endswith("k_deflate")).most_common(1)[0][0]
    s5 = [e for e in ev if e[2] == bs]
    passes = [[s5[0]]]
    for e in s5[1:]:
        if e[0] - passes[-1][-1][1] > 30e6:       # a gap > 30 ms separates CLI passes
            passes.append([])
        passes[-1].append(e)
    print(f"batch stream {bs}")
    for p in passes:
        if not any(e[3].endswith("k_deflate") for e in p) or len(p) < 50:
            continue
        t0, t1 = p[0][0], max(e[1] for e in p)
        busy = sum(e[1] - e[0] for e in p)
        per = collections.Counter()
        for e in p:
            per[e[3]] += (e[1] - e[0]) / 1e6
        oth = collections.Counter()
        for e in ev:
            if e[2] != bs and e[0] >= t0 and e[1] <= t1:
                oth[f"stream {e[2]} {e[3]}"] += (e[1] - e[0]) / 1e6
        print(f"pass: span {(t1 - t0) / 1e6:.1f} ms, batch stream busy {busy / 1e6:.1f} ms "
              f"({100.0 * busy / (t1 - t0):.0f} %)")
        for k, v in per.most_common(10):
            print(f"    {k:45s} {v:8.1f} ms")
        for k, v in oth.most_common(5):
            print(f"    (other) {k:37s} {v:8.1f} ms")
    cb = collections.Counter(e[2] for e in ev if e[3].endswith("copyBuffer"))
    print("copy kernels (__amd_rocclr_copyBuffer) per stream:", dict(cb))
    print("copy-engine transfers per direction:", dict(collections.Counter(r["Direction"] for r in mc)))


if __name__ == "__main__":
    main()
