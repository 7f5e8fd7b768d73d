"""Copy/compute overlap from a rocprofv3 --kernel-trace --memory-copy-trace
run: the share of H2D / D2H copy time during which a kernel was running,
and the GPU's busy time (union of kernels and copies).
usage: python tools/overlap.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>"""
import csv
import glob
import os
import sys


def intervals(path, kind_col=None):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            s = int(row.get("Start_Timestamp") or row.get("start_timestamp") or 0)
            e = int(row.get("End_Timestamp") or row.get("end_timestamp") or 0)
            if e > s:
                out.append((s, e, row.get(kind_col, "") if kind_col else row.get("Kernel_Name", "")))
    return out


def union(iv):
    iv = sorted((s, e) for s, e, *_ in iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], e))
        else:
            out.append((s, e))
    return out


def overlap_len(a, u):
    """length of interval a covered by the sorted disjoint intervals u"""
    s, e = a
    tot = 0
    for us, ue in u:
        if ue <= s:
            continue
        if us >= e:
            break
        tot += min(e, ue) - max(s, us)
    return tot


def main():
    d = sys.argv[1]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    allk = intervals(kt[0])
    # runtime blit kernels (hipMemcpy* into / out of pinned host memory that the
    # runtime runs as copy kernels) count as copies, not as compute
    kern = [k for k in allk if not k[2].startswith("__amd_rocclr_copy")]
    blits = [(s, e, "BLIT (__amd_rocclr_copyBuffer kernels)") for s, e, n in allk
             if n.startswith("__amd_rocclr_copy")]
    copies = (intervals(mt[0], "Direction") if mt else []) + blits
    ku = union(kern)
    busy_k = sum(e - s for s, e in ku)
    res = {}
    for direction in sorted({c[2] for c in copies}):
        cs = [c for c in copies if c[2] == direction]
        tot = sum(e - s for s, e, _ in cs)
        hid = sum(overlap_len((s, e), ku) for s, e, _ in cs)
        res[direction] = (len(cs), tot, hid)
    allu = union(kern + copies)
    span = allu[-1][1] - allu[0][0] if allu else 0
    print(f"kernels: {len(kern)}, busy {busy_k / 1e6:.2f} ms; GPU busy (kernels or copies) "
          f"{sum(e - s for s, e in allu) / 1e6:.2f} ms over a {span / 1e6:.2f} ms span")
    for k, (n, tot, hid) in res.items():
        print(f"{k}: {n} copies, {tot / 1e6:.2f} ms, {hid / 1e6:.2f} ms of it under a running kernel "
              f"({100.0 * hid / max(tot, 1):.1f} % overlapped)")


if __name__ == "__main__":
    main()
