"""Per-kernel PMC counters from a rocprofv3 database (pmc_results.db, the
default output format): counter totals per dispatch averaged over a kernel's
dispatches, and per record when the record count of a launch is given.

    python3 tools/pmc_db.py DIR_OR_DB [records-per-launch] [kernel-substring ...]
"""
import collections
import glob
import os
import sqlite3
import sys


def main():
    p = sys.argv[1]
    dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
    nrec = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    want = sys.argv[3:] or ["dcr"]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for db in dbs:
        c = sqlite3.connect(db)
        for name, did, ctr, val in c.execute("select name, dispatch_id, counter_name, counter_value from pmc_events"):
            if not any(w in name for w in want):
                continue
            k = name.split("(")[0]
            tot[k][ctr] += val
            disp[k].add(did)
    for k in sorted(tot):
        n = len(disp[k])
        print(f"== {k}  ({n} dispatches)")
        w = tot[k].get("SQ_WAVES", 0.0)
        for ctr in sorted(tot[k]):
            v = tot[k][ctr] / n
            extra = f"   per record {v / nrec:10.1f}" if nrec else ""
            print(f"   {ctr:24s} {v:16.6g} per launch{extra}")
        if w:
            print(f"   (waves per launch {w / n:.0f})")


if __name__ == "__main__":
    main()
