"""Summarise rocprofv3 PMC csv passes per kernel: totals and per-wave values."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{out}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, d in agg.items():
    if "dcr" not in k and "dinf" not in k:
        continue
    w = d.get("SQ_WAVES", 0) or 1
    print(f"== {k}  (dispatches {len(disp[(k, 'SQ_WAVES')])}, waves {w:.0f})")
    for c in sorted(d):
        print(f"   {c:28s} {d[c]:14.4g}   per-wave {d[c] / w:10.1f}")
