"""Per-launch-shape kernel durations from a rocprofv3 kernel trace.

rocprofv3 --stats averages every launch of a kernel together; bench.py
launches the single-strand kernel both on the full device-resident batch
(the roofline's launches) and on the CLI's smaller batches.  This groups the
trace by (kernel, grid size) so the roofline launch's average can be read
off beside bench.py's HIP-event time.

    python3 tools/kt_grid.py kernel_trace.csv [name-substring ...] > out.txt
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    want = sys.argv[2:]
    groups = defaultdict(list)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if want and not any(w in name for w in want):
                continue
            grid = row.get("Grid_Size_X") or row.get("Grid_Size") or "?"
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            groups[(name, int(grid))].append(dur)
    print("kernel,grid_x,calls,avg_us,min_us,max_us")
    for (name, grid), d in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        print(f"\"{name}\",{grid},{len(d)},{sum(d) / len(d) / 1e3:.2f},{min(d) / 1e3:.2f},{max(d) / 1e3:.2f}")


if __name__ == "__main__":
    main()
