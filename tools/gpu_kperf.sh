#!/bin/bash
# Device-resident C2 kernel times (bench --kernel-only) and a kernel-trace
# profile of the same command split by launch shape.
#   usage: tools/gpu_kperf.sh TAG [env assignments for an A/B run, e.g. DCR_NO_PAIR=1]
set -o pipefail
TAG=${1:-kperf}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 python3 -u bench.py --kernel-only --no-cpu --kernel-steps 20 > "$O/bench_k.json" 2> "$O/bench_k.log" || { echo "bench failed"; tail -20 "$O/bench_k.log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k.json')); k=d['config']['device_resident']['kernel_ms']; print({a: round(b,4) for a,b in k.items()}, 'step', round(d['config']['device_resident']['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --kernel-only --no-cpu --kernel-steps 5 --steps 1 --warmup 0 > "$O/kt.log" 2>&1 || { echo "trace failed"; tail -20 "$O/kt.log"; exit 1; }
find "$O/kt" -name "*kernel_trace.csv" -exec python3 tools/kt_grid.py {} k_consensus k_recmeta k_scatter \; > "$O/kernel_grid.csv"
rm -rf "$O/kt"
cat "$O/kernel_grid.csv"
