#!/bin/bash
# Bench line (default C2, as the driver runs it), a kernel-trace profile of
# the same command, and one bench line per other config shape.
#   usage: tools/gpu_r02t.sh TAG
set -o pipefail
TAG=${1:-r02t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 500 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$O/bench_prof.json" 2> "$O/bench_prof.log" || { echo "prof failed"; tail -30 "$O/bench_prof.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
cut -d, -f1-8 "$O/kernel_stats.csv" | head -24
find "$O/kt" -name "*kernel_trace.csv" -exec python3 tools/kt_grid.py {} k_consensus_fast k_scatter \; > "$O/kernel_grid.csv"
cat "$O/kernel_grid.csv"
rm -rf "$O/kt"
for c in C3 C4 C5; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > "$O/bench_$c.json" 2> "$O/bench_$c.log" || { echo "bench $c failed"; tail -20 "$O/bench_$c.log"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('$c', '%.3g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['config']['device_resident']['kernel_ms'].items()}, 'frac %.3f'%d['roofline']['frac'])"
done
