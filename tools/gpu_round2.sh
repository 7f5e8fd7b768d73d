#!/bin/bash
# Round evidence: GPU parity tests, the bench line (driver's default
# command), a kernel-trace profile of that command with per-launch-shape
# durations, the PMC traffic passes, and one device-resident line per other
# config shape.  Every GPU step has its own time limit; the chain stops at
# the first failure.
#   usage: tools/gpu_round2.sh TAG
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 500 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$O/bench_prof.json" 2> "$O/bench_prof.log" || { echo "prof failed"; tail -30 "$O/bench_prof.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/kt" -name "*kernel_trace.csv" -exec python3 tools/kt_grid.py {} k_consensus_fast k_recmeta k_deflate k_inflate \; > "$O/kernel_grid.csv"
rm -rf "$O/kt"
head -12 "$O/kernel_grid.csv"
bash tools/gpu_traffic.sh "$TAG" || exit 1
for c in C3 C4 C5; do
  timeout -k 10 300 python3 -u bench.py --config $c --kernel-only --steps 5 --warmup 2 --no-cpu > "$O/bench_$c.json" 2> "$O/bench_$c.log" || { echo "bench $c failed"; tail -20 "$O/bench_$c.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); c=d['config']; k=c.get('device_resident', c); print('$c', 'ms/step %.3f' % k['ms_per_step'], {a: round(b, 3) for a, b in k['kernel_ms'].items()})"
done
echo "round evidence done"
