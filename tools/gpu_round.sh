#!/bin/bash
# One GPU session: parity tests, the bench line, a kernel-trace profile of the
# same bench command, and the two PMC traffic passes.  Every GPU step has its
# own time limit; the chain stops at the first failure.
#   usage: tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
BENCH="bench.py --steps 10 --warmup 3 --no-cpu"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
fi
timeout -k 10 300 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 $BENCH > "$O/kt.log" 2>&1 || { echo "kernel trace failed"; tail -20 "$O/kt.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
head -8 "$O/kernel_stats.csv"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$O/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$O/pmc_write.log" 2>&1 || { echo "pmc write failed"; exit 1; }
python3 tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" 312500 "$O/traffic.json"
echo "gpu round done"
