#!/bin/bash
# Quick GPU iteration: parity tests then one bench line (each step time-limited).
set -o pipefail
TAG=${1:-quick}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert" "$O/pytest_gpu.log" | tail -25
[ $rc -ne 0 ] && { tail -40 "$O/pytest_gpu.log"; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
