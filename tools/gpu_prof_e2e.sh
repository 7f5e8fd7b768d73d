#!/bin/bash
# kernel trace of one whole-node bench pass (device writer included)
set -o pipefail
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_writer.py -x -q --timeout 240 --timeout-method thread > "$O/pytest_writer.log" 2>&1 || { echo "writer tests failed"; tail -30 "$O/pytest_writer.log"; exit 1; }
tail -2 "$O/pytest_writer.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 0 --kernel-steps 3 --no-cpu > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
cat "$O/kernel_stats.csv" | cut -d, -f1-8 | head -20
tail -3 "$O/bench.log"
