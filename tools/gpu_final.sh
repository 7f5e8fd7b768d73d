#!/bin/bash
# round end: the GPU suite, smoke() and the default bench line on the tree as committed
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-final}
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread 2>&1 | tee "$O/pytest_gpu.log" | grep -E "FAILED|ERROR|passed|failed|c3 shard" || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tee "$O/smoke.log" | tail -2 || exit 1
timeout -k 10 500 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
