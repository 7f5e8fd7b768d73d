#!/bin/bash
# Round-2 GPU session: parity tests, the whole-node bench line (C2), and a
# kernel-trace profile of the device-resident part.
#   usage: tools/gpu_r02.sh TAG [skip-tests] [bench args...]
set -o pipefail
TAG=${1:-r02}
SKIP=$2
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
if [ "$SKIP" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
fi
timeout -k 10 600 python3 -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
tail -5 "$O/bench.log"
