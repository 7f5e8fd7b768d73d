#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02s
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
bash tools/gpu_traffic.sh r02s_traffic
