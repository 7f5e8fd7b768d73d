#!/bin/bash
# round 4: GPU suite after the inflate-stream fixes, then the 16/16 pool bench twice
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04a}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$O/pytest_gpu.log"
tail -3 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
tools/gpu_pool_ab.sh "${1:-r04a}_pool" "16/16"
