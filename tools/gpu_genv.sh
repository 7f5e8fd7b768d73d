#!/bin/bash
# one diagnostic general-kernel build on the first golden GPU test, bounded
set -o pipefail
V=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/genv
DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_genv$V.so timeout -k 10 75 python3 -u -m pytest -x -v -m gpu "tests/test_gpu_parity.py::test_gpu_matches_reference_goldens" > gpurun_out/genv/v$V.log 2>&1
rc=$?
echo "variant $V rc=$rc"
tail -5 gpurun_out/genv/v$V.log
exit $rc
