#!/bin/bash
# round 4: the exact pass with every tile's products at once and the quality
# table in LDS, against the previous build (C5, C3, C2), and the parity suite
# on it.  Each GPU step under its own limit; the first failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04s}
mkdir -p "$O"
step() { local name=$1; shift; "$@" > "$O/$name.txt" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 "$O/$name.txt" | cut -c1-300; return $rc; }
ABL_CONFIG=C5 step ablate_C5 timeout -k 10 300 python3 -u tools/ablate.py 200000 $L/libdcr_prev.so $L/libdcr.so || exit 1
ABL_CONFIG=C3 step ablate_C3 timeout -k 10 300 python3 -u tools/ablate.py 100000 $L/libdcr_prev.so $L/libdcr.so || exit 1
step ablate timeout -k 10 300 python3 -u tools/ablate.py 312500 $L/libdcr_prev.so $L/libdcr.so || exit 1
step pytest timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_cli_cases.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
