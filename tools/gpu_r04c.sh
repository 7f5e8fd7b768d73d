#!/bin/bash
# round 4: attribution of the fast-kernel changes (store / scalar / mean
# modes), the event layout on C3, parity tests of the current libdcr.so
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04c}
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/ablate.py 312500 $L/libdcr_base.so $L/libdcr_s00.so $L/libdcr_s10.so $L/libdcr_m0.so $L/libdcr_m1.so $L/libdcr_m2.so > "$O/ablate.txt" 2>&1; echo "rc=$?"
cat "$O/ablate.txt"
ABL_CONFIG=C3 timeout -k 10 300 python3 -u tools/ablate.py 100000 $L/libdcr_base.so $L/libdcr_s00.so $L/libdcr_ev2.so > "$O/ablate_C3.txt" 2>&1; echo "rc=$?"
cat "$O/ablate_C3.txt"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; echo "pytest rc=$?"
tail -3 "$O/pytest.log"
