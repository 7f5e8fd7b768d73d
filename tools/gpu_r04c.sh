#!/bin/bash
# round 4: attribution of the fast-kernel changes (store / scalar / mean
# modes), the event layout on C3, exact-queue counts on C5, parity tests of
# the current libdcr.so.  Each GPU step under its own limit; the first failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04c}
mkdir -p "$O"
step() { local name=$1; shift; "$@" > "$O/$name.txt" 2>&1; local rc=$?; echo "$name rc=$rc"; cat "$O/$name.txt" | tail -12; return $rc; }
step ablate timeout -k 10 300 python3 -u tools/ablate.py 312500 $L/libdcr_base.so $L/libdcr_s00.so $L/libdcr_s10.so $L/libdcr_m0.so $L/libdcr_m1.so $L/libdcr_m2.so || exit 1
ABL_CONFIG=C3 step ablate_C3 timeout -k 10 300 python3 -u tools/ablate.py 100000 $L/libdcr_base.so $L/libdcr_s00.so $L/libdcr_ev2.so || exit 1
ABL_CONFIG=C5 step ablate_C5 timeout -k 10 300 python3 -u tools/ablate.py 200000 $L/libdcr.so $L/libdcr_base.so || exit 1
for v in libdcr libdcr_r4k libdcr_r4k9 libdcr_lb9; do
  DCR_LIB_PATH=$PWD/$L/$v.so step infl_$v timeout -k 10 240 python3 -u tools/inflate_speed.py 100000 1 || exit 1
done
step pytest timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
