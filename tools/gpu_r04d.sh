#!/bin/bash
# round 4: the fast kernel's LDS (5 vs 4 blocks per CU) and its store /
# scalar / mean modes, interleaved in one process; PMC of base vs the fix.
# Each GPU step under its own limit; the first failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04d}
mkdir -p "$O"
step() { local name=$1; shift; "$@" > "$O/$name.txt" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -12 "$O/$name.txt"; return $rc; }
step ablate timeout -k 10 300 python3 -u tools/ablate.py 312500 $L/libdcr_base.so $L/libdcr_lf1.so $L/libdcr_lfpad.so $L/libdcr_lfs00.so $L/libdcr_lfm1.so $L/libdcr_lfm2.so || exit 1
ABL_CONFIG=C5 step ablate_C5 timeout -k 10 300 python3 -u tools/ablate.py 200000 $L/libdcr_xu2.so $L/libdcr_lf1.so $L/libdcr_base.so || exit 1
for v in base lf1; do
  step pmc_$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$O/pmc_$v" -o pmc -- python3 tools/ablate.py 312500 $PWD/$L/libdcr_$v.so || exit 1
done
