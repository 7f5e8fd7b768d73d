#!/bin/bash
# round 4: fast-kernel A/B (base vs v8), C3 general-kernel A/B (base vs the
# event layout), the GPU suite, the 16/16 pool bench
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
T=${1:-r04b}
L=duplexumiconsensusreads_amd
mkdir -p gpurun_out/${T}_ab
ABL_CONFIG=C3 timeout -k 10 300 python3 -u tools/ablate.py 100000 $L/libdcr_base.so $L/libdcr_v8ev.so > gpurun_out/${T}_ab/ablate_C3.txt 2>&1; echo "C3 ablate rc=$?"; cat gpurun_out/${T}_ab/ablate_C3.txt
tools/gpu_fastab.sh "${T}_ab" $L/libdcr_base.so $L/libdcr_v8.so $L/libdcr_v8ev.so || exit 1
tools/gpu_r04a.sh "$T"
