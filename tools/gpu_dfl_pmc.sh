#!/bin/bash
# PMC passes over tools/deflate_probe.py (k_deflate alone): instruction mix,
# LDS waits and bank conflicts.   usage: tools/gpu_dfl_pmc.sh TAG
set -o pipefail
TAG=${1:-dflpmc}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/p1 -o p --output-format csv -- python3 tools/deflate_probe.py > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d $O/p2 -o p --output-format csv -- python3 tools/deflate_probe.py > $O/pmc2.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt
grep -A20 "k_deflate" $O/pmc_summary.txt
rm -rf $O/p1 $O/p2
