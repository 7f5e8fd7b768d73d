#!/bin/bash
# Instruction counts of the fast kernel's phases: one PMC pass (SQ_INSTS_*)
# per build (product, staging only = DCR_ABL 1, + evidence = DCR_ABL 2) over
# the C2 batch; differences attribute VALU / SALU / LDS to the phases.
#   usage: tools/gpu_abl_pmc.sh TAG
set -o pipefail
TAG=${1:-ablpmc}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
L=duplexumiconsensusreads_amd
for b in libdcr libdcr_abl1 libdcr_abl2; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$O/$b/p1" -o p --output-format csv -- python3 tools/ablate.py 312500 $L/$b.so > "$O/$b.log" 2>&1 || { tail -5 "$O/$b.log"; exit 1; }
  python3 tools/pmc_summary.py "$O/$b" > "$O/pmc_$b.txt"
  echo "== $b"; grep -A9 "k_consensus_fast<false, false>" "$O/pmc_$b.txt"
  rm -rf "$O/$b/p1"
done
