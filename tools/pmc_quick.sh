#!/bin/bash
# Per-wave PMC counters of the consensus kernels over a short bench run
# (one rocprofv3 run per pass, within the gfx950 slot limits).
set -o pipefail
OUT=$1; shift
ARGS=${*:-"--families 100000 --steps 1 --warmup 1 --no-cpu"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run p2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH &&
run p3 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT &&
python3 tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.txt" && cat "$OUT/pmc_summary.txt"
