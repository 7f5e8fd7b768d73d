#!/bin/bash
# PMC + kernel-trace passes over a short bench run (one rocprofv3 run per pass,
# counters per MI355X_MICROARCH.md slot limits).  Usage: tools/profile_pmc.sh OUTDIR [bench args]
set -o pipefail
OUT=$1; shift
ARGS=${*:-"--families 100000 --steps 2 --warmup 1 --no-cpu"}
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1 &&
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run p2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH &&
run p3 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE GRBM_COUNT &&
run p4 FETCH_SIZE &&
run p5 WRITE_SIZE
echo "profile done"
