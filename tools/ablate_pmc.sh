#!/bin/bash
# Per-phase instruction counts: each ablation build of libdcr under one PMC pass.
set -o pipefail
OUT=$1
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"; mkdir -p "$OUT"
for v in libdcr libdcr_abl1 libdcr_abl2 libdcr_abl3; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$OUT/$v" -o p --output-format csv -- python3 tools/ablate.py 100000 duplexumiconsensusreads_amd/$v.so > "$OUT/$v.log" 2>&1 || exit 1
done
echo done
