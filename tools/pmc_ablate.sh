#!/bin/bash
# Instruction counts of the fast kernel per ablation build (tools/build_ablate.sh):
# one rocprofv3 --pmc pass per library over tools/ablate.py.
set -o pipefail
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
mkdir -p "$OUT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD \
    -d "$OUT/$name/p1" -o "$name" --output-format csv -- python3 tools/ablate.py 312500 "$lib" > "$OUT/$name.log" 2>&1 || exit 1
  python3 tools/pmc_summary.py "$OUT/$name" | grep -A9 "k_consensus_fast<false>" > "$OUT/$name.txt"; echo "## $name"; cat "$OUT/$name.txt"
done
