#!/bin/bash
# A/B of libdcr builds on the C2 batch: kernel times interleaved in one
# process (tools/ablate.py), then one PMC pass per build (instruction counts
# of the fast kernel), then the fast-kernel parity tests on the last build
# (installed as libdcr.so by the caller).
#   usage: tools/gpu_fastab.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/ablate.py 312500 "$@" > "$O/ablate.txt" 2>&1 || { tail -20 "$O/ablate.txt"; exit 1; }
cat "$O/ablate.txt"
for b in "$@"; do
  n=$(basename "$b" .so)
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$O/$n/p1" -o p --output-format csv -- python3 tools/ablate.py 312500 "$b" > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
  python3 tools/pmc_summary.py "$O/$n" > "$O/pmc_$n.txt"
  echo "== $n"; grep -A9 "k_consensus_fast<false, false>" "$O/pmc_$n.txt"
  rm -rf "$O/$n/p1"
done
