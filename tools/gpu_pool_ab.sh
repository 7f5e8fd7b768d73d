#!/bin/bash
# Whole-node A/B of the ingest's scanner / pack pool sizes with the GPU
# inflate on (the host inflate pool idle): DCR_SCAN_THREADS / DCR_PACK_THREADS.
#   usage: tools/gpu_pool_ab.sh TAG "s1/p1 s2/p2 ..."
set -o pipefail
TAG=${1:-poolab}
CFGS=${2:-"8/8 12/12 16/16"}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for rep in 1 2; do
  for c in $CFGS; do
    sc=${c%/*}; pk=${c#*/}
    f="$O/b_${sc}_${pk}_$rep"
    DCR_SCAN_THREADS=$sc DCR_PACK_THREADS=$pk timeout -k 10 300 python3 -u bench.py --no-cpu --kernel-steps 2 --steps 4 --warmup 1 > "$f.json" 2> "$f.log"
    rc=$?
    # the exit status (124/137: the timeout; 134 abort; 139 SIGSEGV; 137 also
    # an OOM kill) and the kernel log's last lines go into the run's own log
    echo "[gpu_pool_ab] bench rc=$rc at $(date +%T)" >> "$f.log"
    if [ $rc -ne 0 ]; then
      { echo "[gpu_pool_ab] dmesg tail:"; dmesg 2>&1 | tail -20; } >> "$f.log"
      echo "bench failed rc=$rc"; tail -40 "$f.log"; exit 1
    fi
    python3 -c "import json; d=json.load(open('$f.json')); s=d['config']['stages_s_last_pass']; print('scan $sc pack $pk', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'))" | tee -a "$O/summary.txt"
  done
done
