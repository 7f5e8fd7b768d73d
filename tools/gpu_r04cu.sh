#!/bin/bash
# round 4: the inflate span stream masked to k of every 4 CUs
# (DCR_INFLATE_CU_SHARE) against every CU, interleaved whole-node benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04cu}
mkdir -p "$O"
for rep in 1 2 3; do
  for k in 0 3 2; do
    DCR_INFLATE_CU_SHARE=$k timeout -k 10 300 python3 -u bench.py --no-cpu > "$O/b_${k}_$rep.json" 2> "$O/b_${k}_$rep.log" || { echo "bench $k failed"; tail -20 "$O/b_${k}_$rep.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${k}_$rep.json')); s=d['config']['stages_s_last_pass']; print('share $k rep $rep', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'))" | tee -a "$O/summary.txt"
  done
done
