#!/bin/bash
# round 4: run-to-run spread of the whole-node bench on one box (five
# default runs back to back).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04x}
mkdir -p "$O"
for rep in 1 2 3 4 5; do
  timeout -k 10 300 python3 -u bench.py --no-cpu > "$O/b_$rep.json" 2> "$O/b_$rep.log" || { echo "bench $rep failed"; tail -20 "$O/b_$rep.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$rep.json')); s=d['config']['stages_s_last_pass']; print('$rep', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'), 'fast', round(d['roofline']['kernel_ms'],3))" | tee -a "$O/summary.txt"
done
