#!/bin/bash
# Whole-node (CLI from BAM open to output close) lines for the other
# BASELINE shapes: C3, C4 (--max_reads 1000 and the default 100, which
# downsamples with random.seed(4)), C5 streamed (2 M families, ~10 M reads
# through pinned batches), and C2 from a level-6 input.
#   usage: tools/gpu_e2e_configs.sh TAG [runs...]
set -o pipefail
TAG=${1:-e2e}
shift
RUNS=${*:-"C3 C4 C4_100 C5 C2_L6"}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $RUNS; do
  case $r in
    C3) A="--config C3" ;;
    C4) A="--config C4" ;;
    C4_100) A="--config C4 --max-reads 100" ;;
    C5) A="--config C5 --families 1000000" ;;
    C2_L6) A="--config C2 --in-level 6" ;;
    *) echo "unknown run $r"; exit 1 ;;
  esac
  timeout -k 10 600 python3 -u bench.py $A --no-cpu --kernel-steps 3 --steps 3 --warmup 1 > "$O/bench_$r.json" 2> "$O/bench_$r.log" || { echo "bench $r failed"; tail -20 "$O/bench_$r.log"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$r.json')); c=d['config']; s=c['stages_s_last_pass']
print('$r', round(d['value']/1e6,2), 'M consensus bases/s whole node;', 'input', round((c['input_bases_per_s'] or 0)/1e9,2), 'G bases/s;', 'reads', c['input_reads_per_gpu'], 'passes', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'device step ms', round(c['device_resident']['ms_per_step'],3))" | tee -a "$O/summary.txt"
done
