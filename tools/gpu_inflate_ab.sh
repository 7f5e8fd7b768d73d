#!/bin/bash
# Whole-node A/B of the input inflate: device inflater (cli.gpu_inflate) vs
# the host pool (DCR_GPU_INFLATE=0), input BGZF levels 1 and 6, interleaved;
# then a kernel trace of the GPU-inflate bench (k_inflate launches).
#   usage: tools/gpu_inflate_ab.sh TAG [levels]
set -o pipefail
TAG=${1:-infab}
LEVELS=${2:-"1 6"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for lvl in $LEVELS; do
  for g in 1 0 1 0; do
    f="$O/b_l${lvl}_g${g}"
    DCR_GPU_INFLATE=$g timeout -k 10 300 python3 -u bench.py --no-cpu --kernel-steps 2 --steps 4 --warmup 1 --in-level "$lvl" > "$f.json" 2> "$f.log" || { echo "bench failed"; tail -20 "$f.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$f.json')); c=d['config']; s=c['stages_s_last_pass']; print('level $lvl gpu_inflate=$g', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), s.get('gpu_inflate'))" | tee -a "$O/summary.txt"
  done
done
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 60 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -20 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
DCR_GPU_INFLATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --no-cpu --kernel-steps 2 --steps 2 --warmup 1 > "$O/prof.json" 2> "$O/prof.log" || { echo "prof failed"; tail -20 "$O/prof.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/kt" -name "*kernel_trace.csv" -exec python3 tools/kt_grid.py {} k_inflate k_deflate k_consensus_fast \; > "$O/kernel_grid.csv"
rm -rf "$O/kt"
head -8 "$O/kernel_stats.csv" | cut -c1-150
cat "$O/kernel_grid.csv" | head -12
