#!/bin/bash
# round 4: the runtime's copies as blit kernels (default) vs the SDMA engines
# (GPU_FORCE_BLIT_COPY_SIZE=0), interleaved whole-node benches, a kernel
# trace of each (copy kernels counted), and the ingest alone with the
# slimmer parsed records.  Each GPU step under its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04w}
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/ingest_profile.py /tmp/c2_ingest.bam gpu 16 2>&1 | tee "$O/ingest.txt" || exit 1
run() {   # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --no-cpu > "$O/b_$tag.json" 2> "$O/b_$tag.log" || { echo "bench $tag failed"; tail -20 "$O/b_$tag.log"; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$tag.json')); s=d['config']['stages_s_last_pass']; print('$tag', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  run def$rep DCR_AB=def || exit 1
  run sdma$rep GPU_FORCE_BLIT_COPY_SIZE=0 || exit 1
done
GPU_FORCE_BLIT_COPY_SIZE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_sdma" -o kt --output-format csv -- python3 -u bench.py --no-cpu --kernel-steps 1 --steps 2 --warmup 1 > "$O/kt_sdma.log" 2>&1 || exit 1
find "$O/kt_sdma" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_sdma.csv" \;
rm -rf "$O/kt_sdma"
head -6 "$O/kernel_stats_sdma.csv" | cut -c1-160
