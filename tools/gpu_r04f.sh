#!/bin/bash
# round 4: whole-node C2 bench with the runtime's copy engine choice A/B
# (default vs HSA_ENABLE_SDMA=1 / GPU_BLIT_ENGINE_TYPE), interleaved; one
# kernel trace each (the __amd_rocclr_copyBuffer blit kernels vs SDMA).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04f}
mkdir -p "$O"
env | grep -E "^(HSA|GPU_|HIP_|ROC|AMD_)" | sort > "$O/env.txt"
run() {   # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --no-cpu --kernel-steps 2 --steps 4 --warmup 1 > "$O/b_$tag.json" 2> "$O/b_$tag.log"
  local rc=$?
  echo "[r04f] $tag rc=$rc" >> "$O/b_$tag.log"
  [ $rc -ne 0 ] && { echo "bench $tag failed rc=$rc"; tail -30 "$O/b_$tag.log"; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$tag.json')); s=d['config']['stages_s_last_pass']; print('$tag', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  run def$rep DCR_NOTHING=1 || exit 1
  run sdma$rep HSA_ENABLE_SDMA=1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_def" -o kt -- python3 -u bench.py --no-cpu --kernel-steps 1 --steps 2 --warmup 1 > "$O/kt_def.log" 2>&1 || exit 1
HSA_ENABLE_SDMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_sdma" -o kt -- python3 -u bench.py --no-cpu --kernel-steps 1 --steps 2 --warmup 1 > "$O/kt_sdma.log" 2>&1 || exit 1
