#!/bin/bash
# round 4: k_inflate ring / root-table sizes around the new default (4 KiB,
# 9 bits); the exact pass at five blocks per CU (no LDS tables); the general
# kernel with and without the event layout; the GPU inflate tests on the new
# default; whole-node C2 bench with the runtime's default copy engine and
# with HSA_ENABLE_SDMA=1.  Each GPU step under its own limit; the first
# failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04g}
mkdir -p "$O"
env | grep -E "^(HSA|GPU_|HIP_|ROC|AMD_)" | sort > "$O/env.txt"
step() { local name=$1; shift; "$@" > "$O/$name.txt" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 "$O/$name.txt" | cut -c1-400; return $rc; }
for v in libdcr libdcr_r2k9 libdcr_r2k8 libdcr_r4k8 libdcr_r8k10; do
  DCR_LIB_PATH=$PWD/$L/$v.so step infl_$v timeout -k 10 240 python3 -u tools/inflate_speed.py 100000 1 || exit 1
done
step pytest_inflate timeout -k 10 300 python3 -u -m pytest tests/test_gpu_inflate.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
ABL_CONFIG=C5 step ablate_C5 timeout -k 10 300 python3 -u tools/ablate.py 200000 $L/libdcr.so $L/libdcr_x5.so || exit 1
ABL_CONFIG=C3 step ablate_C3 timeout -k 10 300 python3 -u tools/ablate.py 100000 $L/libdcr.so $L/libdcr_noev.so $L/libdcr_base.so || exit 1
run() {   # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --no-cpu --kernel-steps 2 --steps 4 --warmup 1 > "$O/b_$tag.json" 2> "$O/b_$tag.log"
  local rc=$?
  echo "[r04g] $tag rc=$rc" >> "$O/b_$tag.log"
  [ $rc -ne 0 ] && { echo "bench $tag failed rc=$rc"; tail -30 "$O/b_$tag.log"; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$tag.json')); s=d['config']['stages_s_last_pass']; print('$tag', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'infl', s.get('gpu_inflate'))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  run def$rep DCR_AB=def || exit 1
  run sdma$rep HSA_ENABLE_SDMA=1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_def" -o kt -- python3 -u bench.py --no-cpu --kernel-steps 1 --steps 2 --warmup 1 > "$O/kt_def.log" 2>&1 || exit 1
