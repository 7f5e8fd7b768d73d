#!/bin/bash
# Whole-node A/B of libdcr builds: bench.py (no CPU leg) with DCR_LIB set to
# each build in turn, interleaved, REPS rounds; the value and the last pass's
# stages per run into gpurun_out/TAG/ab.txt.
#   usage: [AB_VAR=DCR_IO_LIB] tools/ab_bench.sh TAG REPS STEPS lib1.so lib2.so ...
# (AB_VAR: the variable the library path goes into, DCR_LIB by default)
# An argument NAME=VALUE instead of a library runs the default build with
# that variable set (NAME=default: nothing set), e.g. runtime knobs.
set -o pipefail
TAG=$1; REPS=$2; STEPS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG; mkdir -p "$O"
for r in $(seq 1 "$REPS"); do
  for lib in "$@"; do
    f="$O/b_${lib%.so}_$r"; f=${f//=/_}
    if [[ "$lib" == *=* ]]; then
      if [[ "$lib" == *=default ]]; then set_env="DCR_AB_ARM=default"; else set_env="$lib"; fi
    else
      set_env="${AB_VAR:-DCR_LIB}=duplexumiconsensusreads_amd/$lib"
    fi
    env "$set_env" timeout -k 10 300 python3 -u bench.py --no-cpu --steps "$STEPS" --warmup 2 > "$f.txt" 2>&1 || { echo "bench $lib failed rc=$?"; tail -20 "$f.txt"; exit 1; }
    grep '^{' "$f.txt" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['config']['stages_s_last_pass']; print('$lib', round(d['value']/1e6,1), 'M', 'l6', round(d['config']['whole_node_level6_input']['value']/1e6,1), 'ingest', s['ingest_s'], 'wait', s['wait_s'], 'idle', s['idle_s'], 'inflate_ms', round(s['gpu_inflate']['kernel_ms_per_pass'],1), 'host_cpu_s', s.get('host_cpu_s_per_pass'))" | tee -a "$O/ab.txt"
  done
done
