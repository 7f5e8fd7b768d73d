#!/bin/bash
# Whole-node bench lines alternating the current libdcr_io.so with
# libdcr_io_old.so (same box, interleaved: new old new old).
#   usage: tools/gpu_e2e_ab.sh TAG
set -o pipefail
TAG=${1:-e2e_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
L=duplexumiconsensusreads_amd
cp $L/libdcr_io.so /tmp/io_new.so
for lib in new old new old; do
  if [ $lib = new ]; then cp /tmp/io_new.so $L/libdcr_io.so; else cp $L/libdcr_io_old.so $L/libdcr_io.so; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu > "$O/bench_$lib.json" 2> "$O/bench_$lib.log" || { echo "bench $lib failed"; tail -20 "$O/bench_$lib.log"; cp /tmp/io_new.so $L/libdcr_io.so; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$lib.json')); s=d['config']['stages_s_last_pass']; print('$lib', 'value %.4g' % d['value'], 'passes', s['passes_s'], 'open %.3f close %.3f writers %.3f' % (s['open_s'], s['close_s'], s['close_writers_s']))"
done
cp /tmp/io_new.so $L/libdcr_io.so
