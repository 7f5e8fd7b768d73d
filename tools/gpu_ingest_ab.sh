#!/bin/bash
# GPU tests, the default bench line, then the host ingest alone with the
# current libdcr_io.so and with libdcr_io_old.so (A/B on the same box).
#   usage: tools/gpu_ingest_ab.sh TAG
set -o pipefail
TAG=${1:-ingest}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 500 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config']; print('value %.4g' % d['value'], c['stages_s_last_pass'])"
B=/tmp/ingest_ab.bam
for lib in new old new old; do
  if [ $lib = old ]; then cp duplexumiconsensusreads_amd/libdcr_io.so /tmp/io_new.so && cp duplexumiconsensusreads_amd/libdcr_io_old.so duplexumiconsensusreads_amd/libdcr_io.so; fi
  echo "== $lib"; timeout -k 10 200 python3 -u tools/ingest_profile.py $B 16 2>&1 | tail -2
  if [ $lib = old ]; then cp /tmp/io_new.so duplexumiconsensusreads_amd/libdcr_io.so; fi
done > "$O/ingest_ab.txt"
cat "$O/ingest_ab.txt"
