#!/bin/bash
# round 4: every k-th ingest chunk inflated by the host pool beside the GPU
# inflate stream (DCR_HOST_CHUNK_EVERY), interleaved whole-node benches, then
# the full-size CLI byte-identity tests with k = 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04hc}
mkdir -p "$O"
for rep in 1 2; do
  for k in 0 2 3 4; do
    DCR_HOST_CHUNK_EVERY=$k timeout -k 10 300 python3 -u bench.py --no-cpu > "$O/b_${k}_$rep.json" 2> "$O/b_${k}_$rep.log" || { echo "bench $k failed"; tail -20 "$O/b_${k}_$rep.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${k}_$rep.json')); s=d['config']['stages_s_last_pass']; print('every $k rep $rep', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'))" | tee -a "$O/summary.txt"
  done
done
DCR_HOST_CHUNK_EVERY=3 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_inflate.py -m gpu -x -v --timeout 400 --timeout-method thread 2>&1 | tee "$O/pytest.log" | grep -E "PASSED|FAILED|ERROR|passed|failed"
