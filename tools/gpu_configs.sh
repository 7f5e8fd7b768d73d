#!/bin/bash
# GPU parity tests (optionally a -k filter) then one bench line per config shape.
#   usage: tools/gpu_configs.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-cfg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
K=${2:+-k "$2"}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
grep -cE "PASSED" "$O/pytest_gpu.log"; tail -2 "$O/pytest_gpu.log"
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > "$O/bench_$c.json" 2> "$O/bench_$c.log" || { echo "bench $c failed"; tail -20 "$O/bench_$c.log"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('$c', '%.3g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['config']['device_resident']['kernel_ms'].items()}, 'frac %.3f'%d['roofline']['frac'])"
done
