#!/bin/bash
# Kernel iteration: GPU parity tests, then device-resident kernel times
# (bench --kernel-only) for the given configs.
#   usage: tools/gpu_kq.sh TAG [configs...]   (default C2 C5)
set -o pipefail
TAG=${1:-kq}
shift
CFGS=${*:-C2 C5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" "$O/pytest_gpu.log" | head -20; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for c in $CFGS; do
  timeout -k 10 200 python3 -u bench.py --config $c --kernel-only --no-cpu --kernel-steps 20 > "$O/k_$c.json" 2> "$O/k_$c.log" || { echo "bench $c failed"; tail -20 "$O/k_$c.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/k_$c.json')); r=d['config']['device_resident']; print('$c dev %.3f ms'%r['ms_per_step'], {k: round(v,3) for k,v in r['kernel_ms'].items()}, 'frac %.3f'%d['roofline']['frac'], 'bad', r['records_not_ok'])"
done
