#!/bin/bash
# C5 / C3 / C2 device-resident steps with and without the direct exact queue
# (DCR_EXACT_DIRECT_R=0 turns it off), after the parity tests.
#   usage: tools/gpu_c5ab.sh TAG
set -o pipefail
TAG=${1:-c5ab}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for c in C5 C3 C2; do
  for d in 3 0; do
    DCR_EXACT_DIRECT_R=$d timeout -k 10 300 python3 -u bench.py --config $c --kernel-only --no-cpu --kernel-steps 10 --steps 1 --warmup 1 > "$O/b_${c}_$d.json" 2> "$O/b_${c}_$d.log" || { tail -10 "$O/b_${c}_$d.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${c}_$d.json')); k=d['config']['device_resident']; print('$c direct_r=$d', 'step %.3f' % k['ms_per_step'], {a: round(b,3) for a,b in k['kernel_ms'].items()})"
  done
done
