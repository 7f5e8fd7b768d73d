#!/bin/bash
# Whole-node bench lines with and without environment assignments (A/B on one
# box, interleaved: base env base env), 6 passes each.
#   usage: tools/gpu_e2e_env_ab.sh TAG VAR=value [VAR=value ...]
set -o pipefail
TAG=${1:-e2e_env}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for k in 1 2; do
  for v in base env; do
    if [ $v = env ]; then E="$*"; else E=""; fi
    timeout -k 10 400 env $E python3 -u bench.py --no-cpu --steps 6 > "$O/bench_${v}_$k.json" 2> "$O/bench_${v}_$k.log" || { echo "bench $v failed"; tail -20 "$O/bench_${v}_$k.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$k.json')); s=d['config']['stages_s_last_pass']; print('$v', 'value %.4g' % d['value'], 'passes', s['passes_s'])"
  done
done
