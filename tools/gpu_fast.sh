#!/bin/bash
# Fast-kernel iteration: GPU parity tests, device-resident C2 kernel times,
# and the phase stamps of a DCR_STAMP build (libdcr_stamp.so).
#   usage: tools/gpu_fast.sh TAG
set -o pipefail
TAG=${1:-fast}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 -u bench.py --kernel-only --no-cpu --kernel-steps 20 > "$O/bench_k.json" 2> "$O/bench_k.log" || { echo "bench failed"; tail -20 "$O/bench_k.log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k.json')); k=d['config']['device_resident']['kernel_ms'] if 'device_resident' in d['config'] else d['config']['kernel_ms']; print({a: round(b,4) for a,b in k.items()}, 'frac', round(d['roofline']['frac'],4))"
if [ -f duplexumiconsensusreads_amd/libdcr_stamp.so ]; then
  timeout -k 10 200 python3 -u tools/stamps.py 312500 duplexumiconsensusreads_amd/libdcr_stamp.so > "$O/stamps.txt" 2>&1 || { echo "stamps failed"; tail -5 "$O/stamps.txt"; exit 1; }
  head -12 "$O/stamps.txt"
fi
