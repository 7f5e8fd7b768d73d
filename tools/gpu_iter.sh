#!/bin/bash
# Kernel iteration on the GPU: the consensus parity tests, device-resident C2
# kernel times, and one rocprofv3 PMC pass of per-kernel instruction counts
# (SQ_INSTS_*; its own run, no trace options).  Every GPU step has its own
# time limit and the chain stops at the first failure.
#   usage: tools/gpu_iter.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-iter}
K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py "${KARG[@]}" -x -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$O/pytest_gpu.log" | head -30; exit 1; }
timeout -k 10 300 python3 -u bench.py --kernel-only --no-cpu --kernel-steps 20 > "$O/bench_k.json" 2> "$O/bench_k.log" || { echo "bench failed"; tail -20 "$O/bench_k.log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k.json')); k=d['config']['device_resident']['kernel_ms']; print({a: round(b,4) for a,b in k.items()}, 'step', round(d['config']['device_resident']['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d "$O/p1" -o p --output-format csv -- python3 bench.py --kernel-only --kernel-steps 3 --steps 1 --warmup 0 --no-cpu > "$O/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$O/pmc.log"; exit 1; }
python3 tools/pmc_summary.py "$O" > "$O/pmc_summary.txt" && grep -A9 "k_consensus_fast<false, false>" "$O/pmc_summary.txt"
rm -rf "$O/p1"
