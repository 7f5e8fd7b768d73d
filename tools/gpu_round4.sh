#!/bin/bash
# Round-4 evidence: the GPU suite, the batch-tail regression test against
# round 3's library (expected to fail there), the bench line (driver's
# default command), a kernel-trace profile of that command with per-launch-
# shape durations, the PMC traffic passes, and one device-resident line per
# other config shape.  Every GPU step has its own time limit; the chain
# stops at the first failure.
#   usage: tools/gpu_round4.sh TAG
set -o pipefail
TAG=${1:-round4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
L=duplexumiconsensusreads_amd
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 580 --timeout-method thread 2>&1 | tee "$O/pytest_gpu.log" | grep -E "PASSED|FAILED|ERROR|passed|failed|c3 shard" || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
DCR_LIB_PATH=$PWD/$L/libdcr_base.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k batch_end_tail -m gpu -v --timeout 120 --timeout-method thread > "$O/pytest_tail_round3_lib.log" 2>&1
echo "batch-tail test on round 3's library: rc=$? (nonzero expected)"; grep -E "passed|failed" "$O/pytest_tail_round3_lib.log" | tail -1
timeout -k 10 500 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
cat "$O/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$O/bench_prof.json" 2> "$O/bench_prof.log" || { echo "prof failed"; tail -30 "$O/bench_prof.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/kt" -name "*kernel_trace.csv" -exec python3 tools/kt_grid.py {} k_consensus_fast k_recmeta k_deflate k_inflate \; > "$O/kernel_grid.csv"
rm -rf "$O/kt"
head -12 "$O/kernel_grid.csv"
bash tools/gpu_traffic.sh "$TAG" || exit 1
for c in C3 C4 C5; do
  timeout -k 10 300 python3 -u bench.py --config $c --kernel-only --steps 5 --warmup 2 --no-cpu > "$O/bench_$c.json" 2> "$O/bench_$c.log" || { echo "bench $c failed"; tail -20 "$O/bench_$c.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); c=d['config']; k=c.get('device_resident', c); print('$c', 'ms/step %.3f' % k['ms_per_step'], {a: round(b, 3) for a, b in k['kernel_ms'].items()})"
done
timeout -k 10 300 python3 -u tools/ingest_profile.py /tmp/c2_ingest.bam gpu 16 > "$O/ingest.txt" 2>&1 && tail -2 "$O/ingest.txt"
echo "round evidence done"
