#!/bin/bash
# A/B of diagnostic builds on one box: device-resident kernel times of each
# library (alternating, to cancel clock drift) and one PMC pass of issue
# counters per library.
#   usage: tools/ab_kernels.sh TAG CONFIG lib1.so lib2.so ...
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    DCR_LIB_PATH=$R/$L timeout -k 10 200 python3 -u bench.py --config $CFG --kernel-only --no-cpu --kernel-steps 20 > "$O/${n}_$rep.json" 2> "$O/${n}_$rep.log" || { echo "bench $n failed"; tail -20 "$O/${n}_$rep.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$rep.json')); r=d['config']['device_resident']; k=r['kernel_ms']; print('$n', 'dev %.3f'%r['ms_per_step'], 'fast_ss %.4f'%k['k_consensus_fast<ss>'], 'fast_ds %.4f'%k['k_consensus_fast<ds>'], 'exact_ss %.4f'%k['k_consensus_exact<ss>'], 'bad', r['records_not_ok'])"
  done
done
for L in "$@"; do
  n=$(basename "$L" .so)
  DCR_LIB_PATH=$R/$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_MUL_F64 -d "$O/pmc_$n/p1" -o p1 --output-format csv -- python3 bench.py --config $CFG --families 100000 --kernel-only --no-cpu --kernel-steps 1 > "$O/pmc_$n.log" 2>&1 || { echo "pmc $n failed"; tail -5 "$O/pmc_$n.log"; exit 1; }
  python3 tools/pmc_summary.py "$O/pmc_$n" > "$O/pmc_$n.txt" && grep -A9 "k_consensus_fast<false, false>" "$O/pmc_$n.txt" | sed "s/^/$n /"
done
