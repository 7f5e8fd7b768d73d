#!/bin/bash
# Kernel-trace stats of the device-resident bench of one config shape.
#   usage: tools/gpu_kt.sh TAG CONFIG [extra bench args]
set -o pipefail
TAG=${1:-kt}; CFG=${2:-C2}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_$CFG" -o kt --output-format csv -- python3 bench.py --config $CFG --kernel-only --no-cpu --steps 3 --warmup 1 "$@" > "$O/kt_$CFG.json" 2> "$O/kt_$CFG.log" || { echo "kernel trace failed"; tail -20 "$O/kt_$CFG.log"; exit 1; }
find "$O/kt_$CFG" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_$CFG.csv" \;
rm -rf "$O/kt_$CFG"
cut -d, -f1-4 "$O/kernel_stats_$CFG.csv" | head -16
