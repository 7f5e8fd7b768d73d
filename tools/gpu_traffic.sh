#!/bin/bash
# HBM traffic per launch of the consensus kernels: two rocprofv3 PMC passes
# (FETCH_SIZE, WRITE_SIZE; each its own run, no trace options) over the
# device-resident bench loop (C2, or the config named by the second argument:
# C3 ...), corrected by tools/pmc_traffic.py
set -o pipefail
TAG=${1:-traffic}
CFG=${2:-}
if [ -n "$CFG" ]; then
  CARGS="--config $CFG"; SFX="_$CFG"
  FAMS=${3:-400000}      # families per launch (bench.py --config C3 --kernel-only: 400 k)
else
  CARGS=""; SFX=""; FAMS=312500
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o f --output-format csv -- python3 bench.py $CARGS --kernel-only --kernel-steps 3 --steps 1 --warmup 0 --no-cpu > "$O/pmc_fetch$SFX.log" 2>&1 || { echo "pmc fetch failed"; tail -5 "$O/pmc_fetch$SFX.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o w --output-format csv -- python3 bench.py $CARGS --kernel-only --kernel-steps 3 --steps 1 --warmup 0 --no-cpu > "$O/pmc_write$SFX.log" 2>&1 || { echo "pmc write failed"; tail -5 "$O/pmc_write$SFX.log"; exit 1; }
python3 tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" "$FAMS" "$O/traffic$SFX.json" && python3 -c "
import json; d = json.load(open('$O/traffic$SFX.json'))
for k, v in d['kernels'].items(): print(k, round(v['hbm_bytes_per_launch'] / 1e9, 3), 'GB')"
rm -rf "$O/pmc_fetch" "$O/pmc_write"
