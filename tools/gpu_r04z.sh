#!/bin/bash
# round 4: k_deflate instruction mix and LDS behaviour (PMC passes over the
# deflate probe), and the gfx950 counter list for later passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04z}
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || echo "list rc=$?"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d "$O/p1" -o p --output-format csv -- python3 tools/deflate_probe.py > "$O/p1.log" 2>&1 || { tail -5 "$O/p1.log"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d "$O/p2" -o p --output-format csv -- python3 tools/deflate_probe.py > "$O/p2.log" 2>&1 || { tail -5 "$O/p2.log"; exit 1; }
python3 tools/pmc_summary.py "$O" > "$O/pmc.txt"
rm -rf "$O/p1" "$O/p2"
grep -A16 "k_deflate" "$O/pmc.txt"
