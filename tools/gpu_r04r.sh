#!/bin/bash
# round 4: per-phase s_memtime stamps of the fast and exact kernels on C5
# and C2 (a DCR_STAMP=1 build).  Each GPU step under its own limit.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04r}
L=duplexumiconsensusreads_amd
mkdir -p "$O"
ABL_CONFIG=C5 timeout -k 10 300 python3 -u tools/stamps.py 200000 $PWD/$L/libdcr_stamp.so 2>&1 | tee "$O/stamps_C5.txt" || exit 1
timeout -k 10 300 python3 -u tools/stamps.py 312500 $PWD/$L/libdcr_stamp.so 2>&1 | tee "$O/stamps_C2.txt" || exit 1
# HBM traffic of the C3 kernels (two PMC passes, tools/pmc_traffic.py)
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o f --output-format csv -- python3 bench.py --config C3 --kernel-only --kernel-steps 2 --steps 1 --warmup 0 --no-cpu > "$O/pmc_fetch.log" 2>&1 || { tail -5 "$O/pmc_fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o w --output-format csv -- python3 bench.py --config C3 --kernel-only --kernel-steps 2 --steps 1 --warmup 0 --no-cpu > "$O/pmc_write.log" 2>&1 || { tail -5 "$O/pmc_write.log"; exit 1; }
python3 tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" 400000 "$O/traffic_C3.json" && rm -rf "$O/pmc_fetch" "$O/pmc_write"
