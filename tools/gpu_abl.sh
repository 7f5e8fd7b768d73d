#!/bin/bash
# Fast-kernel cost split: ablation builds (libdcr_abl{1,2,5}.so: staging only,
# + evidence, no per-column stores) timed against the product build in one
# process, then the phase stamps of the DCR_STAMP build.
#   usage: tools/gpu_abl.sh TAG
set -o pipefail
TAG=${1:-abl}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
L=duplexumiconsensusreads_amd
timeout -k 10 300 python3 -u tools/ablate.py 312500 $L/libdcr.so $L/libdcr_abl1.so $L/libdcr_abl2.so $L/libdcr_abl5.so > "$O/ablate.txt" 2>&1 || { tail -20 "$O/ablate.txt"; exit 1; }
cat "$O/ablate.txt"
timeout -k 10 200 python3 -u tools/stamps.py 312500 $L/libdcr_stamp.so > "$O/stamps.txt" 2>&1 || { tail -5 "$O/stamps.txt"; exit 1; }
head -12 "$O/stamps.txt"
