#!/bin/bash
# fast-kernel phase stamps and ablations on the C2 batch (diagnostic builds)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/fastabl
mkdir -p "$O"
L=duplexumiconsensusreads_amd
timeout -k 10 150 python3 -u tools/stamps.py 312500 $L/libdcr_stamp.so 2>&1 | grep -v amdgpu.ids | tee "$O/stamps.txt" || exit 1
timeout -k 10 200 python3 -u tools/ablate.py 312500 $L/libdcr.so $L/libdcr_abl1.so $L/libdcr_abl2.so $L/libdcr_abl5.so $L/libdcr_abl6.so $L/libdcr_abl13.so 2>&1 | grep slots | tee "$O/ablate.txt"
