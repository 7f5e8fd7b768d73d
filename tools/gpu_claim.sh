#!/bin/bash
# general kernel: dynamic wave-uniform claiming (libdcr.so) vs the round-1
# static stride (libdcr_genstatic.so) on C3 and C4 shards, after the parity
# tests that exercise the general kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/claim
mkdir -p "$O"
timeout -k 10 170 python3 -u -m pytest -x -v --timeout 160 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py > "$O/pytest.log" 2>&1 || { echo "tests failed"; tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
L=duplexumiconsensusreads_amd
for cfg in C3 C4 C5; do
  n=100000; [ $cfg = C4 ] && n=1000
  ABL_CONFIG=$cfg timeout -k 10 200 python3 -u tools/ablate.py $n $L/libdcr_genstatic.so $L/libdcr.so 2>&1 | grep "slots" | sed "s/^/$cfg /" | tee -a "$O/ablate.txt" || exit 1
done
