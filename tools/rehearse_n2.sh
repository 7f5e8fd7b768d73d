#!/bin/bash
# 2-rank rehearsal of the bench's N>1 path on one GPU (both ranks wrap onto GPU 0; gloo control plane)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$1; mkdir -p "$O"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > "$O/bench_n2.txt" 2>&1; rc=$?
tail -3 "$O/bench_n2.txt"; echo "n2 rc=$rc"; exit $rc
