#!/bin/bash
# The sharded CLI (cli --gpus: split points, one process per rank over a
# range of whole families, parallel part merge) timed by bench.py --sharded:
# one rank, then two ranks sharing the box's one GPU (a rehearsal of the
# machinery, not a scaling number: both ranks share one GPU and 16 CPUs).
#   usage: tools/gpu_sharded.sh TAG
set -o pipefail
TAG=${1:-sharded}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --sharded --no-cpu --kernel-steps 2 --steps 3 --warmup 1 > "$O/sharded_n1.json" 2> "$O/sharded_n1.log" || { tail -20 "$O/sharded_n1.log"; exit 1; }
tail -c 600 "$O/sharded_n1.json"; echo
timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --sharded --no-cpu --kernel-steps 2 --steps 3 --warmup 1 > "$O/sharded_n2_one_gpu.json" 2> "$O/sharded_n2_one_gpu.log" || { tail -20 "$O/sharded_n2_one_gpu.log"; exit 1; }
python3 -c "
import json
for f in ('sharded_n1', 'sharded_n2_one_gpu'):
    d = json.loads(open('$O/' + f + '.json').read().strip().splitlines()[-1]); c = d['config']
    print(f, round(d['value'] / 1e6, 1), 'M consensus bases/s', 'ms/pass', round(d['ms_per_step'], 1), [{k: r.get(k) for k in ('rank', 'e2e_s_per_pass', 'ingest_s', 'merge_s', 'shard_rounds')} for r in c['per_rank']])
" | tee "$O/summary.txt"
