#!/bin/bash
# round 4: whole-node bench three times after the ingest close / pool-cache
# change, then the CLI GPU tests.  Each GPU step under its own limit.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04u}
mkdir -p "$O"
for i in 1 2 3; do
  timeout -k 10 600 python3 -u bench.py --no-cpu > "$O/bench$i.json" 2> "$O/bench$i.log" || { tail -20 "$O/bench$i.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench$i.json')); s=d['config']['stages_s_last_pass']; print(round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'), 'open', s.get('open_s'), 'close', s.get('close_s'))"
done
timeout -k 10 600 python3 -u -m pytest tests/test_cli_cases.py tests/test_cli_e2e.py tests/test_gpu_shard.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 580 --timeout-method thread 2>&1 | tee "$O/pytest_cli.txt" | grep -E "PASSED|FAILED|passed|failed|c3 shard" || exit 1
