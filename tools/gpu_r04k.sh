#!/bin/bash
# round 4: the C3-shard difference (which tag, which columns); the ingest
# with families completed on the packer thread (DCR_INGEST_PROF) and the
# default bench line.  Each GPU step under its own limit.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04k}
mkdir -p "$O"
timeout -k 10 400 python3 -u tools/c3shard_diff.py 400000 6 2>&1 | tee "$O/diff_cur.txt"
timeout -k 10 300 python3 -u tools/ingest_profile.py /tmp/c2_ingest.bam gpu 16 2>&1 | tee "$O/ingest.txt" || exit 1
timeout -k 10 600 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { tail -20 "$O/bench.log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); s=d['config']['stages_s_last_pass']; print(round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'))"
