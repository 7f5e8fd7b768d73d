set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
timeout -k 10 400 python3 -u bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/ab/cached.json 2> gpurun_out/ab/cached.log || exit 1
DCR_BACKEND_CACHE=0 timeout -k 10 400 python3 -u bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/ab/fresh.json 2> gpurun_out/ab/fresh.log || exit 1
for f in cached fresh; do python3 -c "import json; d=json.load(open('gpurun_out/ab/$f.json')); s=d['config']['stages_s_last_pass']; print('$f', round(d['value']/1e6,1), s['passes_s'], s['first_pass_s'], 'wait', s['wait_s'], 'ingest', s['ingest_s'])"; done
