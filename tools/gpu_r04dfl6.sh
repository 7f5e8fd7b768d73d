#!/bin/bash
# round 4: k_deflate parse scheduling (e2: before, sp: parse_dev) timed
# interleaved, the device-writer tests on the new libdcr.so (members equal
# to the host emulation's), and two whole-node bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04dfl6}
mkdir -p "$O"
for rep in 1 2; do
  for v in e2 sp; do
    DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_dfl$v.so timeout -k 10 200 python3 -u tools/deflate_probe.py > "$O/${v}_$rep.txt" 2>&1 || { echo "== $v failed"; tail -20 "$O/${v}_$rep.txt"; exit 1; }
    echo "== $v $rep"; grep -v amdgpu.ids "$O/${v}_$rep.txt"
  done
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_writer.py tests/test_gpu_inflate.py -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
grep -E "passed|failed" "$O/pytest.log" | tail -3; [ $rc = 0 ] || { tail -30 "$O/pytest.log"; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu > "$O/b_$rep.json" 2> "$O/b_$rep.log" || { echo "bench failed"; tail -20 "$O/b_$rep.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$rep.json')); s=d['config']['stages_s_last_pass']; print('$rep', round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'))" | tee -a "$O/summary.txt"
done
