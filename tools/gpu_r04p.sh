#!/bin/bash
# round 4: the batch-end tail fix (general kernel's staged windows) on the
# regression test and the C3-shard CLI case; the ingest with deferred
# families and the bench line.  Each GPU step under its own limit.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04p}
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "batch_end_tail" -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee "$O/pytest_tail.txt" || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py::test_cli_device_writer_c3_shard -m gpu -x -v --timeout 580 --timeout-method thread 2>&1 | tee "$O/pytest_c3shard.txt" || exit 1
timeout -k 10 300 python3 -u tools/ingest_profile.py /tmp/c2_ingest.bam gpu 16 2>&1 | tee "$O/ingest.txt" || exit 1
timeout -k 10 600 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { tail -20 "$O/bench.log"; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); s=d['config']['stages_s_last_pass']; print(round(d['value']/1e6,1), 'M/s', s.get('passes_s'), 'ingest', s.get('ingest_s'), 'wait', s.get('wait_s'), 'idle', s.get('idle_s'))"
