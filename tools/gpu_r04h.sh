#!/bin/bash
# round 4: the kept build (LDS fix, inflate 4 KiB ring / 9-bit table, no event
# layout): the GPU suite, kernel A/B against round 3 on C2 / C3 / C5, the
# ingest alone with the GPU inflate, the default bench line, then the long
# C3-shard CLI parity case on its own.  Each GPU step under its own limit;
# the first failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04h}
mkdir -p "$O"
step() { local name=$1; shift; "$@" > "$O/$name.txt" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -8 "$O/$name.txt" | cut -c1-400; return $rc; }
step pytest timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_fullsize.py::test_cli_device_writer_c3_shard || exit 1
step ablate timeout -k 10 300 python3 -u tools/ablate.py 312500 $L/libdcr_base.so $L/libdcr.so || exit 1
ABL_CONFIG=C3 step ablate_C3 timeout -k 10 300 python3 -u tools/ablate.py 100000 $L/libdcr_base.so $L/libdcr.so || exit 1
ABL_CONFIG=C5 step ablate_C5 timeout -k 10 300 python3 -u tools/ablate.py 200000 $L/libdcr_base.so $L/libdcr.so || exit 1
step ingest timeout -k 10 300 python3 -u tools/ingest_profile.py /tmp/c2_ingest.bam gpu 16 || exit 1
step bench timeout -k 10 600 python3 -u bench.py || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py::test_cli_device_writer_c3_shard -m gpu -x -v --timeout 580 --timeout-method thread 2>&1 | tee "$O/pytest_c3shard.txt" || exit 1
