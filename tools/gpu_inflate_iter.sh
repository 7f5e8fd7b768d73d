#!/bin/bash
# Inflate kernel iteration: GPU inflate tests, speed (tools/inflate_speed.py),
# the DINF_STAMP build's phase cycles, one PMC pass of instruction counts.
#   usage: tools/gpu_inflate_iter.sh TAG
set -o pipefail
TAG=${1:-iiter}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 60 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -u tools/inflate_speed.py 100000 1 > $O/speed.json || exit 1
cat $O/speed.json
DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_istamp.so timeout -k 10 200 python3 -u tools/inflate_speed.py 20000 1 > $O/stamp.json || exit 1
cat $O/stamp.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $O/p1 -o p --output-format csv -- python3 tools/inflate_speed.py 20000 1 > $O/pmc1.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt
grep -A10 "k_inflate" $O/pmc_summary.txt
rm -rf $O/p1
