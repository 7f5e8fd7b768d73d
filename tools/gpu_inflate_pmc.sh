set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ipmc
mkdir -p $O
timeout -k 10 200 python3 -u tools/inflate_speed.py 100000 1 > $O/speed.json || exit 1
cat $O/speed.json
DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_istamp.so timeout -k 10 200 python3 -u tools/inflate_speed.py 100000 1 > $O/stamp.json || exit 1
cat $O/stamp.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $O/p1 -o p --output-format csv -- python3 tools/inflate_speed.py 20000 1 > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d $O/p2 -o p --output-format csv -- python3 tools/inflate_speed.py 20000 1 > $O/pmc2.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt
grep -A20 "k_inflate" $O/pmc_summary.txt
rm -rf $O/p1 $O/p2
