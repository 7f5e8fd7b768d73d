set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py --families 100000 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM -d gpurun_out/prof_pmc1 -o p1 --output-format csv -- python3 bench.py --families 100000 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/prof_pmc2 -o p2 --output-format csv -- python3 bench.py --families 100000 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pmc2.log 2>&1
echo done
