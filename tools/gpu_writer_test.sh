set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_writer.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r02d/pytest_writer.log 2>&1; rc=$?
tail -30 gpurun_out/r02d/pytest_writer.log
exit $rc
