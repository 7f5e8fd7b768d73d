#!/bin/bash
# k_deflate shapes: tools/deflate_probe.py (time, ratio, phase stamps, zlib
# check of every member) on libdcr.so and the tools/build_dfl.sh variants.
#   usage: tools/gpu_dfl.sh TAG [variants]
set -o pipefail
TAG=${1:-dfl}
VARS=${2-"512 1024"}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python3 -u tools/deflate_probe.py > $O/base.txt 2>&1 || { tail -20 $O/base.txt; exit 1; }
echo "== base"; grep -v amdgpu.ids $O/base.txt
for v in $VARS; do
  DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_dfl$v.so timeout -k 10 200 python3 -u tools/deflate_probe.py > $O/v$v.txt 2>&1 || { tail -20 $O/v$v.txt; exit 1; }
  echo "== T=$v"; grep -v amdgpu.ids $O/v$v.txt
done
