#!/bin/bash
# round 4: k_deflate variants (tools/build_dfl.sh) through the deflate probe,
# interleaved twice: time, ratio, phase stamps, zlib check, output hash.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04dfl}
VARS=${2:-"base crc xq both"}
mkdir -p "$O"
for rep in 1 2; do
  for v in $VARS; do
    DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_dfl$v.so timeout -k 10 200 python3 -u tools/deflate_probe.py > "$O/${v}_$rep.txt" 2>&1 || { echo "== $v failed"; tail -20 "$O/${v}_$rep.txt"; exit 1; }
    echo "== $v $rep"; grep -v amdgpu.ids "$O/${v}_$rep.txt"
  done
done
