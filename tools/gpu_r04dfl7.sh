#!/bin/bash
# round 4: k_deflate count-phase ablations (timing only; members invalid)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04dfl7}
mkdir -p "$O"
for rep in 1 2; do
  for v in ${VARS:-sp nocnt nocrc nowarm}; do
    nv=1; [ $v = sp ] && nv=
    DFL_NOVERIFY=$nv DCR_LIB_PATH=duplexumiconsensusreads_amd/libdcr_dfl$v.so timeout -k 10 60 python3 -u tools/deflate_probe.py > "$O/${v}_$rep.txt" 2>&1 || { echo "== $v failed"; tail -20 "$O/${v}_$rep.txt"; exit 1; }
    echo "== $v $rep"; grep -v amdgpu.ids "$O/${v}_$rep.txt"
  done
done
