#!/bin/bash
# round 4: the C3-shard CLI case where the GPU and oracle outputs differ:
# first differing record, with the current library and with round 3's.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
L=duplexumiconsensusreads_amd
O=gpurun_out/${1:-r04i}
mkdir -p "$O"
timeout -k 10 400 python3 -u tools/c3shard_diff.py 400000 6 2>&1 | tee "$O/diff_cur.txt"
rc=$?; echo "diff_cur rc=$rc"; [ $rc -ge 124 ] && exit 1
DCR_LIB_PATH=$PWD/$L/libdcr_base.so timeout -k 10 400 python3 -u tools/c3shard_diff.py 400000 6 2>&1 | tee "$O/diff_base.txt"
echo "diff_base rc=$?"
