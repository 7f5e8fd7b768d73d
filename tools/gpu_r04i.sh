#!/bin/bash
# round 4: the C3-shard CLI case where the GPU and oracle outputs differ:
# the first differing record.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04i}
mkdir -p "$O"
timeout -k 10 400 python3 -u tools/c3shard_diff.py 400000 6 2>&1 | tee "$O/diff_cur.txt"
