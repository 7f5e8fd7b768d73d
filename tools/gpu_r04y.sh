#!/bin/bash
# round 4: deflate phase split now, and 8 MB of the C2 record stream for
# host-side parse studies.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04y}
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/deflate_probe.py "$O/records.bin" 2>&1 | tee "$O/deflate_probe.txt"
