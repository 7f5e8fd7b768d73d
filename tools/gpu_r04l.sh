#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:-r04l}
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/fam_bisect.py 34042 2>&1 | tee "$O/bisect.txt"
