#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/probe
timeout -k 10 180 python3 -u tools/deflate_probe.py "$@" 2>&1 | tee gpurun_out/probe/deflate_probe.txt
