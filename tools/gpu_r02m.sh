#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r02m}
mkdir -p "$O"
timeout -k 10 200 python3 -u tools/ingest_profile.py /tmp/c2.bam 16 16 12 > "$O/ingest_profile.txt" 2>&1 || { echo "ingest profile failed"; tail -20 "$O/ingest_profile.txt"; exit 1; }
cat "$O/ingest_profile.txt"
bash tools/gpu_r02.sh ${TAG:-r02m} run --kernel-steps 5
