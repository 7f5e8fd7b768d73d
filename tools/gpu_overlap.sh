#!/bin/bash
# host ingest profile on the box's cores, then a kernel + memory-copy trace
# of device-bound streaming (pre-ingested C5 batches through the two-slot
# DeviceStream) and its copy/compute overlap
set -o pipefail
TAG=${1:-overlap}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 200 python3 -u tools/ingest_profile.py /tmp/c2.bam 16 16 > "$O/ingest_profile.txt" 2>&1 || { echo "ingest profile failed"; tail -20 "$O/ingest_profile.txt"; exit 1; }
cat "$O/ingest_profile.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$O/tr" -o tr --output-format csv -- python3 -u tools/stream_resident.py /tmp/sr 250000 1048576 3 > "$O/stream_resident.txt" 2>&1 || { echo "trace failed"; tail -30 "$O/stream_resident.txt"; exit 1; }
grep -v "^W20\|^E20\|rocprofv3" "$O/stream_resident.txt" | tail -5
python3 tools/overlap.py "$O/tr" | tee "$O/overlap.txt"
find "$O/tr" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/tr" -name "*memory_copy_stats.csv" -exec cp {} "$O/memory_copy_stats.csv" \;
