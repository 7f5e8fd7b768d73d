#!/bin/bash
# Diagnostic builds of libdcr with other k_deflate shapes (dcr_deflate.h:
# -DDFL_T lanes per block, -DDFL_LS recency sets per lane, -DDFL_MW dwords
# per match-extension step), timed by tools/deflate_probe.py (DCR_LIB_PATH).
#   usage: tools/build_dfl.sh "name:flags" ...
set -e
cd "$(dirname "$0")/.."
C=duplexumiconsensusreads_amd/csrc
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags \
    -o duplexumiconsensusreads_amd/libdcr_dfl$name.so $C/dcr_kernels.hip $C/dcr_capi.hip $C/dcr_writer.hip $C/dcr_inflate.hip &
done
wait
