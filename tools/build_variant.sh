#!/bin/bash
# Build libdcr variants for A/B runs (tools/ablate.py, tools/gpu.sh ablate=...):
#   tools/build_variant.sh NAME "-DFLAG=1 ..." [NAME "FLAGS" ...]  -> duplexumiconsensusreads_amd/libdcr_NAME.so
# (DCR_STAMP=1: per-phase stamps for tools/stamps.py; DCR_ABL=n: ablations)
set -e
cd "$(dirname "$0")/.."
C=duplexumiconsensusreads_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  # shellcheck disable=SC2086
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags \
    -o duplexumiconsensusreads_amd/libdcr_$name.so $C/dcr_kernels.hip $C/dcr_capi.hip $C/dcr_writer.hip $C/dcr_inflate.hip &
done
wait
