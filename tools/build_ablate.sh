#!/bin/bash
# Diagnostic builds of libdcr with -DDCR_ABL=n (see dcr_kernels.hip): phases of
# the fast kernel cut off one at a time, timed by tools/ablate.py.
set -e
cd "$(dirname "$0")/.."
C=duplexumiconsensusreads_amd/csrc
for n in 1 2 4 5 6 7 8; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -DDCR_ABL=$n \
    -o duplexumiconsensusreads_amd/libdcr_abl$n.so $C/dcr_kernels.hip $C/dcr_capi.hip $C/dcr_writer.hip &
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -DDCR_STAMP=1 \
  -o duplexumiconsensusreads_amd/libdcr_stamp.so $C/dcr_kernels.hip $C/dcr_capi.hip $C/dcr_writer.hip &
wait
