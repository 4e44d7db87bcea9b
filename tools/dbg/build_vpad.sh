#!/bin/bash
# k_emit VGPR-allocation builds for the ChunkData.hash item:
#   libmcdc_vpad0.so  k_emit unpadded: 184 VGPRs used of 184 allocated (the failing build)
#   libmcdc_vpadN.so  k_emit with v<N> touched, so next_free_vgpr = N + 1
# Probe: MCDC_LIBRARY=tools/dbg/libmcdc_vpad0.so python tools/dbg/hash_check.py 64 5
set -e
cd "$(dirname "$0")/../../mapache_amd"
for n in ${PADS:-0}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result -DMCDC_EMIT_VPAD=$n -fPIC -shared \
    -I../include -o ../tools/dbg/libmcdc_vpad$n.so csrc/mcdc_kernels.hip csrc/mcdc_blake3.hip csrc/mcdc_aead.hip \
    csrc/mcdc_api.hip &
done
wait
