#!/bin/bash
# Sealing builds with MCDC_AEAD_PERSIST = 0..3 (bit 0: persistent k_aead_polyval,
# bit 1: persistent k_aead_ctr): libmcdc_persistN.so
set -e
cd "$(dirname "$0")/../../mapache_amd"
for n in ${MODES:-0 1 2}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result -DMCDC_AEAD_PERSIST=$n -fPIC -shared \
    -I../include -o ../tools/dbg/libmcdc_persist$n.so csrc/mcdc_kernels.hip csrc/mcdc_blake3.hip csrc/mcdc_aead.hip \
    csrc/mcdc_api.hip &
done
wait
