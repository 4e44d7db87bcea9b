#!/bin/bash
# k_aead_ctr A/B builds (no VGPR guard: measurement only):
#   libmcdc_ctr_W_I.so  MCDC_CTR_WAVES=W waves per block, MCDC_CTR_ILP=I blocks per lane per AES call
# Probe: MCDC_LIBRARY=tools/dbg/libmcdc_ctr_16_1.so python tools/aead_bench.py 64 3
set -e
cd "$(dirname "$0")/../../mapache_amd"
for cfg in ${CFGS:-16_1 8_1 8_2}; do
  w=${cfg%_*}; i=${cfg#*_}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result -DMCDC_CTR_WAVES=$w -DMCDC_CTR_ILP=$i \
    -fPIC -shared -I../include -o ../tools/dbg/libmcdc_ctr_$cfg.so csrc/mcdc_kernels.hip csrc/mcdc_blake3.hip \
    csrc/mcdc_aead.hip csrc/mcdc_api.hip &
done
wait
