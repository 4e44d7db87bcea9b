#!/bin/bash
# LDS-table builds of libmcdc.so for the k_emit_long item:
#   libmcdc_dbg1.so  k_emit_long reads GEAR from an LDS copy (88 VGPRs, exact fill)
#   libmcdc_dbg5.so  same, the copy 512 bytes into the LDS allocation
#   libmcdc_dbg6.so  =1 with one more VGPR touched (90 used, 96 allocated)
# Probe: MCDC_LIBRARY=tools/dbg/libmcdc_dbgN.so PROBE_TINY_ONLY=1 python tools/dbg/lds_probe.py 1000
set -e
cd "$(dirname "$0")/../../mapache_amd"
for m in ${MODES:-1 5 6}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result -DMCDC_DBG_LDS=$m -fPIC -shared \
    -I../include -o ../tools/dbg/libmcdc_dbg$m.so csrc/mcdc_kernels.hip csrc/mcdc_blake3.hip csrc/mcdc_api.hip &
done
wait
