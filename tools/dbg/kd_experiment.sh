#!/bin/bash
# §3a experiment: the unpadded k_emit (184 of 184 VGPRs) against
# the byte-identical code with only its descriptor's allocation raised to 192
# (tools/dbg/kd_patch.py).  64 GiB headline stream, 5 calls each, hashes
# compared across calls and against the oracle (tools/dbg/hash_check.py).
set -o pipefail
mkdir -p gpurun_out/kd
for v in ${VARIANTS:-vpad0 vpad0_kd192}; do
  echo "== $v" | tee -a gpurun_out/kd/summary.txt
  MCDC_LIBRARY=tools/dbg/vp/libmcdc_$v.so timeout -k 10 240 python -u tools/dbg/hash_check.py 64 ${REPS:-5} \
    > gpurun_out/kd/$v.txt 2>&1 || { echo "rc=$? for $v" | tee -a gpurun_out/kd/summary.txt; exit 1; }
  grep "mismatches" gpurun_out/kd/$v.txt | tee -a gpurun_out/kd/summary.txt
done
