#!/bin/bash
# Chunk-ID A/B: round-2 transpose (80-byte rows) vs the swizzled 64-byte rows,
# alternating builds on one box (tools/b3bench.py, 16 GiB), then PMC of the
# new build: LDS bank conflicts and HBM read bytes (FETCH_SIZE, x2 on gfx950).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b3swz
for i in 1 2; do
  for v in old new; do
    L=""; [ $v = old ] && L=$R/ablib/libmcdc_b3old.so
    MCDC_LIBRARY=$L timeout -k 10 120 python3 $R/tools/b3bench.py 16 5 >> $R/gpurun_out/b3swz/ab_$v.txt 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for set in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "FETCH_SIZE"; do
  for v in old new; do
    L=""; [ $v = old ] && L=$R/ablib/libmcdc_b3old.so
    MCDC_LIBRARY=$L timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/b3swz/pmc_${v}_${set%% *} -o run -- python3 $R/tools/b3bench.py 8 2 > $R/gpurun_out/b3swz/pmc_$v.log 2>&1 || exit 1
  done
done
