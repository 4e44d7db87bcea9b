#!/bin/bash
# PMC passes over the chunk-ID kernels (GPU box): usage tools/pmc_b3.sh <outdir> [GiB]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
GIB=${2:-8}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES" \
           "VALUBusy" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/b3/p$i -o run -- python3 $R/tools/b3bench.py $GIB 2 > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/fail.log; case $rc in 124|137|134|139) exit $rc;; esac; }
done
