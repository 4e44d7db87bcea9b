#!/bin/bash
# PMC passes over the product scan kernel (scanbench prod); run on the GPU box.
# usage: tools/pmc_prod.sh <outdir> [GiB]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
GIB=${2:-16}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE" \
           "VALUBusy" "VALUUtilization" \
           "TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "FETCH_SIZE" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/prod/p$i -o run -- $R/tools/scanbench $GIB prod > $OUT/prod.p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/fail.log; case $rc in 124|137|134|139) exit $rc;; esac; }
done
