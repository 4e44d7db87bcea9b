#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
for mode in "$@"; do
i=0
for set in "SQC_ICACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_TC_INST_REQ SQC_TC_STALL SQ_IFETCH GRBM_GUI_ACTIVE" \
           "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_BRANCH SQ_IFETCH_LEVEL SQ_BUSY_CU_CYCLES" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/$mode/p$i -o run -- $R/tools/scanbench 16 $mode > $OUT/$mode.p$i.log 2>&1 || echo "pass $mode $i failed rc=$?" >> $OUT/fail.log
done
done
