#!/bin/bash
# PMC passes over scanbench modes (run on the GPU box): usage pmc_scan.sh <outdir> <mode>...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
for mode in "$@"; do
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS" \
           "TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TA_BUFFER_WAVEFRONTS_sum" \
           "FETCH_SIZE" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/$mode/p$i -o run -- $R/tools/scanbench 16 $mode > $OUT/$mode.p$i.log 2>&1 || echo "pass $mode $i failed rc=$?" >> $OUT/fail.log
done
done
