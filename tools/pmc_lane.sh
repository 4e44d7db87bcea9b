#!/bin/bash
# PMC passes over the lane-walk resolution kernels (GPU box), one counter
# group per pass (MI355X_MICROARCH.md): address path (TA), L1 / UTCL1
# translation, L1->L2 requests and latency, SQ instruction mix.
# usage: tools/pmc_lane.sh <outdir> [GiB]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
G=${2:-64}
mkdir -p $OUT
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  GIB=$G timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/dbg/dbg_lane.py > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo pmc done
