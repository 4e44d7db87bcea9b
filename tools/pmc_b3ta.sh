#!/bin/bash
# TA/TD busy of the chunk-ID kernels (GPU box): usage tools/pmc_b3ta.sh <outdir> [GiB]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
GIB=${2:-8}
mkdir -p $OUT
i=0
for set in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TD_BUSY_avr GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/b3bench.py $GIB 2 > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/fail.log; exit $rc; }
done
