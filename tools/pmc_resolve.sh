#!/bin/bash
# PMC passes over the resolution kernels (GPU box): usage tools/pmc_resolve.sh <outdir>
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM" \
           "VALUBusy"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/res/p$i -o run -- python3 $R/bench.py --gib 16 --steps 2 --warmup 1 --no-cpu --e2e-gib 0 --batch-files 0 --small-files 0 --no-ids > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/fail.log; case $rc in 124|137|134|139) exit $rc;; esac; }
done
