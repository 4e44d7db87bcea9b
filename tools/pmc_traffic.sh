#!/bin/bash
# HBM traffic of the scan kernel from PMC counters (run on the GPU box).
# usage: tools/pmc_traffic.sh <outdir> [GiB]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
GIB=${2:-8}
mkdir -p $OUT
i=0
for set in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --gib $GIB --steps 1 --warmup 1 --no-cpu --e2e-gib 0 > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/fail.log; case $rc in 124|137|134|139) exit $rc;; esac; }
done
