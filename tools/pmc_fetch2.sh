#!/bin/bash
# FETCH_SIZE of the product scan inside bench.py (8 GiB call) and of the
# calibration pattern (tools/scanbench quadread, known 8 GiB), one pass each.
# usage: tools/pmc_fetch2.sh <tag>
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/quadread -o run -- $R/tools/scanbench 8 quadread \
  > $OUT/quadread.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/bench -o run -- python3 $R/bench.py --gib 8 --steps 2 \
  --warmup 1 --no-cpu --e2e-gib 0 --batch-files 0 --small-files 0 --no-ids > $OUT/bench.log 2>&1
