#!/bin/bash
# FETCH_SIZE calibration: product scan vs the same load pattern without hashing.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
for mode in quadread prod; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$mode -o run -- $R/tools/scanbench 8 $mode > $OUT/$mode.log 2>&1 || { rc=$?; echo "$mode failed rc=$rc" >> $OUT/fail.log; exit $rc; }
done
