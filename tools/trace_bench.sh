#!/bin/bash
# Kernel timeline of a short headline bench (GPU box): rocprofv3 kernel trace (csv).
# usage: tools/trace_bench.sh <outdir> [env assignments...]
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
mkdir -p $OUT
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o trace -- python3 $GRAFT_REPO_ROOT/bench.py \
  --steps 3 --warmup 1 --no-cpu --e2e-gib 0 --batch-files 0 --small-files 0 > $OUT/bench.log 2>&1
