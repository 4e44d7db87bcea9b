#!/bin/bash
# Kernel timeline of the configs[3] stand-in (80 000 small files), GPU box.
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o trace -- python3 $GRAFT_REPO_ROOT/bench.py \
  --steps 2 --warmup 1 --gib 2 --no-cpu --no-ids --e2e-gib 0 --batch-files 0 > $OUT/bench.log 2>&1
