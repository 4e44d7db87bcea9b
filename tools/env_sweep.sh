#!/bin/bash
# A/B sweep of one environment knob (GPU box): headline bench per value.
# usage: tools/env_sweep.sh <outdir> <VAR> <value>...
OUT=gpurun_out/$1; VAR=$2; shift 2
mkdir -p $OUT
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --e2e-gib 0 --batch-files 0 \
    --small-files 0 --no-ids > $OUT/$VAR-$v.json 2> $OUT/$VAR-$v.err || { rc=$?; echo "$VAR=$v rc=$rc" >> $OUT/fail.log; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/$VAR-$v.json')); o=d['device_only']; print('$VAR=$v', d['value'], o, round(o['device_ms']-o['scan_ms'],3))"
done
