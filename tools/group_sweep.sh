#!/bin/bash
# Chain-group size sweep (GPU box): headline bench per MCDC_GROUP.
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for g in "$@"; do
  MCDC_GROUP=$g timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --e2e-gib 0 --batch-files 0 \
    --no-ids > $OUT/g$g.json 2> $OUT/g$g.err || { rc=$?; echo "g $g rc=$rc" >> $OUT/fail.log; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/g$g.json')); print('g$g', d['value'], d['device_only'], d['small_files']['ms_per_step'])"
done
