#!/bin/bash
# Segment-size sweep (GPU box): headline bench per MCDC_SEG_CHUNKS.
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for k in "$@"; do
  MCDC_SEG_CHUNKS=$k timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --e2e-gib 0 --batch-files 0 \
    --no-ids > $OUT/k$k.json 2> $OUT/k$k.err || { rc=$?; echo "k $k rc=$rc" >> $OUT/fail.log; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/k$k.json')); o=d['device_only']; print('k$k', d['value'], o, round(o['device_ms']-o['scan_ms'],3), d['small_files']['ms_per_step'])"
done
