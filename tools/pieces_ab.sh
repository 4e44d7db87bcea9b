#!/bin/bash
# A/B of the scan's lane pieces per run (MCDC_SCAN_PIECES: 1 = one lane per
# 4 KiB run, 0 = size-dependent choice) on calls of 1-16 GiB and on the
# configs[3] small-file stand-in.  usage: tools/pieces_ab.sh <tag>
set -u
OUT=gpurun_out/$1
mkdir -p $OUT
for gib in 1 4 16; do
  for pc in 1 0 1 0; do
    echo "gib=$gib pieces=$pc" >> $OUT/pieces.log
    MCDC_SCAN_PIECES=$pc timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gib $gib --no-cpu --no-ids \
      --e2e-gib 0 --batch-files 0 --small-files $([ $gib = 1 ] && echo 80000 || echo 0) > $OUT/b.tmp 2>&1 || { cat $OUT/b.tmp; exit 1; }
    grep '^{' $OUT/b.tmp | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['device_only'], d.get('small_files',{}).get('gib_s'), d.get('small_files',{}).get('ms_per_step'))" >> $OUT/pieces.log
  done
done
cat $OUT/pieces.log
