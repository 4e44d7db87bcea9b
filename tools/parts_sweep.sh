#!/bin/bash
# Staged-pipeline sweep (GPU box): headline bench per MCDC_PARTS / MCDC_TAIL_ROUNDS setting.
# usage: tools/parts_sweep.sh <outdir> "parts:tail" ...
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for cfg in "$@"; do
  P=${cfg%%:*}; T=${cfg##*:}
  MCDC_PARTS=$P MCDC_TAIL_ROUNDS=$T timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --e2e-gib 0 \
    --batch-files 0 --small-files 0 > $OUT/p${P}_t${T}.json 2> $OUT/p${P}_t${T}.err || { rc=$?; echo "cfg $cfg rc=$rc" >> $OUT/fail.log; exit $rc; }
  python -c "import json,sys; d=json.load(open('$OUT/p${P}_t${T}.json')); print('$cfg', d['value'], d['ms_per_step'], d['device_only'])"
done
