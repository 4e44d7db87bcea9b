#!/bin/bash
# Round profile set (run on the GPU box): rocprofv3 kernel-trace + stats of
# the bench command, then separate --pmc passes (one counter group each, as
# MI355X_MICROARCH.md prescribes) on tools/prof_workload.py, and the
# FETCH_SIZE calibration of tools/pmc_calib.sh; then the sealing kernels'
# kernel trace (tools/aead_bench.py) and PMC passes (tools/aead_pmc.sh).
# Usage: profile_round.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$1
mkdir -p $OUT
cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- \
  python3 bench.py --batch-files 0 --small-files 0 --e2e-gib 0 --no-cpu --corpus-files-per-gpu 0 > $OUT/bench_under_rocprof.json 2> $OUT/stats.err || { echo "stats rc=$?"; exit 1; }
i=0
for ctrs in "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmc/p$i -o run -- python3 tools/prof_workload.py --gib 16 > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
done
for mode in quadread prod; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib/$mode -o run -- $R/tools/scanbench 8 $mode > $OUT/calib_$mode.log 2>&1 || { echo "calib $mode rc=$?"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/aead_stats -o aead --output-format csv -- \
  python3 tools/aead_bench.py 64 3 > $OUT/aead_under_rocprof.log 2>&1 || { echo "aead stats rc=$?"; exit 1; }
bash tools/aead_pmc.sh $OUT/aead_pmc || { echo "aead pmc rc=$?"; exit 1; }
echo profile done
