#!/bin/bash
# Round-4 GPU pass (run on the GPU box).  Stages, chosen by the arguments:
#   suite    smoke + the GPU test suite
#   bench    default bench.py
#   prof     rocprofv3 kernel trace + stats of the timed headline steps only
#            (bench.py --headline-only), FETCH_SIZE calibration (tools/scanbench
#            quadread vs prod) and the counter groups of tools/prof_workload.py
# Usage: tools/gpu_round4.sh <tag> <stage>...   Stops at the first failure;
# every GPU step has its own time limit.
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for stage in "$@"; do
  case $stage in
  suite)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
      || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 \
      || { echo "suite rc=$?"; tail -30 $OUT/gputest.log; exit 1; }
    tail -2 $OUT/gputest.log ;;
  bench)
    timeout -k 10 700 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
      || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
    tail -c 400 $OUT/bench.json ;;
  prof)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o headline --output-format csv -- \
      python3 $R/bench.py --headline-only > $OUT/headline_under_rocprof.json 2> $OUT/stats.err \
      || { echo "stats rc=$?"; tail -5 $OUT/stats.err; exit 1; }
    for mode in quadread prod; do
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib/$mode -o run -- \
        $R/tools/scanbench 8 $mode > $OUT/calib_$mode.log 2>&1 || { echo "calib $mode rc=$?"; exit 1; }
    done
    i=0
    for ctrs in "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
                "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmc/p$i -o run -- \
        python3 $R/tools/prof_workload.py --gib 16 > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
    done
    cd $R
    echo prof done ;;
  *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo round4 "$@" done
