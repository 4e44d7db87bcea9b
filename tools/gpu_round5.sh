#!/bin/bash
# Round-5 GPU steps (run under gpurun from the repo root): each step has its
# own time limit, and the script stops at the first failing step.
#   tests FILES..   pytest -m gpu on the given test files
#   zcb KINDS P     tools/zc_bench.py 2 GiB, 3 steps (P16 or P512)
#   zcstat KINDS P  kernel trace + stats of tools/zc_bench.py 1 GiB, 2 steps
#   bench ARGS..    bench.py with ARGS
# Output under gpurun_out/$TAG (TAG from the environment, default r5).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5}
mkdir -p $OUT
mode=$1
shift
case $mode in
  tests)
    timeout -k 10 900 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread \
      > $OUT/tests.log 2>&1
    rc=$?
    tail -3 $OUT/tests.log
    exit $rc ;;
  zcb)
    timeout -k 10 300 python -u tools/zc_bench.py 2 3 $1 $2 > $OUT/zcb_$2.json 2>&1
    rc=$?
    cat $OUT/zcb_$2.json
    exit $rc ;;
  zcstat)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/zcstat_$2 -o zc --output-format csv -- \
      python3 $R/tools/zc_bench.py 1 2 $1 $2 > $OUT/zcstat_$2.json 2> $OUT/zcstat_$2.err \
      || { echo "zc stats rc=$?"; tail -5 $OUT/zcstat_$2.err; exit 1; }
    cd $R
    python3 tools/kcsv.py $OUT/zcstat_$2/zc_kernel_stats.csv 16 ;;
  bench)
    timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
    rc=$?
    tail -c 3000 $OUT/bench.json
    exit $rc ;;
  *)
    echo "unknown mode $mode"
    exit 2 ;;
esac
