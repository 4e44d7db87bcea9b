#!/bin/bash
# Round-3 GPU pass (run on the GPU box): smoke, the GPU suite, the default
# bench, a rocprofv3 kernel-trace + stats profile of the headline bench.
# Stops at the first failure; every GPU step has its own time limit.
set -o pipefail
OUT=gpurun_out/${1:-r3final}
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 \
  || { echo "suite rc=$?"; tail -30 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
  || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$OUT/stats -o bench --output-format csv -- \
  python3 $R/bench.py --batch-files 0 --small-files 0 --e2e-gib 0 --no-cpu --corpus-files-per-gpu 0 \
  > $R/$OUT/bench_under_rocprof.json 2> $R/$OUT/stats.err || { echo "stats rc=$?"; exit 1; }
echo round done
