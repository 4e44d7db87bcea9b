#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel trace.  Each GPU step
# has its own time limit; stop at the first timeout / abort / crash.
# usage: tools/gpu_session.sh <tag> [steps...]   steps: test smoke bench prof
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { case $1 in 124|137|134|139|133) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/session.log
  tail -5 $OUT/$name.log | tee -a $OUT/session.log
  if fatal $rc; then echo "FATAL rc=$rc in $name; stopping" | tee -a $OUT/session.log; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    test)  run pytest_gpu 1200 python -m pytest tests -q -m gpu -x --timeout=900 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    scanvar) run scanvar 300 ./tools/scanbench 16 var ;;
    benchq) run benchq 600 python bench.py --steps 5 --warmup 2 --cpu-sample-gib 4 --e2e-gib 4 ;;
    prof)  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --e2e-gib 0 \
             --batch-files 0 --small-files 0 --no-ids \
             > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1); rc=$?; echo "== prof rc=$rc" | tee -a $OUT/session.log
           if fatal $rc; then exit $rc; fi ;;
    profall) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $GRAFT_REPO_ROOT/$OUT/profall -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu \
             --e2e-gib 0 > $GRAFT_REPO_ROOT/$OUT/profall.log 2>&1); rc=$?; echo "== profall rc=$rc" | tee -a $OUT/session.log
           if fatal $rc; then exit $rc; fi ;;
    pmc)   (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d $GRAFT_REPO_ROOT/$OUT/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --e2e-gib 0 \
             > $GRAFT_REPO_ROOT/$OUT/pmc_fetch.log 2>&1); rc=$?; echo "== pmc rc=$rc" | tee -a $OUT/session.log
           if fatal $rc; then exit $rc; fi ;;
  esac
done
echo "== session done" | tee -a $OUT/session.log
