set -o pipefail
mkdir -p gpurun_out/pmcx; cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
run_probe() {  # $1 tag  $2 library
  MCDC_LIBRARY=$2 PROBE_TINY_ONLY=1 PROBE_SECONDS=40 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES_SAVED -d gpurun_out/pmcx/$1 -o run --output-format csv -- python3 -u tools/dbg/lds_probe.py 1000 > gpurun_out/pmcx/$1.log 2>&1 || return 1
  echo "$1: calls $(grep -c 'tiny dev' gpurun_out/pmcx/$1.log) failing $(grep -c 'hash-bad [1-9]' gpurun_out/pmcx/$1.log)"
}
run_probe product mapache_amd/libmcdc.so && run_probe mode5 tools/dbg/libmcdc_dbg5.so || exit 1
for t in 87 81; do timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES_SAVED -d gpurun_out/pmcx/mb$t -o run --output-format csv -- tools/dbg/lds_bcast_v$t 0 300 80000 > gpurun_out/pmcx/mb$t.log 2>&1 || exit 1; echo "mb$t: $(grep 'bad' gpurun_out/pmcx/mb$t.log | head -2)"; done
