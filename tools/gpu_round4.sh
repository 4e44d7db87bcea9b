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
  zc)  # the GPU compressor: its tests, the save path's, then tools/zc_bench.py (2 GiB per corpus)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_zcomp.py tests/test_gpu_save.py -m gpu -x -v --timeout 300 \
      --timeout-method thread > $OUT/zc_tests.log 2>&1 || { echo "zc tests rc=$?"; tail -30 $OUT/zc_tests.log; exit 1; }
    tail -2 $OUT/zc_tests.log
    timeout -k 10 300 python -u tools/zc_bench.py 2 3 > $OUT/zc_bench.json 2> $OUT/zc_bench.err \
      || { echo "zc bench rc=$?"; tail -20 $OUT/zc_bench.err; exit 1; }
    cat $OUT/zc_bench.json ;;
  zcab)  # tools/zc_bench.py with each abship/*.so variant beside the product library (2 GiB text, binary)
    timeout -k 10 200 python -u tools/zc_bench.py 2 3 text,binary > $OUT/zcab_product.json 2>&1 || { echo "zcab product rc=$?"; exit 1; }
    echo "product $(cat $OUT/zcab_product.json)"
    for so in abship/*.so; do
      b=$(basename $so .so)
      MCDC_LIBRARY=$R/$so timeout -k 10 200 python -u tools/zc_bench.py 2 3 text,binary > $OUT/zcab_$b.json 2>&1 \
        || { echo "zcab $b rc=$?"; exit 1; }
      echo "$b $(cat $OUT/zcab_$b.json)"
    done ;;
  zcabs)  # kernel stats of the compressor with each abship/*.so variant (1 GiB text)
    cd /tmp && export TMPDIR=/tmp
    for so in $R/abship/*.so; do
      b=$(basename $so .so)
      MCDC_LIBRARY=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/zcabs_$b -o zc --output-format csv -- \
        python3 $R/tools/zc_bench.py 1 2 ${ZCAB_KIND:-text} > $OUT/zcabs_$b.json 2> $OUT/zcabs_$b.err || { echo "zcabs $b rc=$?"; exit 1; }
      echo "== $b $(cat $OUT/zcabs_$b.json)"
      python3 $R/tools/kcsv.py $OUT/zcabs_$b/zc_kernel_stats.csv
    done
    cd $R ;;
  zcstats)  # kernel trace + stats of the compressor only (1 GiB of text and of binary)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/zc_stats -o zc --output-format csv -- \
      python3 $R/tools/zc_bench.py 1 2 text,binary > $OUT/zc_under_rocprof.json 2> $OUT/zc_stats.err \
      || { echo "zc stats rc=$?"; tail -5 $OUT/zc_stats.err; exit 1; }
    python3 $R/tools/kcsv.py $OUT/zc_stats/zc_kernel_stats.csv
    cd $R ;;
  zcprof)  # kernel trace + stats of the compressor (1 GiB text), then PMC passes
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/zc_stats -o zc --output-format csv -- \
      python3 $R/tools/zc_bench.py 1 2 text,binary > $OUT/zc_under_rocprof.json 2> $OUT/zc_stats.err \
      || { echo "zc stats rc=$?"; tail -5 $OUT/zc_stats.err; exit 1; }
    i=0
    for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE" \
                "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
                "FETCH_SIZE" "WRITE_SIZE" \
                "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "VALUBusy GRBM_GUI_ACTIVE" \
                "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/zc_pmc/p$i -o run -- \
        python3 $R/tools/zc_bench.py 1 1 text > $OUT/zc_pmc_p$i.log 2>&1 || { echo "zc pmc pass $i rc=$?"; exit 1; }
    done
    cd $R
    echo zcprof done ;;
  c3trace)  # kernel traces of the configs[3] paths: 80 000 small files chunked (tools/small_probe.py)
             # and the kernel-tree save path with GPU compression (tools/tree_probe.py, 3 calls)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/small_trace -o small --output-format csv -- \
      python3 $R/tools/small_probe.py > $OUT/small_probe.log 2> $OUT/small_trace.err \
      || { echo "small trace rc=$?"; tail -5 $OUT/small_trace.err; exit 1; }
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/tree_trace -o tree --output-format csv -- \
      python3 $R/tools/tree_probe.py 80000 3 > $OUT/tree_probe.log 2> $OUT/tree_trace.err \
      || { echo "tree trace rc=$?"; tail -5 $OUT/tree_trace.err; exit 1; }
    cd $R
    cat $OUT/small_probe.log $OUT/tree_probe.log
    echo c3trace done ;;
  b3pmc)  # chunk-ID kernel counters (tools/b3bench.py 16 GiB): instruction mix, VALUBusy, the held clock
    cd /tmp && export TMPDIR=/tmp
    i=0
    for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
                "VALUBusy GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/b3pmc/p$i -o run -- \
        python3 $R/tools/b3bench.py 16 2 > $OUT/b3pmc_p$i.log 2>&1 || { echo "b3 pmc pass $i rc=$?"; exit 1; }
    done
    cd $R
    echo b3pmc done ;;
  calib)  # FETCH_SIZE of the scan (tools/scanbench prod) against the bare load pattern (quadread)
    cd /tmp && export TMPDIR=/tmp
    for mode in quadread prod; do
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib/$mode -o run -- \
        $R/tools/scanbench 8 $mode > $OUT/calib_$mode.log 2>&1 || { echo "calib $mode rc=$?"; exit 1; }
    done
    cd $R
    echo calib done ;;
  *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo round4 "$@" done
