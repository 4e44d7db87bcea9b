#!/bin/bash
# Frame-writer A/B on one box: tools/zframe_bench.py with each library build
# in turn, twice.  usage: tools/zf_ab.sh lib1.so lib2.so ...
set -o pipefail
for r in 1 2; do
  for L in "$@"; do
    MCDC_LIBRARY=$L timeout -k 10 120 python -u tools/zframe_bench.py 16 5 || exit $?
  done
done
