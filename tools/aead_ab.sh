#!/bin/bash
# Sealing A/B on one box: tools/aead_bench.py with each library build in turn
# (ABAB), 64 GiB stream.  usage: tools/aead_ab.sh lib1.so lib2.so ...
set -o pipefail
for r in 1 2; do
  for L in "$@"; do
    MCDC_LIBRARY=$L timeout -k 10 300 python -u tools/aead_bench.py 64 3 || exit $?
  done
done
