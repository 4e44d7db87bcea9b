#!/bin/bash
# Chunk-ID kernel A/B on one box: tools/b3bench.py with each library build in
# turn (ABAB...), 64 GiB stream.  usage: tools/b3_ab.sh lib1.so lib2.so ...
set -o pipefail
for r in 1 2; do
  for L in "$@"; do
    MCDC_LIBRARY=$L timeout -k 10 240 python -u tools/b3bench.py 64 5 || exit $?
  done
done
