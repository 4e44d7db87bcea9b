#!/bin/bash
# PMC passes over the sealing kernels (tools/aead_bench.py, 8 GiB, 1 call each
# of seal and open): LDS conflicts/activity, instruction mix, wave cycles and
# the GPU clock.  Usage: tools/aead_pmc.sh <outdir>
set -e
OUT=${1:-gpurun_out/aead_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_SALU"
i=0
for ctrs in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/p$i -o run -- python3 tools/aead_bench.py 8 1 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
done
