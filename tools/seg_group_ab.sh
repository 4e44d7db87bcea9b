set -o pipefail
AB="0:10,0:16,0:24,0:32" AB_KNOB=MCDC_SEG_CHUNKS AB_GIB="64" timeout -k 10 300 python -u tools/pieces_big.py > gpurun_out/s4l_seg.log 2>&1 || exit $?
for g in 8 16; do MCDC_GROUP=$g AB="0:12,0:16,0:24" AB_KNOB=MCDC_SEG_CHUNKS AB_GIB="64" timeout -k 10 300 python -u tools/pieces_big.py > gpurun_out/s4l_g$g.log 2>&1 || exit $?; done
cat gpurun_out/s4l_seg.log gpurun_out/s4l_g8.log gpurun_out/s4l_g16.log
