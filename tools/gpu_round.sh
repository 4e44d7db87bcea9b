#!/bin/bash
# Round-end GPU pass (run on the GPU box): smoke, the GPU suite, the default
# bench and a 2-rank rehearsal on one device.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/gputest.log 2>&1 \
  || { echo "suite rc=$?"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
tail -c 1500 gpurun_out/bench.json
MCDC_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --gib 16 \
  --corpus-files-per-gpu 1024 --no-seal > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.err \
  || { echo "rehearse rc=$?"; tail -20 gpurun_out/bench_rehearse2.err; exit 1; }
echo round done
