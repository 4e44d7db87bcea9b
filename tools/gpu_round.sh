set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/gputest.log 2>&1
echo "suite rc=$?"; tail -3 gpurun_out/gputest.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"; tail -c 3000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
MCDC_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --gib 16 --corpus-files-per-gpu 1024 > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.err
echo "rehearse rc=$?"; tail -c 2000 gpurun_out/bench_rehearse2.json; tail -5 gpurun_out/bench_rehearse2.err
