for v in 1 0 1 0; do
  MCDC_PINNED_DIRECT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --e2e-gib 0 --batch-files 0 --small-files 0 --no-ids > gpurun_out/s4s_$v.json 2>gpurun_out/s4s_$v.err || exit $?
  python -c "import json; d=json.loads([x for x in open('gpurun_out/s4s_$v.json') if x.startswith('{')][-1]); print('direct=$v', d['ms_per_step'], d['host_out'])" >> gpurun_out/s4s.log
done
cat gpurun_out/s4s.log
