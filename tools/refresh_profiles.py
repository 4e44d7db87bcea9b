"""Copy a gpu_session.sh run (gpurun_out/<tag>) into profiles/r01: the bench
line, the rocprofv3 --stats summaries, the bench line measured under the
profiler and the per-launch scan durations from the trace.
usage: python tools/refresh_profiles.py <tag>"""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1]
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", "r01")
line = [x for x in open(os.path.join(src, "bench.log")) if x.startswith("{")][-1]
open(os.path.join(dst, "bench_default.json"), "w").write(line)
shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(dst, "bench_kernel_stats.csv"))
shutil.copy(os.path.join(src, "profall", "run_kernel_stats.csv"),
            os.path.join(dst, "bench_all_workloads_kernel_stats.csv"))
prof_line = [x for x in open(os.path.join(src, "prof.log")) if x.startswith("{")][-1]
open(os.path.join(dst, "bench_under_rocprof.json"), "w").write(prof_line)
rows = [r for r in csv.DictReader(open(os.path.join(src, "prof", "run_kernel_trace.csv")))
        if "k_scan_q" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
timed = d[2:7]
out = {"source": f"rocprofv3 --kernel-trace (gpurun_out/{tag}/prof/run_kernel_trace.csv) of: python3 bench.py "
                 "--steps 5 --warmup 2 --no-cpu --e2e-gib 0 --batch-files 0 --small-files 0 --no-ids",
       "k_scan_q_launch_ms_in_order": [round(x, 3) for x in d],
       "order": "2 warm-up + 5 timed headline steps, 1 + 3 host_out steps, 1 + 3 steps at 512K/1M/8M",
       "timed_headline_mean_ms": round(sum(timed) / len(timed), 3),
       "bench_hip_event_avg_launch_ms_same_run": json.loads(prof_line)["roofline"]["avg_launch_ms"]}
json.dump(out, open(os.path.join(dst, "scan_launches_from_trace.json"), "w"), indent=1)
print(json.dumps(out))
