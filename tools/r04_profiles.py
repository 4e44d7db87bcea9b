"""Copy a GPU pass (tools/gpu_round4.sh <tag> suite bench prof zcprof, merged
back as gpurun_out/<tag>/) into profiles/rNN/ (round 4 by default):

  bench_default.json          the default bench line
  gpu_suite.txt               the GPU suite's summary lines
  headline_kernel_stats.csv   rocprofv3 --stats of bench.py --headline-only
  headline_trace_summary.json per-launch scan durations from that trace, the
                              profile-derived roofline fraction beside the line's
  pmc_traffic.json            calibrated FETCH_SIZE of the shipping scan
                              (tools/scanbench prod vs quadread, MI355X_MICROARCH.md)
  zstd/zc_kernel_stats.csv    rocprofv3 --stats of tools/zc_bench.py 1 2 text,binary
  zstd/pmc_text.json          the compressor's counter groups (tools/zc_pmc_summary.py)

usage: python tools/r04_profiles.py <tag> [round]"""
import csv
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def line(path):
    return [x for x in open(path) if x.startswith("{")][-1]


def fetch(path, match):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if match in r["Kernel_Name"]]
    return v


def main(tag, rnd=4):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", f"r{rnd:02d}")
    os.makedirs(os.path.join(dst, "zstd"), exist_ok=True)
    bench = line(os.path.join(src, "bench.json"))
    open(os.path.join(dst, "bench_default.json"), "w").write(bench)
    suite = [x for x in open(os.path.join(src, "gputest.log")) if "passed" in x or "failed" in x]
    open(os.path.join(dst, "gpu_suite.txt"), "w").write("".join(suite[-2:]))
    shutil.copy(os.path.join(src, "stats", "headline_kernel_stats.csv"), os.path.join(dst, "headline_kernel_stats.csv"))
    # per-launch durations of the headline scan (3 warm-up + 10 timed launches)
    rows = [r for r in csv.DictReader(open(os.path.join(src, "stats", "headline_kernel_trace.csv")))
            if "k_scan_q" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    prof_line = json.loads(line(os.path.join(src, "headline_under_rocprof.json")))
    warm = prof_line["warmup"]
    timed = d[warm:]
    rl = prof_line["roofline"]
    frac = rl["bytes_per_launch"] / (statistics.mean(timed) * 1e-3) / 1e9 / rl["peak"]
    json.dump({"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --headline-only (tools/gpu_round4.sh prof)",
               "k_scan_q_launches": len(d), "warmup": warm, "steps": len(timed),
               "launch_ms": [round(x, 3) for x in d],
               "timed_mean_ms": round(statistics.mean(timed), 4), "timed_min_ms": round(min(timed), 4),
               "timed_max_ms": round(max(timed), 4), "warmup_first_ms": round(d[0], 3),
               "frac_from_trace": round(frac, 4), "line_avg_launch_ms_hip_events": rl["avg_launch_ms"],
               "line_frac": rl["frac"], "agreement": round(min(frac, rl["frac"]) / max(frac, rl["frac"]), 3),
               "source": f"gpurun_out/{tag}/stats",
               "note": "every launch is the 64 GiB headline call; the first (warm-up) launch runs on freshly "
                       "written memory and is the slow outlier"},
              open(os.path.join(dst, "headline_trace_summary.json"), "w"), indent=1)
    # calibrated traffic: known 8 GiB read by the product's load pattern vs the scan over the same 8 GiB
    nbytes = 8 << 30
    q = fetch(os.path.join(src, "calib", "quadread", "run_counter_collection.csv"), "k_read_quad")
    s = fetch(os.path.join(src, "calib", "prod", "run_counter_collection.csv"), "k_scan_q")
    fq, fs = statistics.median(q), statistics.median(s)
    factor = nbytes / (fq * 1024)
    json.dump({"what": "HBM/fabric read traffic of the shipping k_scan_q<4096, 2, true> from rocprofv3 --pmc "
                       "FETCH_SIZE (separate passes, tools/gpu_round4.sh prof / calib)",
               "input_bytes": nbytes, "fetch_size_kib_calibration_kernel": fq, "calibration_launches": len(q),
               "calibration": "tools/scanbench quadread: the product's quad-coalesced 16 B/lane load pattern, no "
                              "hashing, known 8 GiB; factor = bytes / (FETCH_SIZE*1024) (MI355X_MICROARCH.md: "
                              "FETCH_SIZE counts ~1/2 of wide streaming reads on gfx950)",
               "calibration_factor": round(factor, 4), "kernel": "k_scan_q<4096, 2, true>",
               "fetch_size_kib_scan": fs, "scan_launches": len(s),
               "scan_read_bytes_corrected": int(fs * 1024 * factor),
               "traffic_per_input_byte": round(fs * 1024 * factor / nbytes, 4),
               "measured": f"gpurun_out/{tag}/calib (tools/scanbench 8 prod vs quadread, 8 GiB), round {rnd}"},
              open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, "zc_stats", "zc_kernel_stats.csv"), os.path.join(dst, "zstd", "zc_kernel_stats.csv"))
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "zc_pmc_summary.py"), tag,
                    os.path.join("profiles", f"r{rnd:02d}", "zstd", "pmc_text.json")], check=True, cwd=ROOT)
    print(bench.strip()[:300])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
