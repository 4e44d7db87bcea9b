"""Summarise the chunk-ID PMC passes (tools/gpu_round4.sh <tag> b3pmc, copied
back as gpurun_out/<tag>/b3pmc/) into profiles/<round>/b3_pmc.json: per
k_b3_leaves dispatch the median counters, VALU instructions per 64-byte block
and wave, VALUBusy, and the clock the chip held (GRBM_GUI_ACTIVE per XCD over
the dispatch's duration).  Usage: python tools/b3_pmc_summary.py <tag> <round>"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, rnd):
    acc, dur = defaultdict(lambda: defaultdict(float)), {}
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "b3pmc", "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "k_b3_leaves" not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(list)
    clocks = []
    for key, cs in acc.items():
        for c, v in cs.items():
            per[c].append(v)
        if "GRBM_GUI_ACTIVE" in cs:
            clocks.append(cs["GRBM_GUI_ACTIVE"] / 8 / dur[key] / 1e9)
    med = {c: statistics.median(v) for c, v in per.items()}
    n = 16 << 30
    blocks_per_wave_lane = n / 64  # 64-byte blocks; one lane per block
    out = {"what": "k_b3_leaves (chunk IDs) PMC, tools/gpu_round4.sh b3pmc: tools/b3bench.py 16 GiB, one rocprofv3 "
                   "--pmc pass per counter group, medians over the passes' k_b3_leaves dispatches",
           "counters_median": med,
           "valu_per_wave_block": round(med["SQ_INSTS_VALU"] * 64 / blocks_per_wave_lane, 1),
           "algorithmic_valu_per_block": 672,
           "valu_busy_pct": round(med.get("VALUBusy", 0.0), 2),
           "held_clock_ghz": round(statistics.median(clocks), 3) if clocks else None,
           "dispatch_ms_median_under_pmc": round(statistics.median(dur.values()) * 1e3, 3),
           "source": f"gpurun_out/{tag}/b3pmc"}
    os.makedirs(os.path.join(ROOT, "profiles", rnd), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", rnd, "b3_pmc.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_median"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
