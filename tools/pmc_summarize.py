"""Summarise a round's rocprofv3 outputs (tools/profile_round.sh <tag>, copied
back as gpurun_out/prof_<tag>/) into profiles/<tag>/:

  pmc_traffic.json   scan HBM read traffic from FETCH_SIZE, calibrated on the
                     product's own 16 B/lane load pattern (tools/scanbench
                     quadread, known bytes) -- MI355X_MICROARCH.md's HBM recipe
  pmc_summary.json   per-dispatch medians of the counter groups for the scan,
                     the emitters and the chunk-ID kernels (tools/prof_workload.py
                     --gib 16), with derived per-byte / per-block rates
  aead_pmc.json      the sealing kernels (tools/aead_pmc.sh: tools/aead_bench.py
                     8 GiB): LDS conflicts and activity, instruction mix, clock
  bench_kernel_stats.csv, aead_kernel_stats.csv  (copied)

Usage: python tools/pmc_summarize.py <tag>
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def per_dispatch(files, match):
    """{counter: [value per dispatch]} for kernels whose name contains `match`
    (a dispatch's value summed over its rows, e.g. per-XCD instances)."""
    acc = defaultdict(lambda: defaultdict(float))
    dur = {}
    for f in files:
        for r in rows(f):
            if match not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = defaultdict(list)
    for key, cs in acc.items():
        for c, v in cs.items():
            out[c].append(v)
        out["duration_s"].append(dur[key])
    return out


def med(xs):
    return statistics.median(xs) if xs else None


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for a, b in (("stats/bench_kernel_stats.csv", "bench_kernel_stats.csv"),
                 ("aead_stats/aead_kernel_stats.csv", "aead_kernel_stats.csv"),
                 ("bench_under_rocprof.json", "bench_under_rocprof.json")):
        if os.path.exists(os.path.join(src, a)):
            shutil.copy(os.path.join(src, a), os.path.join(dst, b))

    # ---- traffic: calibration on the product's load pattern
    q = per_dispatch([os.path.join(src, "calib/quadread/run_counter_collection.csv")], "k_read_quad")
    p = per_dispatch([os.path.join(src, "calib/prod/run_counter_collection.csv")], "k_scan_q")
    n_cal = 8 << 30
    fq, fp = med(q["FETCH_SIZE"]), med(p["FETCH_SIZE"])
    factor = n_cal / (fq * 1024)
    traffic = {
        "what": "HBM/fabric read traffic of k_scan_q from rocprofv3 --pmc FETCH_SIZE (separate passes, "
                "tools/profile_round.sh)",
        "input_bytes": n_cal, "fetch_size_kib_calibration_kernel": fq, "calibration_launches": len(q["FETCH_SIZE"]),
        "calibration": "tools/scanbench quadread: the product's quad-coalesced 16 B/lane load pattern, no hashing, "
                       "known 8 GiB; factor = bytes / (FETCH_SIZE*1024) (MI355X_MICROARCH.md: FETCH_SIZE counts "
                       "~1/2 of wide streaming reads on gfx950)",
        "calibration_factor": round(factor, 4), "kernel": "k_scan_q<4096, 2, true>", "fetch_size_kib_scan": fp,
        "scan_launches": len(p["FETCH_SIZE"]), "scan_read_bytes_corrected": int(fp * 1024 * factor),
        "traffic_per_input_byte": round(fp * 1024 * factor / n_cal, 4),
        "measured": f"gpurun_out/prof_{tag}/calib (tools/scanbench 8 prod vs quadread)"}
    json.dump(traffic, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)

    # ---- counter groups over tools/prof_workload.py --gib 16
    files = sorted(glob.glob(os.path.join(src, "pmc/p*/run_counter_collection.csv")))
    gib16 = 16 << 30
    kern = {}
    for name, match in (("k_scan_q<4096,2,true>", "k_scan_q<4096, 2, true>"), ("k_spec6", "k_spec6"),
                        ("k_emit", "k_emit<"), ("k_b3_leaves", "k_b3_leaves"), ("k_b3_tree", "k_b3_tree")):
        d = per_dispatch(files, match)
        m = {c: med(v) for c, v in d.items() if c != "duration_s"}
        e = {"counters_median_per_dispatch": m}
        if name.startswith("k_scan_q") and m.get("SQ_INSTS_VALU"):
            e["valu_instr_per_input_byte_per_lane"] = round(m["SQ_INSTS_VALU"] * 64 / gib16, 3)
            e["lds_instr_per_input_byte_per_lane"] = round(m["SQ_INSTS_LDS"] * 64 / gib16, 3)
            e["fetch_bytes_per_input_byte_calibrated"] = round(m["FETCH_SIZE"] * 1024 * factor / gib16, 4)
        if name == "k_b3_leaves" and m.get("SQ_INSTS_VALU"):
            e["valu_instr_per_64B_block_per_wave"] = round(m["SQ_INSTS_VALU"] * 64 / (gib16 / 64), 1)
            e["algorithmic_valu_per_block"] = 672
            e["fetch_bytes_per_input_byte_x2"] = round(m["FETCH_SIZE"] * 1024 * 2 / gib16, 3)
        if m.get("SQ_WAIT_INST_ANY") and m.get("SQ_WAVE_CYCLES"):
            e["wait_fraction_of_wave_cycles"] = round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        kern[name] = e
    json.dump({"workload": "tools/prof_workload.py --gib 16: 16 GiB uniform random, 16/64/256 KiB, 5 chunk calls "
                           "+ 3 chunk-ID calls; one counter group per rocprofv3 --pmc pass (tools/profile_round.sh)",
               "kernels": kern}, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)

    # ---- sealing kernels (tools/aead_pmc.sh: aead_bench 8 GiB, seal + open twice each)
    af = sorted(glob.glob(os.path.join(src, "aead_pmc/p*/run_counter_collection.csv")))
    blocks = (8 << 30) / 16
    aead = {}
    for name in ("k_aead_ctr", "k_aead_polyval", "k_aead_prep", "k_aead_tag"):
        d = per_dispatch(af, name)
        m = {c: med(v) for c, v in d.items() if c != "duration_s"}
        e = {"counters_median_per_dispatch": m, "dispatch_ms_median_under_pmc": round(med(d["duration_s"]) * 1e3, 3)}
        if name in ("k_aead_ctr", "k_aead_polyval") and m.get("SQ_INSTS_VALU"):
            e["valu_lane_ops_per_16B_block"] = round(m["SQ_INSTS_VALU"] * 64 / blocks, 1)
            e["lds_instr_per_16B_block_per_lane"] = round(m["SQ_INSTS_LDS"] * 64 / blocks, 1)
            e["lds_bank_conflict_fraction_of_lds_cycles"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 3)
            dur = med(d["duration_s"])
            e["lds_busy_fraction_per_cu_at_gui_clock"] = round(
                m["SQ_LDS_IDX_ACTIVE"] / 256 / (m["GRBM_GUI_ACTIVE"] / 8), 3)
            e["gui_clock_ghz_per_xcd"] = round(m["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9, 2)
        if m.get("SQ_WAIT_INST_ANY") and m.get("SQ_WAVE_CYCLES"):
            e["wait_fraction_of_wave_cycles"] = round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        aead[name] = e
    json.dump({"workload": "tools/aead_bench.py 8 1: the chunks of an 8 GiB device stream sealed and opened "
                           "(2 calls each per pass); counter groups in tools/aead_pmc.sh", "kernels": aead},
              open(os.path.join(dst, "aead_pmc.json"), "w"), indent=1)
    print(json.dumps({"traffic_per_input_byte": traffic["traffic_per_input_byte"],
                      "scan": {k: v for k, v in kern["k_scan_q<4096,2,true>"].items() if k != "counters_median_per_dispatch"},
                      "aead_ctr": {k: v for k, v in aead["k_aead_ctr"].items() if k != "counters_median_per_dispatch"},
                      "aead_polyval": {k: v for k, v in aead["k_aead_polyval"].items()
                                       if k != "counters_median_per_dispatch"}}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
