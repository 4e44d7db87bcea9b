"""Summarise the compressor's PMC passes (tools/gpu_round4.sh <tag> zcprof:
tools/zc_bench.py 1 GiB of text, one rocprofv3 --pmc pass per counter group)
into per-kernel medians per dispatch and derived rates.
Usage: python tools/zc_pmc_summary.py <tag> [out.json]"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_zc_find", "k_zc_parse", "k_zc_huff", "k_zc_plan", "k_zc_chain", "k_zc_encode", "k_zc_final")


def main(tag, out=None):
    acc, dur = defaultdict(lambda: defaultdict(float)), {}
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "zc_pmc", "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = next((x for x in KERNELS if x in r["Kernel_Name"]), None)
            if not k:
                continue
            key = (k, f, r["Dispatch_Id"])
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    res = {}
    for k in KERNELS:
        per = defaultdict(list)
        ds = []
        for key, cs in acc.items():
            if key[0] != k:
                continue
            for c, v in cs.items():
                per[c].append(v)
            ds.append(dur[key])
        if not per:
            continue
        m = {c: statistics.median(v) for c, v in per.items()}
        e = {"counters_median_per_dispatch": m, "dispatch_ms_median_under_pmc": round(statistics.median(ds) * 1e3, 3)}
        # bytes per dispatch: each pass runs tools/zc_bench.py 1 1 text = one
        # warm-up + one timed call over 1 GiB; a kernel's dispatches per pass
        # are the batches of those two calls
        per_pass = defaultdict(int)
        for key in acc:
            if key[0] == k:
                per_pass[key[1]] += 1
        batch = 2 * (1 << 30) / statistics.median(per_pass.values())
        e["input_bytes_per_dispatch"] = int(batch)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
            if c in m:
                e[c.lower() + "_per_input_byte"] = round(m[c] / batch, 3)
        if m.get("SQ_WAIT_ANY") and m.get("SQ_WAVE_CYCLES"):
            e["wait_fraction_of_wave_cycles"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_cycles_per_lds_active"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 3)
        if m.get("SQ_INSTS_LDS"):
            e["lds_bank_conflict_cycles_per_lds_instr"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"], 3)
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM"):
            if c in m and m.get("SQ_WAVE_CYCLES"):
                e[c.lower() + "_per_wave_cycle"] = round(m[c] / m["SQ_WAVE_CYCLES"], 3)
        if "VALUBusy" in m:
            e["valu_busy_pct"] = round(m["VALUBusy"], 2)
        if "FETCH_SIZE" in m:
            e["fetch_bytes_x2_per_input_byte"] = round(m["FETCH_SIZE"] * 1024 * 2 / batch, 3)
        if "WRITE_SIZE" in m:
            e["write_bytes_per_input_byte"] = round(m["WRITE_SIZE"] * 1024 / batch, 3)
        res[k] = e
    doc = {"workload": "tools/zc_bench.py 1 1 text (1 GiB of text in 16/64/256 KiB chunks; per-byte rates over each dispatch's share of the input); "
                       "one counter group per rocprofv3 --pmc pass (tools/gpu_round4.sh zcprof)",
           "source": f"gpurun_out/{tag}/zc_pmc", "kernels": res}
    if out:
        os.makedirs(os.path.dirname(os.path.join(ROOT, out)), exist_ok=True)
        json.dump(doc, open(os.path.join(ROOT, out), "w"), indent=1)
    for k, e in res.items():
        print(k, {x: y for x, y in e.items() if x != "counters_median_per_dispatch"})


if __name__ == "__main__":
    main(*sys.argv[1:])
