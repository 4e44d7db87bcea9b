"""Summarise the compressor's PMC passes (tools/gpu_round4.sh <tag> zcprof:
tools/zc_bench.py 1 GiB of text, one rocprofv3 --pmc pass per counter group)
into per-kernel totals per pass and derived per-input-byte rates.
Usage: python tools/zc_pmc_summary.py <tag> [out.json]"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_zc_nblocks", "k_zc_blocks", "k_zc_segorder", "k_zc_probe", "k_zc_small", "k_zc_far", "k_zc_find",
           "k_zc_parse", "k_zc_huff", "k_zc_plan", "k_zc_chain", "k_zc_encode", "k_zc_final")


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
    # Per-byte rates over the whole input: each counter is collected in one
    # pass (tools/zc_bench.py 1 1 text: a warm-up and a timed call, 2 GiB in
    # all), so a counter's sum over the kernel's dispatches in that pass,
    # divided by the 2 GiB, is exact -- the dispatches are unequal (two full
    # batch sets and a remainder), and dividing one dispatch's counters by the
    # mean input per dispatch (round 5) biased every rate.
    pass_bytes = 2 * (1 << 30)
    for k in KERNELS:
        tot, ds, nd = defaultdict(float), [], defaultdict(int)
        for key, cs in acc.items():
            if key[0] != k:
                continue
            for c, v in cs.items():
                tot[c] += v
            ds.append(dur[key])
            nd[key[1]] += 1
        if not tot:
            continue
        m = dict(tot)
        e = {"counters_total_per_pass": m, "dispatches_per_pass": max(nd.values()),
             "dispatch_ms_median_under_pmc": round(statistics.median(ds) * 1e3, 3),
             "kernel_ms_per_pass_under_pmc": round(sum(ds) / max(1, len(nd)) * 1e3, 3),
             "input_bytes_per_pass": pass_bytes}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
            if c in m:
                e[c.lower() + "_per_input_byte"] = round(m[c] / pass_bytes, 3)
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
        if "VALUBusy" in m:  # (a percentage per dispatch: its median, not a sum)
            vb = [cs["VALUBusy"] for key, cs in acc.items() if key[0] == k and "VALUBusy" in cs]
            e["valu_busy_pct_median"] = round(statistics.median(vb), 2)
            del m["VALUBusy"]
        if "FETCH_SIZE" in m:  # (KiB; x2: gfx950 undercounts 16-byte-per-lane reads, MI355X_MICROARCH.md)
            e["fetch_bytes_x2_per_input_byte"] = round(m["FETCH_SIZE"] * 1024 * 2 / pass_bytes, 3)
        if "WRITE_SIZE" in m:
            e["write_bytes_per_input_byte"] = round(m["WRITE_SIZE"] * 1024 / pass_bytes, 3)
        res[k] = e
    doc = {"workload": "tools/zc_bench.py 1 1 text (1 GiB of text in 16/64/256 KiB chunks, a warm-up and a timed call per pass); per-byte rates: each counter summed over the kernel's dispatches of its pass / the pass's 2 GiB; "
                       "one counter group per rocprofv3 --pmc pass (tools/gpu_round4.sh zcprof)",
           "source": f"gpurun_out/{tag}/zc_pmc", "kernels": res}
    if out:
        os.makedirs(os.path.dirname(os.path.join(ROOT, out)), exist_ok=True)
        json.dump(doc, open(os.path.join(ROOT, out), "w"), indent=1)
    for k, e in res.items():
        print(k, {x: y for x, y in e.items() if x != "counters_total_per_pass"})


if __name__ == "__main__":
    main(*sys.argv[1:])
