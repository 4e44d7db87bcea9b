"""Summarise rocprofv3 --pmc CSV passes: median per counter for kernels matching a pattern."""
import csv, glob, os, sys, collections
root, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_scan"
for mode in sorted(os.listdir(root)):
    d = os.path.join(root, mode)
    if not os.path.isdir(d):
        continue
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {mode}")
    for k in sorted(agg):
        v = sorted(agg[k])
        print(f"  {k:28s} {v[len(v)//2]:.4g}")
