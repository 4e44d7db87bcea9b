"""Per-batch kernel times of the GPU compressor from a rocprofv3 kernel
trace (tools/ztrace.py <kernel_trace.csv>): one line per batch (a batch
starts at k_zc_blocks), microseconds per kernel, in launch order."""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
batches, cur = [], None
for r in rows:
    m = re.search(r"(k_zc_\w+)", r["Kernel_Name"])
    if not m:
        continue
    k, d = m.group(1)[5:], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k == "blocks":
        cur = collections.OrderedDict()
        batches.append(cur)
    if cur is not None:
        cur[k] = cur.get(k, 0) + d
for i, b in enumerate(batches):
    print(f"{i:3d} sum={sum(b.values()):7.0f} " + " ".join(f"{k}={v:.0f}" for k, v in b.items()))
