"""One call's kernels from a rocprofv3 kernel trace, in launch order, with the
gap before each (tools only).  Calls are split where the device is idle for
more than --split microseconds.

usage: python tools/calltrace.py <kernel_trace.csv> [--split US] [--call K] [--summary]
  --call K    print call K's kernels (default: the last call)
  --summary   one line per call: device span, busy time, kernels, largest kernels"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    m = re.search(r"(k_\w+|\w*Scan\w*|\w*Kernel\w*)", name)
    return (m.group(1) if m else name)[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split", type=float, default=200.0)
    ap.add_argument("--call", type=int, default=-1)
    ap.add_argument("--summary", action="store_true")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur, end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if end is not None and s - end > a.split * 1e3:
            calls.append(cur)
            cur = []
        cur.append((short(r["Kernel_Name"]), s, e))
        end = e if end is None else max(end, e)
    if cur:
        calls.append(cur)
    if a.summary:
        prev_end = None
        for i, c in enumerate(calls):
            t0, t1 = c[0][1], max(x[2] for x in c)
            gap = (t0 - prev_end) / 1e3 if prev_end is not None else 0.0
            prev_end = t1
            per = collections.Counter()
            for k, s, e in c:
                per[k] += (e - s) / 1e3
            top = ", ".join(f"{k} {v:.0f}" for k, v in per.most_common(4))
            print(f"call {i:3d}: gap {gap:9.1f} us  span {(t1 - t0) / 1e3:9.1f} us  kernels {len(c):4d}  {top}")
        return
    c = calls[a.call]
    t0, prev = c[0][1], c[0][1]
    busy = collections.Counter()
    for k, s, e in c:
        print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev) / 1e3:7.1f}  {k:40s} {(e - s) / 1e3:8.1f} us")
        prev = max(prev, e)
        busy[k] += (e - s) / 1e3
    print(f"span {(max(x[2] for x in c) - t0) / 1e3:.1f} us, {len(c)} kernels")
    for k, v in busy.most_common(8):
        print(f"  {k:40s} {v:8.1f} us")


if __name__ == "__main__":
    main()
