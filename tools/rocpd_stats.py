"""Kernel statistics and a CSV kernel trace from a rocprofv3 rocpd database
(`rocprofv3 --kernel-trace` without --output-format csv writes one; tools
only).  usage: python tools/rocpd_stats.py <results.db> [--csv trace.csv] [--top N]"""
import argparse
import collections
import csv
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None, help="write a kernel trace CSV (Kernel_Name, Start/End_Timestamp)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = list(c.execute(f"select {name}, start, end from kernels order by start"))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
            w.writerows(rows)
    st = collections.defaultdict(list)
    for n, s, e in rows:
        st[n].append(e - s)
    tot = sum(sum(v) for v in st.values())
    print(f"{'kernel':60s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'max_us':>9s} {'%':>6s}")
    for n, v in sorted(st.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        m = re.search(r"(k_\w+(<[^>]*>)?|\w*Scan\w*|\w*Kernel\w*|__amd\w+)", n)
        print(f"{(m.group(1) if m else n)[:60]:60s} {len(v):6d} {sum(v) / 1e3:10.1f} {sum(v) / len(v) / 1e3:9.1f} "
              f"{max(v) / 1e3:9.1f} {100 * sum(v) / tot:6.2f}")


if __name__ == "__main__":
    main()
