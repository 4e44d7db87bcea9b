"""Per-kernel summary of a rocprofv3 --stats CSV (tools/kcsv.py <kernel_stats.csv> [top])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for r in rows[:top]:
    print(f"{r['Name'][:70]:70s} n={int(r['Calls']):5d} avg={float(r['AverageNs']) / 1e6:9.3f} ms "
          f"total={float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['Percentage']):5.1f}%")
