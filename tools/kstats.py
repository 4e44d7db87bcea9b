"""Per-kernel duration summary of a rocprofv3 --kernel-trace database
(tools/kstats.py <dir-or-db> [top]); also writes <db>.kernel_stats.csv."""
import glob
import os
import sqlite3
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
rows = list(c.execute(f"select s.kernel_name, count(*), avg(d.end-d.start)/1e6, sum(d.end-d.start)/1e6, "
                      f"min(d.end-d.start)/1e6, max(d.end-d.start)/1e6 from {kd} d join {ks} s on d.kernel_id=s.id "
                      f"group by s.kernel_name order by 4 desc"))
with open(db + ".kernel_stats.csv", "w") as f:
    f.write("Name,Calls,AverageMs,TotalMs,MinMs,MaxMs\n")
    for r in rows:
        f.write(f'"{r[0]}",{r[1]},{r[2]:.6f},{r[3]:.6f},{r[4]:.6f},{r[5]:.6f}\n')
for r in rows[:top]:
    print(f"{r[0][:72]:72s} n={r[1]:4d} avg={r[2]:9.3f} ms  total={r[3]:9.2f}")
