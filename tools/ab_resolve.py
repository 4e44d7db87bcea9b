"""A/B timing of libmcdc variants on one box: python tools/ab_resolve.py GiB lib1 [lib2 ...]
Each library runs in its own subprocess (MCDC_LIBRARY), 2 warmups + 7 timed calls,
medians of scan / resolve / device / call ms printed per library, twice (ABAB)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, numpy as np
sys.path.insert(0, sys.argv[2])
from mapache_amd import _lib
n = int(float(sys.argv[1]) * (1 << 30))
p = _lib.params(16384, 65536, 262144, 1)
ctx = _lib.Context(0, n)
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, 0x6d61706163686521)
out = ctx.pinned_out(n // (p.min_size - 1) + 2)
rows = []
for i in range(9):
    ch = ctx.chunk_device(p, dp, n, out=out)
    t = ctx.timing()
    if i >= 2:
        rows.append((t["scan_ms"], t["resolve_ms"], t["device_ms"], t["total_ms"]))
med = [float(np.median([r[k] for r in rows])) for k in range(4)]
print(json.dumps({"chunks": int(len(ch)), "scan": med[0], "resolve": med[1], "device": med[2], "call": med[3]}))
'''

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
gib, libs = sys.argv[1], sys.argv[2:]
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for lib in libs:
        env = dict(os.environ, MCDC_LIBRARY=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", CHILD, gib, root], env=env, capture_output=True, text=True,
                           timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-400:]
        print(f"{os.path.basename(lib):24s} {line}", flush=True)
        if r.returncode != 0:
            sys.exit(1)
