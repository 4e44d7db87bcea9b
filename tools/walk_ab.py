"""A/B of the chain walks on one box: python tools/walk_ab.py GiB [reps] [env=val ...]
Each setting of MCDC_LANE_WALK (0: group walk, 1: the default) runs in its own
subprocess: 2 warm-up + 9 timed device-resident calls (boundary list in HBM)
of the synthetic stream at 16/64/256 KiB; prints the median scan / resolve /
device ms and every call's resolve ms, alternating settings (ABAB).  Extra
env=val arguments apply to both."""
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
cap = n // (p.min_size - 1) + 2
d_out = ctx.device_alloc(cap * 24)
rows, k = [], 0
for i in range(11):
    k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
    t = ctx.timing()
    if i >= 2:
        rows.append((t["scan_ms"], t["resolve_ms"], t["device_ms"], t["total_ms"]))
med = [float(np.median([r[j] for r in rows])) for j in range(4)]
print(json.dumps({"chunks": int(k), "lane_walk": int(t["lane_walk"]), "handed_back": int(t["handed_back"]),
                  "scan": round(med[0], 3), "resolve": round(med[1], 3), "device": round(med[2], 3),
                  "call": round(med[3], 3), "resolve_all": [round(r[1], 3) for r in rows]}))
'''

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
gib = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
extra = dict(kv.split("=", 1) for kv in sys.argv[3:])
for rep in range(reps):
    for walk in ("0", "1"):
        env = dict(os.environ, MCDC_LANE_WALK=walk, **extra)
        r = subprocess.run([sys.executable, "-c", CHILD, gib, root], env=env, capture_output=True, text=True,
                           timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-400:]
        print(f"walk={walk} {line}", flush=True)
        if r.returncode != 0:
            sys.exit(1)
