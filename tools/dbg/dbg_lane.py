import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mapache_amd import _lib
n = int(float(os.environ.get("GIB", "64")) * (1 << 30))
p = _lib.params(16384, 65536, 262144, 1)
ctx = _lib.Context(0, n)
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, 0x6d61706163686521)
cap = n // (p.min_size - 1) + 2
d_out = ctx.device_alloc(cap * 24)
for i in range(6):
    k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
    t = ctx.timing()
    print(os.environ.get("MCDC_DBG_LANE"), "resolve", round(t["resolve_ms"], 3), "scan", round(t["scan_ms"], 3), flush=True)
