"""Where the configs[3] stand-in call (80 000 device-resident files) spends
its time: Python wall clock vs the library's total, device and D2H times.
Probe; not part of the product."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

rng = np.random.default_rng(20251016)
sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, 80000)).astype(np.uint64) + 1, 64 << 20)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
n = int(sizes.sum())
p = _lib.params(16384, 65536, 262144, 1)
with _lib.Context(0, 2 << 30) as ctx:
    arena = ctx.device_alloc(n + 16)
    ctx.fill_random(arena, n, 99)
    cap = int(sum(int(s) // (p.min_size - 1) + 2 for s in sizes))
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    for rep in range(3):
        rows = []
        for _ in range(8):
            t0 = time.perf_counter()
            ctx.chunk_batch_device_to_device(p, arena, offs, sizes, d_out, cap)
            wall = (time.perf_counter() - t0) * 1e3
            t = ctx.timing()
            rows.append((wall, t["total_ms"], t["device_ms"], t["scan_ms"], t["d2h_ms"]))
        m = np.median(np.array(rows[1:]), axis=0)
        print("wall %.3f  lib total %.3f  device %.3f  scan %.3f  d2h(wait+copies) %.3f ms" % tuple(m), flush=True)
