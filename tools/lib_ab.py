"""Scan / device time of one library build (path in argv[1]) on 16 and 64 GiB
one-file calls; run alternately with two builds for a compile-time A/B.
Probe; not part of the product."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
p = _lib.params(16384, 65536, 262144, 1)
NMAX = 64 << 30
with _lib.Context(0, NMAX) as ctx:
    arena = ctx.device_alloc(NMAX + 16)
    ctx.fill_random(arena, NMAX, 0x6d61706163686521)
    cap = NMAX // (p.min_size - 1) + 100000
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    for g in (16, 64):
        n = g << 30
        sc, dv = [], []
        for _ in range(7):
            ctx.chunk_batch_device_to_device(p, arena, np.zeros(1, np.uint64), np.array([n], np.uint64), d_out, cap)
            t = ctx.timing()
            sc.append(t["scan_ms"]); dv.append(t["device_ms"])
        print(f"{os.path.basename(sys.argv[1]):20s} {g} GiB  scan {np.median(sc[1:]):.3f} ms  device {np.median(dv[1:]):.3f} ms",
              flush=True)
