"""Scan / device / call time per lane-piece count (MCDC_SCAN_PIECES) on the
configs[3] small-file stand-in (80 000 files, 1.34 GB) and on one-file calls of
0.5-6 GiB.  Probe for choosing the scan_pieces rule; not part of the product."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

rng = np.random.default_rng(20251016)
sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, 80000)).astype(np.uint64) + 1, 64 << 20)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
nsmall = int(sizes.sum())
p = _lib.params(16384, 65536, 262144, 1)
NMAX = 6 << 30
with _lib.Context(0, NMAX) as ctx:
    arena = ctx.device_alloc(NMAX + 16)
    ctx.fill_random(arena, NMAX, 99)
    cap = NMAX // (p.min_size - 1) + 100000
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    cases = [("80k files", offs, sizes)] + [(f"{g} GiB", np.zeros(1, np.uint64), np.array([int(g * (1 << 30))], np.uint64))
                                            for g in (0.5, 1, 1.5, 2, 3, 4, 6)]
    for name, o, l in cases:
        for rep in range(2):
            for pc in (1, 2, 4):
                os.environ["MCDC_SCAN_PIECES"] = str(pc)
                sc, dv, tt = [], [], []
                for _ in range(6):
                    ctx.chunk_batch_device_to_device(p, arena, o, l, d_out, cap)
                    t = ctx.timing()
                    sc.append(t["scan_ms"]); dv.append(t["device_ms"]); tt.append(t["total_ms"])
                print(f"{name:10s} pieces {pc}  scan {np.median(sc[1:]):.3f} ms  device {np.median(dv[1:]):.3f} ms  "
                      f"call {np.median(tt[1:]):.3f} ms", flush=True)
