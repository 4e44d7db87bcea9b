"""Device time per scan configuration on one-file calls of 0.5-64 GiB and on
the configs[3] small-file stand-in, ABAB: lane pieces per run
(MCDC_SCAN_PIECES 1 / 2 / 0 = the library's rule) and each wave's first tile
static (MCDC_FIRST_STATIC).  Probe for the scan_pieces rule; not part of the
product."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

p = _lib.params(16384, 65536, 262144, 1)
NMAX = 64 << 30
rng = np.random.default_rng(20251016)
sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, 80000)).astype(np.uint64) + 1, 64 << 20)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
CONFIGS = [(a, b) for a, b in (v.split(":") for v in os.environ.get("AB", "1:0,1:1,2:0,2:1,0:1").split(","))]
KNOB = os.environ.get("AB_KNOB", "MCDC_FIRST_STATIC")
with _lib.Context(0, NMAX) as ctx:
    arena = ctx.device_alloc(NMAX + 16)
    ctx.fill_random(arena, NMAX, 0x6d61706163686521)
    cap = NMAX // (p.min_size - 1) + 100000
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    cases = [("80k files", offs, sizes)] + [(f"{g} GiB", np.zeros(1, np.uint64), np.array([int(g * 2**30)], np.uint64))
                                            for g in map(float, os.environ.get("AB_GIB", "0.25,0.5,1,2,16,64").split(","))]
    for name, o, l in cases:
        n = int(l.sum())
        for rep in range(2):
            for pc, fs in CONFIGS:
                os.environ["MCDC_SCAN_PIECES"] = pc
                os.environ[KNOB] = fs
                sc, dv = [], []
                for _ in range(5 if n > 8 << 30 else 9):
                    ctx.chunk_batch_device_to_device(p, arena, o, l, d_out, cap)
                    t = ctx.timing()
                    sc.append(t["scan_ms"]); dv.append(t["device_ms"])
                print(f"{name:9s} pieces {pc} {KNOB} {fs}  scan {np.median(sc[1:]):.3f} ms  device "
                      f"{np.median(dv[1:]):.3f} ms  -> {n / 2**30 / np.median(dv[1:]) * 1e3:.0f} GiB/s", flush=True)
