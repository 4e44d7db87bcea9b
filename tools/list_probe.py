"""The configs[3] stand-in (80 000 log-normal files, 1.34 GB) chunked at
16/64/256 KiB with the flat scan (MCDC_RUN_LIST=0) and the list-mode scan
(=1), on a repeated layout and on alternating layouts (every call's plan new),
checked against each other (tools only, not part of the product).
Usage: python tools/list_probe.py [calls]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rng = np.random.default_rng(20251016)  # (bench.py small_files)
sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, 80000)).astype(np.uint64) + 1, 64 << 20)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
n = int(sizes.sum())
p = _lib.params(16384, 65536, 262144, 1)
ref = None
for mode in ("0", "1"):
    os.environ["MCDC_RUN_LIST"] = mode
    with _lib.Context(0, 2 << 30) as ctx:
        arena = ctx.device_alloc(n + 64)
        ctx.fill_random(arena, n + 48, 99)
        cap = int(sum(int(s) // (p.min_size - 1) + 2 for s in sizes))
        d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
        for layout in ("repeated", "alternating"):
            wall, dev, scan, pre = [], [], [], []
            for c in range(calls + 2):
                o = offs + np.uint64(16 * (c % 2)) if layout == "alternating" else offs
                t0 = time.perf_counter()
                total, counts = ctx.chunk_batch_device_to_device(p, arena, o, sizes, d_out, cap)
                dt = time.perf_counter() - t0
                t = ctx.timing()
                if c >= 2:
                    wall.append(dt * 1e3), dev.append(t["device_ms"]), scan.append(t["scan_ms"]), pre.append(t["host_pre_ms"])
                if layout == "repeated" and c == 0:
                    g = ctx.d2h_chunks(d_out, total)
                    if ref is None:
                        ref = g
                    else:
                        same = len(g) == len(ref) and bool((g == ref).all())
                        print(f"list mode output identical to the flat scan's: {same}", flush=True)
            med = lambda x: float(np.median(x))  # noqa: E731
            print(f"MCDC_RUN_LIST={mode} {layout:11s} wall {med(wall):.3f} ms (min {min(wall):.3f})  device "
                  f"{med(dev):.3f}  scan {med(scan):.3f}  host_pre {med(pre):.3f}  -> {n / med(wall) / 1e-3 / 2**30:.0f} GiB/s",
                  flush=True)
        ctx.device_free(d_out)
        ctx.device_free(arena)
