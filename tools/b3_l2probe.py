"""Chunk-ID kernel: HBM-streaming vs L2-resident input, same work (probe, not
part of the product).  1 M chunks of 16 KiB: distinct offsets (16 GiB read
from HBM) vs offsets cycling over a 2 MiB region (L2-resident).
usage: python tools/b3_l2probe.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

N = 1 << 20
L = 16 << 10
with _lib.Context(0, N * L) as ctx:
    dp = ctx.device_alloc(N * L)
    ctx.fill_random(dp, N * L, 7)

    for name, offs in (("hbm", np.arange(N, dtype=np.uint64) * L),
                       ("l2", (np.arange(N, dtype=np.uint64) % 128) * L),
                       ("hbm", np.arange(N, dtype=np.uint64) * L)):
        ch = np.zeros(N, dtype=_lib.CHUNK_DTYPE)
        ch["offset"] = offs
        ch["length"] = L
        best = 1e9
        for _ in range(4):
            t0 = time.perf_counter()
            ctx.chunk_ids(dp, N * L, ch)
            best = min(best, time.perf_counter() - t0)
        t = ctx.timing()
        print(f"{name}: best call {best*1e3:.3f} ms, ids kernels {t['ids_ms']:.3f} ms, "
              f"{N * L / t['ids_ms'] / 1e9:.2f} TB/s", flush=True)
    ctx.device_free(dp)
