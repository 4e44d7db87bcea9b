"""PCIe probe (GPU box): H2D from pinned host memory through the library, and
the end-to-end host entry point, at a few sizes."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from mapache_amd import _lib  # noqa: E402

L = _lib.load()
for gib in (1, 4, 8):
    n = gib << 30
    with _lib.Context(0, n) as ctx:
        hp = ctx.host_alloc(n)
        dp = ctx.device_alloc(n)
        ctx.fill_random(dp, n, 7)
        _lib.check(L.mcdc_memcpy_d2h(ctx._h, ctypes.c_void_p(hp), ctypes.c_void_p(dp), n))
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            _lib.check(L.mcdc_memcpy_h2d(ctx._h, ctypes.c_void_p(dp), ctypes.c_void_p(hp), n))
            ts.append(time.perf_counter() - t0)
        p = _lib.params(16384, 65536, 262144, 1)
        out = np.zeros(n // 16383 + 2, dtype=_lib.CHUNK_DTYPE)
        k = ctypes.c_size_t()
        te = []
        for _ in range(2):
            t0 = time.perf_counter()
            _lib.check(L.mcdc_chunk_host(ctx._h, ctypes.byref(p), ctypes.c_void_p(hp), n, out.ctypes.data, out.size,
                                         ctypes.byref(k)))
            te.append(time.perf_counter() - t0)
        t = ctx.timing()
        print(f"{gib} GiB: h2d {n / min(ts) / 1e9:.1f} GB/s  chunk_host {n / min(te) / 1e9:.1f} GB/s "
              f"(h2d_ms {t['h2d_ms']:.1f} device {t['device_ms']:.2f})", flush=True)
        ctx.host_free(hp)
        ctx.device_free(dp)
