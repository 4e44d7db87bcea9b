"""Which preceding state slows the e2e host path in bench.py? (GPU box)"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from mapache_amd import _lib  # noqa: E402

L = _lib.load()
p = _lib.params(16384, 65536, 262144, 1)


def e2e(ctx, tag, gib=8):
    n = gib << 30
    hp = ctx.host_alloc(n)
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, 7)
    _lib.check(L.mcdc_memcpy_d2h(ctx._h, ctypes.c_void_p(hp), ctypes.c_void_p(dp), n))
    out = np.zeros(n // 16383 + 2, dtype=_lib.CHUNK_DTYPE)
    k = ctypes.c_size_t()
    best = 1e9
    for _ in range(2):
        t0 = time.perf_counter()
        _lib.check(L.mcdc_chunk_host(ctx._h, ctypes.byref(p), ctypes.c_void_p(hp), n, out.ctypes.data, out.size,
                                     ctypes.byref(k)))
        best = min(best, time.perf_counter() - t0)
    t0 = time.perf_counter()
    _lib.check(L.mcdc_memcpy_h2d(ctx._h, ctypes.c_void_p(dp), ctypes.c_void_p(hp), n))
    raw = time.perf_counter() - t0
    print(f"{tag:40s} chunk_host {n / best / 1e9:5.1f} GB/s  raw h2d {n / raw / 1e9:5.1f} GB/s", flush=True)
    ctx.host_free(hp)
    ctx.device_free(dp)


N = 64 << 30
with _lib.Context(0, N) as ctx:
    e2e(ctx, "fresh ctx(64 GiB)")
    big = ctx.device_alloc(N)
    ctx.fill_random(big, N, 1)
    e2e(ctx, "64 GiB buffer allocated")
    cap = N // 16383 + 2
    d_out = ctx.device_alloc(cap * 24)
    ctx.chunk_device_to_device(p, big, N, d_out, cap)
    e2e(ctx, "after a 64 GiB chunk call")
    ctx.device_free(d_out)
    ctx.device_free(big)
    e2e(ctx, "after freeing them")
