"""Scan kernel time vs input size (probe; not part of the product)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

p = _lib.params(16384, 65536, 262144, 1)
N = 16 << 30
with _lib.Context(0, N) as ctx:
    dp = ctx.device_alloc(N)
    ctx.fill_random(dp, N, 5)
    d_out = ctx.device_alloc((N // 16383 + 2) * 24)
    for mib in (64, 256, 1024, 1280, 2048, 4096, 8192, 16384):
        n = mib << 20
        best = None
        for _ in range(5):
            ctx.chunk_device_to_device(p, dp, n, d_out, N // 16383 + 2)
            t = ctx.timing()
            best = t if best is None or t["scan_ms"] < best["scan_ms"] else best
        print(f"{mib:6d} MiB  scan {best['scan_ms']:.3f} ms  {n / best['scan_ms'] / 1e9:.2f} TB/s  device {best['device_ms']:.3f}",
              flush=True)
