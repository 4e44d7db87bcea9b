"""Chunk IDs at mapache's own 512K/1M/8M parameters (and at 16/64/256 KiB for
comparison) over a device-resident stream; device time per call and the
k_b3_* split comes from rocprofv3 when run under it.
usage: python tools/b3bench512.py [GiB]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 16
n = int(gib * (1 << 30))
with _lib.Context(0, n) as ctx:
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, 0x6d61706163686521)
    for prm in ((524288, 1048576, 8388608, 1), (16384, 65536, 262144, 1)):
        p = _lib.params(*prm)
        cap = n // (p.min_size - 1) + 2
        d_out = ctx.device_alloc(cap * 24)
        k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
        d_ids = ctx.device_alloc(32 * k)
        ts = []
        for _ in range(4):
            t0 = time.perf_counter()
            ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)
            ts.append(time.perf_counter() - t0)
        dev = ctx.timing()["ids_ms"]
        print(f"params {prm[0] >> 10}K: {k} chunks, ids wall {min(ts) * 1e3:.2f} ms, device {dev:.2f} ms, "
              f"{n / (dev * 1e-3) / (1 << 30):.0f} GiB/s", flush=True)
        ctx.device_free(d_ids)
        ctx.device_free(d_out)
