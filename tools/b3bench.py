"""Chunk-ID (BLAKE3) kernel microbenchmark: chunk a device-resident random
buffer once (P16), then time mcdc_chunk_ids_device over its boundary list.
usage: python tools/b3bench.py [GiB] [reps]   (MCDC_LIBRARY selects a build;
the digest of all IDs lets builds be compared)"""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = int(gib * (1 << 30))
p = _lib.params(16384, 65536, 262144, 1)
with _lib.Context(0, n) as ctx:
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, 0x6d61706163686521)
    cap = n // (p.min_size - 1) + 2
    d_out = ctx.device_alloc(cap * 24)
    k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
    d_ids = ctx.device_alloc(32 * k)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)
        ts.append(time.perf_counter() - t0)
        dev = ctx.timing()["ids_ms"]
    best = min(ts)
    dig = hashlib.sha256(ctx.d2h_bytes(d_ids, 32 * k).tobytes()).hexdigest()[:16]
    print(f"{os.path.basename(_lib.LIB_PATH)}  ids {dig}  chunks {k}  wall best {best*1e3:.3f} ms  device {dev:.3f} ms  {n/best/1e12:.3f} TB/s  "
          f"{n/(dev*1e-3)/1e12:.3f} TB/s device", flush=True)
