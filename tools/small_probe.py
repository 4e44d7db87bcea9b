"""Scan time of one 1.34 GB arena chunked as one file vs as 80 000 files
(probe for the configs[3] stand-in; not part of the product)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

rng = np.random.default_rng(20251016)
sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, 80000)).astype(np.uint64) + 1, 64 << 20)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
n = int(sizes.sum())
p = _lib.params(16384, 65536, 262144, 1)
with _lib.Context(0, 2 << 30) as ctx:
    arena = ctx.device_alloc(n + 16)
    ctx.fill_random(arena, n, 99)
    cap = int(sum(int(s) // (p.min_size - 1) + 2 for s in sizes))
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    for rep in range(3):
        for name, (o, l) in (("one file", (np.zeros(1, np.uint64), np.array([n], np.uint64))),
                             ("80k files", (offs, sizes))):
            for _ in range(3):
                ctx.chunk_batch_device_to_device(p, arena, o, l, d_out, cap)
            t = ctx.timing()
            print(f"{name:10s} scan {t['scan_ms']:.3f} ms  device {t['device_ms']:.3f} ms  call {t['total_ms']:.3f} ms"
                  f"  host pre {t['host_pre_ms']:.3f} post {t['host_post_ms']:.3f} ms", flush=True)
