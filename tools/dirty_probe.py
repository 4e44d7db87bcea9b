"""Which resolution path the configs[3]-like call takes per segment size:
library timing fields (fallback files, device/scan times) for MCDC_SEG_CHUNKS
in 12/16/24, same arena as tools/pieces_big.py.  Probe; not part of the product."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

rng = np.random.default_rng(20251016)
sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, 80000)).astype(np.uint64) + 1, 64 << 20)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
n = int(sizes.sum())
print("files > 1.25 MiB:", int((sizes > 1310720).sum()), "largest", int(sizes.max()), flush=True)
p = _lib.params(16384, 65536, 262144, 1)
with _lib.Context(0, 2 << 30) as ctx:
    arena = ctx.device_alloc(n + 16)
    ctx.fill_random(arena, n, int(os.environ.get("SEEDX", str(0x6d61706163686521)), 0))
    cap = n // (p.min_size - 1) + 100000
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    for k in ("12", "16", "24"):
        os.environ["MCDC_SEG_CHUNKS"] = k
        for _ in range(3):
            ctx.chunk_batch_device_to_device(p, arena, offs, sizes, d_out, cap)
        print(k, ctx.timing(), flush=True)
