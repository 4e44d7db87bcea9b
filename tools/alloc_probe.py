"""Does the GPU save path's speed depend on what the process allocated and
freed before?  (GPU box; tools only.)  The kernel-tree stand-in through
mcdc_save_files on a fresh context, then again on a context created after
multi-GiB device buffers were allocated, written and freed (as bench.py's
legs do before its kernel_tree leg), with the input arena and the pinned
output allocated before or after the frees.
Usage: python tools/alloc_probe.py [GiB to allocate and free]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402
from tests import corpora  # noqa: E402

gib = int(sys.argv[1]) if len(sys.argv) > 1 else 120
data, offs, lens, dup = corpora.kernel_tree(80000)
n = int(data.size)
p = _lib.params(512 << 10, 1 << 20, 8 << 20, 1)
rng = np.random.default_rng(9)
nonces = rng.integers(0, 256, (80000 + n // (512 << 10) + 64, 12), dtype=np.uint8)
hn, pad = rng.integers(0, 256, (4096, 12), dtype=np.uint8), rng.integers(0, 256, (4096 * 63, 36), dtype=np.uint8)


def alloc(ctx):
    dp = ctx.device_alloc(n + 16)
    ctx.h2d(dp, data)
    return dp, ctx.pinned_bytes(int(n * 1.01) + 4096 * 80000 + (1 << 16))


def run(ctx, tag, dp, ob):
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        with ctx.index_create() as ix:
            ctx.save_files(p, ix, dp, offs, lens, bytes(range(32)), nonces, hn, pad, n=n, gpu_compress=True,
                           out_buf=ob, split=False)
        ts.append(time.perf_counter() - t0)
    print(f"{tag:52s} {np.median(ts[1:]) * 1e3:6.1f} ms (min {min(ts[1:]) * 1e3:.1f})", flush=True)


with _lib.Context(0, 4 << 30) as ctx:
    dp0, ob0 = alloc(ctx)
    run(ctx, "fresh context, input and output before the frees", dp0, ob0)
    bufs = []
    for _ in range(gib // 32):
        b = ctx.device_alloc(32 << 30)
        ctx.fill_random(b, 32 << 30, 5)
        bufs.append(b)
    ctx.synchronize()
    for b in bufs:
        ctx.device_free(b)
    print(f"(allocated, wrote and freed {len(bufs) * 32} GiB)", flush=True)
    run(ctx, "same input and output", dp0, ob0)
    dp1, ob1 = alloc(ctx)
    run(ctx, "input device buffer allocated after the frees", dp1, ob0)
    run(ctx, "output pinned buffer allocated after the frees", dp0, ob1)
    run(ctx, "both allocated after the frees", dp1, ob1)
    with _lib.Context(0, 4 << 30) as ctx2:
        run(ctx2, "a context created after the frees, old buffers", dp0, ob0)
