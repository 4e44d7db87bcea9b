"""The configs[3] kernel-tree stand-in through mcdc_save_files (P512, gate,
key, GPU compression), a few calls, for a kernel trace of what bounds it
(tools only).  Usage: python tools/tree_probe.py [files] [calls] [modes: gpu | host | host,gpu]
(TREE_FREE_HSAVE=1: release the context's pinned host staging between the modes)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402
from tests import corpora  # noqa: E402

nfiles = int(sys.argv[1]) if len(sys.argv) > 1 else 80000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
modes = (sys.argv[3] if len(sys.argv) > 3 else "gpu").split(",")
data, offs, lens, dup = corpora.kernel_tree(nfiles)
n = int(data.size)
p = _lib.params(512 << 10, 1 << 20, 8 << 20, 1)
rng = np.random.default_rng(9)
nonces = rng.integers(0, 256, (nfiles + n // (512 << 10) + 64, 12), dtype=np.uint8)
hn, pad = rng.integers(0, 256, (4096, 12), dtype=np.uint8), rng.integers(0, 256, (4096 * 63, 36), dtype=np.uint8)
with _lib.Context(0, 2 << 30) as ctx:
    for kv in os.environ.get("ZC_OPTS", "").split(","):  # (A/B: "save_group_blocks=16384,zc_small=0")
        if kv:
            ctx.set_option(kv.split("=")[0], int(kv.split("=")[1]))
    dp = ctx.device_alloc(n + 16)
    ctx.h2d(dp, data)
    ob = ctx.pinned_bytes(int(n * 1.01) + 4096 * nfiles + (1 << 16))
    for mode in modes:
        for c in range(calls):
            t0 = time.perf_counter()
            with ctx.index_create() as ix:
                ids, fb, new, packed, packs = ctx.save_files(p, ix, dp, offs, lens, bytes(range(32)), nonces, hn, pad,
                                                         n=n, gpu_compress=mode == "gpu", out_buf=ob, split=False)
            dt = time.perf_counter() - t0
            print(f"{mode} call {c}: {dt * 1e3:.1f} ms  {n / dt / 2**30:.2f} GiB/s  stored {int(new.sum())}  "
                  f"packed {packed.size}", flush=True)
