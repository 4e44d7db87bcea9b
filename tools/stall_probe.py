"""Where the occasional 12-30 ms stall of a kernel-tree save call comes from
(DESIGN.md 0e item 2): save calls with the kernel's page-reclaim / compaction
counters (/proc/vmstat) read around each, first in a fresh process, then
after the process allocated, touched and freed many GiB of host memory (as
bench.py's earlier legs do).  Tools only.  Usage: python tools/stall_probe.py [calls]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402
from tests import corpora  # noqa: E402

KEYS = ("compact_stall", "compact_fail", "compact_success", "thp_fault_alloc", "thp_fault_fallback",
        "allocstall_normal", "allocstall_movable", "pgmajfault", "pgscan_direct", "thp_collapse_alloc")


def vm():
    d = {}
    for line in open("/proc/vmstat"):
        k, v = line.split()
        if k in KEYS:
            d[k] = int(v)
    return d


def thp():
    out = {}
    for f in ("enabled", "defrag"):
        try:
            out[f] = open(f"/sys/kernel/mm/transparent_hugepage/{f}").read().strip()
        except OSError as ex:
            out[f] = str(ex)
    return out


calls = int(sys.argv[1]) if len(sys.argv) > 1 else 8
print("THP", thp(), flush=True)
data, offs, lens, dup = corpora.kernel_tree(80000)
n = int(data.size)
p = _lib.params(512 << 10, 1 << 20, 8 << 20, 1)
rng = np.random.default_rng(9)
nonces = rng.integers(0, 256, (80000 + n // (512 << 10) + 64, 12), dtype=np.uint8)
hn, pad = rng.integers(0, 256, (4096, 12), dtype=np.uint8), rng.integers(0, 256, (4096 * 63, 36), dtype=np.uint8)
with _lib.Context(0, 2 << 30) as ctx:
    dp = ctx.device_alloc(n + 16)
    ctx.h2d(dp, data)
    ob = ctx.pinned_bytes(int(n * 1.01) + 4096 * 80000 + (1 << 16))

    def run(tag):
        for c in range(calls):
            v0 = vm()
            t0 = time.perf_counter()
            with ctx.index_create() as ix:
                ctx.save_files(p, ix, dp, offs, lens, bytes(range(32)), nonces, hn, pad, n=n, gpu_compress=True,
                               out_buf=ob, split=False)
            dt = (time.perf_counter() - t0) * 1e3
            v1 = vm()
            delta = {k: v1[k] - v0.get(k, 0) for k in v1 if v1[k] != v0.get(k, 0)}
            print(f"{tag} call {c}: {dt:.1f} ms  vmstat {delta}", flush=True)

    run("fresh")
    for rep in range(3):  # many GiB allocated, touched, freed (bench.py's e2e / CPU-baseline legs do this)
        bufs = [np.ones(2 << 30, np.uint8) for _ in range(4)]
        small = [np.ones(int(s), np.uint8) for s in rng.integers(1 << 16, 8 << 20, 400)]
        del bufs
        del small[::2]
    run("after-churn")
