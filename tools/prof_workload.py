"""Workload for the PMC passes (tools/profile_round.sh): one uniform-random
stream (`--gib`, default 16) chunked at 16/64/256 KiB device-resident
(`--steps` calls) and its chunk IDs computed (`--id-steps` calls).  Profiling
harness only."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=float, default=16)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--id-steps", type=int, default=3)
a = ap.parse_args()
n = int(a.gib * (1 << 30))
p = _lib.params(16384, 65536, 262144, 1)
with _lib.Context(0, n) as ctx:
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, 0x6d61706163686521)
    cap = n // (p.min_size - 1) + 2
    d_out = ctx.device_alloc(cap * 24)
    k = 0
    for _ in range(a.steps):
        k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
    d_ids = ctx.device_alloc(32 * k)
    for _ in range(a.id_steps):
        ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)
    print("chunks", k, "bytes", n, flush=True)
