"""zstd raw-block frame writer (mcdc_zstd_frames_device) over the chunks of a
device-resident stream: device time per call, HBM rate (input read + frames
written), and a digest of sampled frame bytes for A/B builds (MCDC_LIBRARY).
usage: python tools/zframe_bench.py [GiB] [reps]"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = int(gib * (1 << 30))
with _lib.Context(0, n) as ctx:
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, 0x7a66726d)
    p = _lib.params(16384, 65536, 262144, 1)
    cap = n // (p.min_size - 1) + 2
    d_ch = ctx.device_alloc(cap * 24)
    k = ctx.chunk_device_to_device(p, dp, n, d_ch, cap)
    out_cap = n + 32 * k + (1 << 20)
    d_out = ctx.device_alloc(out_cap)
    ts = []
    for _ in range(reps):
        fr, span = ctx.zstd_frames(dp, n, (d_ch, k), d_out, out_cap)
        ts.append(ctx.timing()["device_ms"])
    h = hashlib.sha256()
    for j in np.linspace(0, k - 1, 64).astype(int):
        o, ln = int(fr[j, 0]), int(fr[j, 1])
        h.update(ctx.d2h_bytes(d_out + o, ln).tobytes())
    t = min(ts)
    print(f"{os.path.basename(os.environ.get('MCDC_LIBRARY', 'libmcdc.so'))}: {k} chunks, frames {t:.2f} ms "
          f"(median {sorted(ts)[len(ts) // 2]:.2f}), {(n + span) / (t * 1e-3) / 1e12:.2f} TB/s, "
          f"digest {h.hexdigest()[:16]}", flush=True)
    for x in (d_out, d_ch, dp):
        ctx.device_free(x)
