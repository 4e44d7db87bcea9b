"""Seal/open microbenchmark (iteration tool; bench.py's `seal` leg is the
reported one): the chunks of an N-GiB device stream as blobs, K timed calls
each, per-call device time from the library's events."""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = int(gib * (1 << 30))
ctx = _lib.Context(0, n + (1 << 20))
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, 0x6d61706163686521)
ch = ctx.chunk_device(_lib.params(16384, 65536, 262144, 1), dp, n)
k = len(ch)
nonces = np.zeros((k, 12), np.uint8)
nonces[:, :4] = np.arange(k, dtype=np.uint32).view(np.uint8).reshape(k, 4)
key = bytes(range(32))
cap = n + 28 * k
ds, do = ctx.device_alloc(cap), ctx.device_alloc(n)
for name, fn in (("seal", lambda: ctx.seal(key, dp, n, ch["offset"], ch["length"], nonces, ds, cap)),
                 ("open", lambda: ctx.open(key, ds, cap, oo[:-1], np.diff(oo), do, n))):
    r = fn()
    if name == "seal":
        oo = r
    dev = []
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
        dev.append(ctx.timing()["aead_ms"])
    dt = (time.perf_counter() - t0) / steps
    dig = ""
    if name == "seal":  # digest of a 256 MiB sample of the sealed output (compares builds)
        dig = hashlib.sha256(ctx.d2h_bytes(ds, min(int(oo[-1]), 256 << 20)).tobytes()).hexdigest()[:16]
    print(f"{os.path.basename(_lib.LIB_PATH)} {dig} {name}: {k} blobs, {dt * 1e3:.2f} ms/call ({n / dt / 2**30:.1f} GiB/s), kernels {np.median(dev):.2f} ms",
          flush=True)
ctx.close()
