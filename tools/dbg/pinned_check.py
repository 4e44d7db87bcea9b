"""Debug: the 64 GiB headline chunked with the boundary list written to device
memory vs straight into pinned host memory (k_emit over PCIe); report where
and how the two lists differ, per repetition."""
import sys
import numpy as np
sys.path.insert(0, ".")
from mapache_amd import _lib

SEED = 0x6d61706163686521
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = int(gib * (1 << 30))
p = _lib.params(16384, 65536, 262144, 1)
ctx = _lib.Context(0, n + 262144)
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, SEED)
cap = n // 16383 + 2
d_out = ctx.device_alloc(cap * 24)
k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
ref = ctx.d2h_chunks(d_out, k)
print("device list", k, flush=True)
out = ctx.pinned_out(cap)
for r in range(reps):
    hc = ctx.chunk_device(p, dp, n, out=out)
    same = len(hc) == len(ref) and (hc == ref).all()
    print(f"rep {r}: count {len(hc)} same={same}", flush=True)
    if not same:
        m = min(len(hc), len(ref))
        bad = np.nonzero(hc[:m] != ref[:m])[0]
        print("  mismatches", len(bad), "first", bad[:10].tolist(), flush=True)
        for i in bad[:5]:
            print("  ", i, hc[i], ref[i], flush=True)
    hc2 = ctx.chunk_device(p, dp, n)  # pageable host out (staged + D2H)
    print(f"   pageable same={len(hc2) == len(ref) and bool((hc2 == ref).all())}", flush=True)
ctx.close()
