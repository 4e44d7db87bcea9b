"""Debug: determinism of ChunkData.hash on the 64 GiB headline.  Device-out
lists from repeated calls compared with each other; mismatching records
checked against the oracle's cut_gear restarted at the chunk."""
import sys
import numpy as np
sys.path.insert(0, ".")
from mapache_amd import _lib
from oracle import oracle as O

SEED = 0x6d61706163686521
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = int(gib * (1 << 30))
P = (16384, 65536, 262144, 1)
p = _lib.params(*P)
ctx = _lib.Context(0, n + 262144)
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, SEED)
cap = n // 16383 + 2
d_out = ctx.device_alloc(cap * 24)
lists = []
for r in range(reps):
    k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
    lists.append(ctx.d2h_chunks(d_out, k))
    t = ctx.timing()
    print(f"rep {r}: {k} chunks, fallback_files {t['fallback_files']}", flush=True)
A = lists[0]
allbad = set()
for r in range(1, reps):
    B = lists[r]
    assert (A["offset"] == B["offset"]).all() and (A["length"] == B["length"]).all()
    bad = np.nonzero(A["hash"] != B["hash"])[0]
    allbad.update(bad.tolist())
    print(f"rep 0 vs {r}: {len(bad)} hash mismatches; first {bad[:8].tolist()}", flush=True)
bad = sorted(allbad)
if bad:
    print("offsets of first mismatches (GiB):", [round(int(A['offset'][i]) / 2**30, 3) for i in bad[:8]])
    print("lengths:", [int(A['length'][i]) for i in bad[:8]])
rng = np.random.default_rng(0)
check = bad[:6] + sorted(rng.choice(len(A), 6, replace=False).tolist())
for i in check:
    o, ln = int(A["offset"][i]), int(A["length"][i])
    w = ctx.d2h_bytes(dp + o, min(P[2] + 1, n - o))
    rh, rl = O.cut_gear(O.Params(*P), w)
    hs = [int(L["hash"][i]) for L in lists]
    print(f"chunk {i} off {o} len {ln}: oracle ({rh}, {rl}) got {hs} -> ok per rep {[h == rh for h in hs]}",
          flush=True)
ctx.close()
