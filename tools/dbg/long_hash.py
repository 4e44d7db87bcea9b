import numpy as np, sys
sys.path.insert(0, '.')
from mapache_amd import _lib
from oracle import oracle as O
p = (64, 256, 1024, 1)
z = 80 << 20
d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(z, np.uint8), O.random_bytes(3 << 20, 10)])
ref = O.chunk(O.Params(*p), d)
with _lib.Context(0, 1 << 30) as ctx:
    for rep in range(3):
        g = ctx.chunk_host(_lib.params(*p), d)
        bad = np.nonzero((g["offset"] != ref["offset"]) | (g["length"] != ref["length"]) | (g["hash"] != ref["hash"]))[0]
        print("host", rep, len(g), len(ref), bad[:10], [hex(int(x)) for x in g["hash"][bad[:5]]], ctx.timing()["fallback_files"], flush=True)
    n = len(d)
    dp = ctx.device_alloc(n + 64)
    ctx.h2d(dp, d)
    back = ctx.d2h_bytes(dp, n)
    print("arena equal", bool((back == d).all()), flush=True)
    cap = n // 63 + 2
    d_out = ctx.device_alloc(cap * 24)
    for rep in range(3):
        cnt = ctx.chunk_device_to_device(_lib.params(*p), dp, n, d_out, cap)
        g = ctx.d2h_chunks(d_out, cnt)
        bad = np.nonzero((g["offset"] != ref["offset"]) | (g["length"] != ref["length"]) | (g["hash"] != ref["hash"]))[0]
        print("dev", rep, cnt, bad[:10], [hex(int(x)) for x in g["hash"][bad[:5]]], flush=True)
