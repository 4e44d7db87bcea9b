import numpy as np, sys
sys.path.insert(0, '.')
from mapache_amd import _lib
from oracle import oracle as O

P512 = (524288, 1048576, 8388608, 1)
TINY = (64, 256, 1024, 1)

def check(tag, p, g, d):
    ref = O.chunk(O.Params(*p), d)
    bad = np.nonzero((g["offset"] != ref["offset"]) | (g["length"] != ref["length"]) | (g["hash"] != ref["hash"]))[0]
    print(tag, p, len(g), len(ref), len(bad), bad[:4], [hex(int(x)) for x in g["hash"][bad[:2]]], flush=True)

def dev_call(ctx, p, d):
    n = len(d)
    dp = ctx.device_alloc(n + 64)
    ctx.h2d(dp, d)
    cap = n // (p[0] - 1) + 2
    do = ctx.device_alloc(cap * 24)
    c = ctx.chunk_device_to_device(_lib.params(*p), dp, n, do, cap)
    g = ctx.d2h_chunks(do, c)
    ctx.device_free(do); ctx.device_free(dp)
    return g

pre = O.random_bytes(100_003, 9)
tail = O.random_bytes(3 << 20, 10)
dt = np.concatenate([pre, np.zeros(80 << 20, np.uint8), tail])
dp = np.concatenate([pre, np.zeros(2200 << 20, np.uint8), tail])
for exp in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    ctx = _lib.Context(0, 16 << 30)
    if exp == 0:
        check("e0 p512 host", P512, ctx.chunk_host(_lib.params(*P512), dp), dp)
        check("e0 tiny dev", TINY, dev_call(ctx, TINY, dt), dt)
    elif exp == 1:
        check("e1 p512 dev", P512, dev_call(ctx, P512, dp), dp)
        check("e1 tiny host", TINY, ctx.chunk_host(_lib.params(*TINY), dt), dt)
    else:
        check("e2 p512 dev", P512, dev_call(ctx, P512, dp), dp)
        check("e2 tiny dev", TINY, dev_call(ctx, TINY, dt), dt)
    ctx.close()
