import numpy as np, sys
sys.path.insert(0, '.')
from mapache_amd import _lib
from oracle import oracle as O

def run(ctx, p, d, tag):
    ref = O.chunk(O.Params(*p), d)
    g = ctx.chunk_host(_lib.params(*p), d)
    bad = np.nonzero((g["offset"] != ref["offset"]) | (g["length"] != ref["length"]) | (g["hash"] != ref["hash"]))[0]
    print(tag, p, len(g), len(ref), len(bad), bad[:6], [hex(int(x)) for x in g["hash"][bad[:3]]], flush=True)
    return bad

ctx = _lib.Context(0, 16 << 30)
pre = O.random_bytes(100_003, 9)
tail = O.random_bytes(3 << 20, 10)
tiny = (64, 256, 1024, 1)
dt = np.concatenate([pre, np.zeros(80 << 20, np.uint8), tail])
run(ctx, tiny, dt, "fresh")
dp = np.concatenate([pre, np.zeros(2200 << 20, np.uint8), tail])
run(ctx, (524288, 1048576, 8388608, 1), dp, "p512")
del dp
b = run(ctx, tiny, dt, "after-p512")
run(ctx, tiny, dt, "again")
run(ctx, (16384, 65536, 262144, 1), dt, "p16")
run(ctx, tiny, dt, "after-p16")
