"""Stress of the host staging path (mcdc_chunk_host from pageable memory):
sequential calls of varying sizes on one context, then 8 threads sharing it;
every result against the oracle.  Prints the failing calls."""
import sys, os, threading, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mapache_amd import _lib
from oracle import oracle as O

P16 = (16384, 65536, 262144, 1)
rng = np.random.default_rng(43)
sizes = [int(s) for s in rng.integers(0, 12 << 20, 24)]
files = [O.random_bytes(s, 8000 + i) for i, s in enumerate(sizes)]
refs = [O.chunk(O.Params(*P16), d) for d in files]

def same(g, r):
    return len(g) == len(r) and bool((g == r).all())

ctx = _lib.Context(0, 16 << 30)
bad = []
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for k in range(len(files)):
        g = ctx.chunk_host(_lib.params(*P16), files[k])
        if not same(g, refs[k]):
            r = refs[k]
            i = next((j for j in range(min(len(g), len(r))) if g[j] != r[j]), min(len(g), len(r)))
            bad.append(("seq", rep, k, sizes[k], len(g), len(r), i))
print("sequential bad:", bad, flush=True)
bad2 = []
def worker(w):
    for rep in range(3):
        for k in range(w, len(files), 8):
            if not same(ctx.chunk_host(_lib.params(*P16), files[k]), refs[k]):
                bad2.append(("thr", w, rep, k, sizes[k]))
ts = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
[t.start() for t in ts]; [t.join() for t in ts]
print("threaded bad:", bad2, flush=True)
print("sizes:", sizes)
