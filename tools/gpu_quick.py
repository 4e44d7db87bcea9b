"""Quick GPU bring-up check: parity vs oracle on small/medium inputs + timing."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from mapache_amd import _lib as M
from oracle import oracle as O

def cmp(name, a, b):
    ok = len(a) == len(b) and (a['offset'] == b['offset']).all() and (a['length'] == b['length']).all()
    okh = ok and (a['hash'] == b['hash']).all()
    print(f"{name}: gpu={len(a)} ref={len(b)} bounds={'OK' if ok else 'MISMATCH'} hash={'OK' if okh else 'MISMATCH'}", flush=True)
    if not ok:
        n = min(len(a), len(b))
        bad = np.nonzero((a['offset'][:n] != b['offset'][:n]) | (a['length'][:n] != b['length'][:n]))[0]
        i = bad[0] if len(bad) else n
        print("  first diff at", i, a[max(0,i-2):i+3], b[max(0,i-2):i+3])
    return okh

ctx = M.Context(0, 64 << 30)
allok = True
cases = [(O.P16, M.params(16384, 65536, 262144, 1)), (O.P512, M.params(524288, 1 << 20, 8 << 20, 1)),
         (O.Params(64, 256, 1024, 1), M.params(64, 256, 1024, 1)),
         (O.Params(4096, 16384, 65536, 2), M.params(4096, 16384, 65536, 2)),
         (O.Params(65, 300, 1111, 3), M.params(65, 300, 1111, 3))]
for seed, n in [(1, 0), (2, 1), (3, 100), (4, 70000), (5, 1 << 20), (6, (1 << 22) + 13), (7, 9 << 20)]:
    d = O.random_bytes(n, seed)
    for op, mp in cases:
        allok &= cmp(f"rand n={n} {op}", ctx.chunk_host(mp, d), O.chunk(op, d))
z = np.zeros(5 << 20, np.uint8)
for op, mp in cases:
    allok &= cmp(f"zeros {op}", ctx.chunk_host(mp, z), O.chunk(op, z))
# batch
files = [O.random_bytes(int(x), 100 + i) for i, x in enumerate([0, 5, 20000, 300000, 1 << 20, 3 << 20, 17])]
out, counts = ctx.chunk_batch(cases[0][1], files)
ref, rc = O.chunk_files(cases[0][0], files)
allok &= cmp("batch P16", out, ref) and (counts == rc).all()
# device-resident 1 GiB digest
n = 1 << 30
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, 0x6d61706163686521)
h = O.random_bytes(n, 0x6d61706163686521)
g = ctx.chunk_device(cases[0][1], dp, n)
allok &= cmp("device 1GiB P16", g, O.chunk(O.P16, h))
print("timing 1GiB:", ctx.timing(), flush=True)
ctx.device_free(dp)
# perf: 16 GiB
n = 16 << 30
dp = ctx.device_alloc(n)
ctx.fill_random(dp, n, 0x6d61706163686521)
for it in range(4):
    t0 = time.time(); g = ctx.chunk_device(cases[0][1], dp, n); t1 = time.time()
    t = ctx.timing()
    print(f"16GiB P16 it{it}: wall {t1-t0:.4f}s  {n/2**30/(t1-t0):.1f} GiB/s  scan {t['scan_ms']:.2f}ms ({n/t['scan_ms']/1e9:.1f} TB/s... GB/ms)  resolve {t['resolve_ms']:.2f}ms  chunks {t['chunks']} fb {t['fallback_files']}", flush=True)
for it in range(2):
    t0 = time.time(); g = ctx.chunk_device(cases[1][1], dp, n); t1 = time.time()
    t = ctx.timing()
    print(f"16GiB P512 it{it}: wall {t1-t0:.4f}s scan {t['scan_ms']:.2f}ms resolve {t['resolve_ms']:.2f}ms chunks {t['chunks']}", flush=True)
print("ALLOK" if allok else "FAILURES")
