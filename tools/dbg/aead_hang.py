"""Debug: the two seal calls of test_rfc8452_vectors_on_gpu, in order, with
progress prints (run under a short timeout)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from mapache_amd import _lib

h = bytes.fromhex
ctx = _lib.Context(0, 1 << 20)


def seal(key, data, offs, lens, nonces):
    a = np.frombuffer(data, np.uint8)
    din = ctx.device_alloc(a.size + 64)
    if a.size:
        ctx.h2d(din, a)
    cap = int(sum(lens)) + 28 * len(lens)
    dout = ctx.device_alloc(cap + 64)
    oo = ctx.seal(key, din, a.size, offs, lens, nonces, dout, cap)
    got = ctx.d2h_bytes(dout, int(oo[-1]))
    ctx.device_free(dout)
    ctx.device_free(din)
    return got, oo


pts = [b"", h("0100000000000000"), h("010000000000000000000000"), h("01000000000000000000000000000000")]
print("call 1", flush=True)
g, oo = seal(h("01") + bytes(31), b"".join(pts), np.cumsum([0] + [len(p) for p in pts[:-1]]), [len(p) for p in pts],
             np.frombuffer(h("030000000000000000000000") * 4, np.uint8))
print("call 1 done", oo, flush=True)
print("call 2", flush=True)
g, oo = seal(bytes(32), bytes(56), [0, 32], [32, 24], np.zeros(24, np.uint8))
print("call 2 done", oo, flush=True)
