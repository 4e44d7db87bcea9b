"""Debug: block types/sizes of the GPU zstd frames of a few chunks."""
import sys
import numpy as np
sys.path.insert(0, ".")
from mapache_amd import _lib
from oracle import oracle as O


def blocks(frame):
    at, out = 6, []
    while at < len(frame):
        h = frame[at] | frame[at + 1] << 8 | frame[at + 2] << 16
        last, typ, size = h & 1, (h >> 1) & 3, h >> 3
        out.append((typ, size))
        at += 3 + (size if typ != 1 else 1)
        if last:
            break
    return out


ctx = _lib.Context(0, 1 << 28)
for kind in ("zeros", "text"):
    if kind == "zeros":
        data = np.zeros(256 << 10, np.uint8)
    else:
        rng = np.random.default_rng(1)
        vocab = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 11, 2000)]
        data = np.frombuffer(b" ".join(vocab[i] for i in rng.integers(0, 2000, 80000))[:256 << 10], np.uint8).copy()
    ch = np.zeros(1, dtype=_lib.CHUNK_DTYPE)
    ch["length"] = data.size
    dp = ctx.device_alloc(data.size)
    cap = _lib.Context.zstd_compress_bound(ch["length"])
    d_out = ctx.device_alloc(cap)
    ctx.h2d(dp, data)
    fr, nb = ctx.zstd_compress(dp, data.size, ch, d_out, cap)
    out = ctx.d2h_bytes(d_out, nb).tobytes()
    print(kind, nb, blocks(out))
