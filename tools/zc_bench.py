"""GPU zstd compression throughput and ratio (mcdc_zstd_compress_device) on a
random stream and on the bench's synthetic corpora, chunked at 16/64/256 KiB
(or mapache's 512K/1M/8M: P512); device-resident in and out.
Kind "tree": the configs[3] kernel-tree stand-in (tests/corpora.kernel_tree,
1.33 GB), one chunk per file as the save path's whole-file branch stores them
(GiB ignored).
Usage: python tools/zc_bench.py [GiB] [steps] [kinds,...] [P16|P512]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mapache_amd import _lib  # noqa: E402
from oracle import oracle as O  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = int(gib * (1 << 30))
p = _lib.params(524288, 1048576, 8388608, 1) if len(sys.argv) > 4 and sys.argv[4] == "P512" else \
    _lib.params(16384, 65536, 262144, 1)
ctx_cap = n + (1 << 20)
ctx = _lib.Context(0, ctx_cap)
ZC_BATCH = int(os.environ.get("ZC_BATCH", "0"))  # (A/B: the compressor's batch, "zc_batch_blocks")
ZC_OPTS = [(k, int(v)) for k, v in (kv.split("=") for kv in os.environ.get("ZC_OPTS", "").split(",") if kv)]
if ZC_BATCH:
    ZC_OPTS.append(("zc_batch_blocks", ZC_BATCH))
for k_, v_ in ZC_OPTS:  # (A/B: "zc_two=0,zc_small=0", mcdc_ctx_set_option)
    ctx.set_option(k_, v_)
res = {}
n_arg = n
for kind in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("random", "text", "records", "binary", "far")):
    n = n_arg
    tree = None
    if kind == "tree":
        from tests import corpora
        tree = corpora.kernel_tree(80000)
        n = int(tree[0].size)
        if n + (1 << 20) > ctx_cap:
            ctx.close()
            ctx_cap = n + (1 << 20)
            ctx = _lib.Context(0, ctx_cap)
            for k_, v_ in ZC_OPTS:
                ctx.set_option(k_, v_)
    dp = ctx.device_alloc(n)
    if tree is not None:
        ctx.h2d(dp, tree[0])
    elif kind == "random":
        ctx.fill_random(dp, n, 0x6d61706163686521)
    else:  # the shared synthetic corpora (tests/corpora.py), a 64 MiB pattern repeated
        sys.path.insert(0, ROOT)
        from tests import corpora
        base = corpora.by_name(kind, 64 << 20).tobytes()
        for o in range(0, n, len(base)):
            ctx.h2d(dp + o, np.frombuffer(base[:min(len(base), n - o)], np.uint8))
    if tree is not None:  # one chunk per file
        ch = np.zeros(tree[1].size, _lib.CHUNK_DTYPE)
        ch["offset"], ch["length"] = tree[1], tree[2]
        k = int(ch.size)
        d_ch = ctx.device_alloc(24 * k)
        ctx.h2d(d_ch, ch.view(np.uint8))
    else:
        cap_c = n // 16383 + 2
        d_ch = ctx.device_alloc(24 * cap_c)
        k = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
        ch = ctx.d2h_chunks(d_ch, k)
    cap = _lib.Context.zstd_compress_bound(ch["length"])
    d_out, d_fr = ctx.device_alloc(cap), ctx.device_alloc(16 * k)
    ctx.zstd_compress(dp, n, (d_ch, k), d_out, cap, frames_out=d_fr)
    t0 = time.perf_counter()
    for _ in range(steps):
        _, nb = ctx.zstd_compress(dp, n, (d_ch, k), d_out, cap, frames_out=d_fr)
    dt = (time.perf_counter() - t0) / steps
    dev = ctx.timing()["device_ms"]
    fr = ctx.d2h_bytes(d_fr, 16 * 8).view(np.uint64).reshape(8, 2)
    z = O.Zstd()
    ok = True
    for i in range(8):
        src = ctx.d2h_bytes(dp + int(ch["offset"][i]), int(ch["length"][i])).tobytes()
        try:
            ok &= z.decompress(ctx.d2h_bytes(d_out + int(fr[i, 0]), int(fr[i, 1])).tobytes(), len(src) + 64) == src
        except AssertionError:  # (A/B timing variants may not decode)
            ok = False
    lv3 = 0  # libzstd level 3 (the crate's streaming encoder) on the first 32 MiB of chunks
    k3 = int(np.searchsorted(np.cumsum(ch["length"].astype(np.int64)), 32 << 20)) + 1
    for i in range(min(k3, k)):
        lv3 += len(z.compress(ctx.d2h_bytes(dp + int(ch["offset"][i]), int(ch["length"][i])).tobytes(), False))
    fr3 = ctx.d2h_bytes(d_fr, 16 * min(k3, k)).view(np.uint64).reshape(-1, 2)
    gpu3 = int(fr3[:, 1].sum())
    res[kind] = {"gib_s": round(n / dt / (1 << 30), 2), "device_ms": round(dev, 3), "ratio": round(n / nb, 4),
                 "chunks": int(k), "probe_ok": bool(ok),
                 "ratio_32mib": round(float(ch["length"][:min(k3, k)].sum()) / gpu3, 4),
                 "level3_ratio_32mib": round(float(ch["length"][:min(k3, k)].sum()) / lv3, 4)}
    for x in (d_fr, d_out, d_ch, dp):
        ctx.device_free(x)
print(json.dumps(res))
