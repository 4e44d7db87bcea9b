"""Probe for the k_emit_long LDS-table item: runs the recorded
failing sequence (a 512K/1M/8M call over 2.2 GiB of zeros, then a 64/256/1024
call over 80 MiB of zeros, each emitted by k_emit_long) against the debug
library built by tools/dbg/build_dbg.sh, whose k_emit / k_emit_long read GEAR
from LDS and compare every chunk hash with the global-table hash, recording
each mismatch with the wave's HW_ID / XCC_ID.

    MCDC_LIBRARY=tools/dbg/libmcdc_dbg.so python tools/dbg/lds_probe.py [iterations]
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mapache_amd import _lib  # noqa: E402
from oracle import oracle as O  # noqa: E402

P512 = (524288, 1048576, 8388608, 1)
TINY = (64, 256, 1024, 1)
P16 = (16384, 65536, 262144, 1)
KINDS = {1: "table@start(emit_long)", 2: "hash(emit_long)", 3: "table@end(emit_long)", 4: "hash(emit)", 5: "suspicious(emit_long)"}


def dbg_dump(tag):
    L = _lib.load()
    if not hasattr(L, "mcdc_dbg_read"):
        return 0
    buf = (ctypes.c_uint64 * (1 + 256 * 16))()
    assert L.mcdc_dbg_read(buf, ctypes.sizeof(buf)) == 0
    n = buf[0]
    if n:
        print(f"  DBG {tag}: {n} records", flush=True)
        for k in range(min(n, 24)):
            v = buf[1 + 16 * k: 17 + 16 * k]
            hw = v[3]
            print("   ", KINDS.get(v[0], v[0]), "blk", v[1], "tid", v[2], "xcc", hw >> 32, "hwid", hex(hw & 0xffffffff),
                  "rest", [hex(x) for x in v[4:16]], flush=True)
        L.mcdc_dbg_reset()
    return n


def check(tag, p, g, d):
    ref = O.chunk(O.Params(*p), d)
    bad = np.nonzero((g["offset"] != ref["offset"]) | (g["length"] != ref["length"]) | (g["hash"] != ref["hash"]))[0]
    hb = np.nonzero(g["hash"] != ref["hash"])[0] if len(g) == len(ref) else []
    print(f"  {tag} {p} chunks {len(g)}/{len(ref)} bad {len(bad)} hash-bad {len(hb)} first {bad[:4]}",
          [hex(int(x)) for x in g["hash"][bad[:2]]], [hex(int(x)) for x in ref["hash"][bad[:2]]], flush=True)
    return len(bad)


def dev_call(ctx, p, d):
    n = len(d)
    dp = ctx.device_alloc(n + 64)
    ctx.h2d(dp, d)
    cap = n // (p[0] - 1) + 2
    do = ctx.device_alloc(cap * 24)
    c = ctx.chunk_device_to_device(_lib.params(*p), dp, n, do, cap)
    g = ctx.d2h_chunks(do, c)
    ctx.device_free(do)
    ctx.device_free(dp)
    return g


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    budget = float(os.environ.get("PROBE_SECONDS", "200"))
    L = _lib.load()
    try:  # the instrumented builds only
        L.mcdc_dbg_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.mcdc_dbg_reset.argtypes = []
        L.mcdc_dbg_reset()
    except AttributeError:
        pass
    pre = O.random_bytes(100_003, 9)
    tail = O.random_bytes(3 << 20, 10)
    dt = np.concatenate([pre, np.zeros(80 << 20, np.uint8), tail])
    dp = np.concatenate([pre, np.zeros(2200 << 20, np.uint8), tail])
    t0 = time.time()
    bad = dbg = 0
    tiny_only = os.environ.get("PROBE_TINY_ONLY") == "1"
    for it in range(iters):
        if tiny_only:
            if time.time() - t0 > budget:
                break
            ctx = _lib.Context(0, 16 << 30)
            print(f"iter {it} tiny only", flush=True)
            for k in range(4):
                bad += check("tiny dev", TINY, dev_call(ctx, TINY, dt), dt)
                dbg += dbg_dump("after tiny dev")
            ctx.close()
            continue
        for exp in range(3):
            if time.time() - t0 > budget:
                break
            ctx = _lib.Context(0, 16 << 30)
            print(f"iter {it} exp {exp}", flush=True)
            if exp == 0:
                bad += check("p512 host", P512, ctx.chunk_host(_lib.params(*P512), dp), dp)
                dbg += dbg_dump("after p512 host")
                bad += check("tiny dev", TINY, dev_call(ctx, TINY, dt), dt)
                dbg += dbg_dump("after tiny dev")
            elif exp == 1:
                bad += check("p512 dev", P512, dev_call(ctx, P512, dp), dp)
                dbg += dbg_dump("after p512 dev")
                bad += check("tiny host", TINY, ctx.chunk_host(_lib.params(*TINY), dt), dt)
                dbg += dbg_dump("after tiny host")
                bad += check("p16 host", P16, ctx.chunk_host(_lib.params(*P16), dt), dt)
                dbg += dbg_dump("after p16 host")
            else:
                bad += check("p512 dev", P512, dev_call(ctx, P512, dp), dp)
                dbg += dbg_dump("after p512 dev")
                bad += check("tiny dev", TINY, dev_call(ctx, TINY, dt), dt)
                dbg += dbg_dump("after tiny dev")
            ctx.close()
    print(f"DONE bad={bad} dbg_records={dbg} seconds={time.time() - t0:.1f}", flush=True)


if __name__ == "__main__":
    main()
