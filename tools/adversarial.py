"""Throughput and parity of the device path on non-random inputs (SURVEY 8d
'value distributions / adversarial'): all zeros, periodic data of several
periods, low-entropy text, long runs.  Not part of the product.

    python tools/adversarial.py [GiB per pattern] [P16|P512]

Each pattern is generated on the host, copied to HBM once, chunked 3 times
device-to-device (best time reported, with the scan / device split), and the
boundary list is compared with the oracle on the whole buffer."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import _lib  # noqa: E402
from oracle import oracle as O  # noqa: E402

GIB = 1 << 30
PARAMS = {"P16": (16384, 65536, 262144, 1), "P512": (524288, 1 << 20, 8 << 20, 1)}


def pattern(name: str, n: int, rng) -> np.ndarray:
    if name == "zeros":
        return np.zeros(n, np.uint8)
    if name.startswith("period"):
        per = int(name[6:])
        blk = rng.integers(0, 256, per, dtype=np.uint8)
        return np.resize(blk, n)
    if name == "text":  # words from a 2 000-word vocabulary of lowercase letters, spaces, newlines
        vocab = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 10, 2000)]
        seq = rng.integers(0, len(vocab), n // 4 + 16)
        body = b" ".join(vocab[i] for i in seq[: 1 << 20])  # ~6 MiB, tiled
        return np.resize(np.frombuffer(body, np.uint8), n)
    if name.startswith("mixed"):  # alternating random / zero blocks of <k> MiB
        k = int(name[5:-1]) << 20
        out = rng.integers(0, 256, n, dtype=np.uint8)
        for b in range(k, n, 2 * k):
            out[b:b + k] = 0
        return out
    if name == "sparse":  # a 4 MiB random extent every 512 MiB, zeros elsewhere (a sparse disk image)
        out = np.zeros(n, np.uint8)
        for b in range(0, n, 512 << 20):
            out[b + 12345:b + 12345 + (4 << 20)] = rng.integers(0, 256, 4 << 20, dtype=np.uint8)[: max(0, min(4 << 20, n - b - 12345))]
        return out
    if name == "runs":  # runs of one random byte, lengths 1..64 KiB
        out = np.empty(n, np.uint8)
        pos = 0
        while pos < n:
            k = int(rng.integers(1, 65536))
            out[pos:pos + k] = rng.integers(0, 256)
            pos += k
        return out
    raise ValueError(name)


def main() -> int:
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    pname = sys.argv[2] if len(sys.argv) > 2 else "P16"
    n = int(gib * GIB)
    p = _lib.params(*PARAMS[pname])
    op = O.Params(*PARAMS[pname])
    rng = np.random.default_rng(7)
    names = ["zeros", "period64", "period1000", "period4096", "period65536", "period1048573", "text", "runs",
             "mixed1m", "mixed32m", "sparse"]
    if len(sys.argv) > 3:
        names = sys.argv[3].split(",")
    with _lib.Context(0, n) as ctx:
        dp = ctx.device_alloc(n)
        cap = n // (p.min_size - 1) + 2
        d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
        for name in names:
            host = pattern(name, n, rng)
            ctx.h2d(dp, host)
            best, bt, count = None, None, 0
            for _ in range(3):
                t0 = time.perf_counter()
                count = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
                dt = time.perf_counter() - t0
                if best is None or dt < best:
                    best, bt = dt, ctx.timing()
            got = ctx.d2h_chunks(d_out, count)
            ref = O.chunk(op, host)
            same = bool(len(got) == len(ref) and (got["offset"] == ref["offset"]).all()
                        and (got["length"] == ref["length"]).all())
            print(json.dumps({"pattern": name, "params": pname, "bytes": n, "chunks": int(count),
                              "gib_s": round(n / best / GIB, 1), "scan_ms": round(bt["scan_ms"], 3),
                              "device_ms": round(bt["device_ms"], 3), "call_ms": round(best * 1e3, 3),
                              "parity": same}), flush=True)
        ctx.device_free(d_out)
        ctx.device_free(dp)
    return 0


if __name__ == "__main__":
    sys.exit(main())
