"""BASELINE.json's configs at their own sizes, against the oracle.

* configs[1]: the 64 GiB uniform-random stream of the headline, device
  resident, chunked as one file at 16/64/256 KiB: the whole boundary list's
  (count, digest, sum of lengths) and the digest of every ChunkData.hash
  against the oracle's, which regenerates the same counter-based stream slab
  by slab (oracle/fastcdc_oracle.c oc_random_stream_digest_h) so the host
  never holds 64 GiB; plus the size-independent invariants (lengths sum to n,
  offsets contiguous, every non-tail chunk within [min, max]), hash spot
  checks, and four more calls (device and pinned-host output) identical to
  the first, record for record (the k_emit VGPR item, DESIGN.md §3a, changed
  ~3 % of the hashes of some calls).
* configs[3] stand-in: the bench's 80 000-file log-normal mix (median 8 KiB,
  1.34 GB; bench.py small_files), one batched device call, every file's
  boundary list and count against oracle.chunk_files.
"""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x6d61706163686521
P16 = (16384, 65536, 262144, 1)


def test_configs1_full_64gib_digest(ctx):
    n = 64 << 30
    p = _lib.params(*P16)
    big = _lib.Context(0, n)
    try:
        dp = big.device_alloc(n)
        cap = n // (P16[0] - 1) + 2
        d_out = big.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
        try:
            big.fill_random(dp, n, SEED)
            k = big.chunk_device_to_device(p, dp, n, d_out, cap)
            g = big.d2h_chunks(d_out, k)
            again = []
            for _ in range(2):
                again.append(big.d2h_chunks(d_out, big.chunk_device_to_device(p, dp, n, d_out, cap)))
                again.append(big.chunk_device(p, dp, n, out=big.pinned_out(cap)).copy())
            samples = []
            for i in np.linspace(0, k - 2, 24).astype(int):
                o = int(g["offset"][i])
                samples.append((i, big.d2h_bytes(dp + o, min(P16[2] + 1, n - o))))
        finally:
            big.device_free(d_out)
            big.device_free(dp)
    finally:
        big.close()
    assert int(g["length"].sum()) == n
    assert (g["offset"][1:] == np.cumsum(g["length"])[:-1]).all() and g["offset"][0] == 0
    assert g["length"][:-1].min() >= P16[0] and g["length"].max() <= P16[2]
    rk, rdig, rsum, rhd = O.random_stream_digest(O.Params(*P16), SEED, n, hashes=True)
    assert rsum == n
    assert rk == k, (rk, k)
    assert _lib.digest(g) == rdig
    assert O.hash_digest(g) == rhd
    for j, a in enumerate(again):
        assert len(a) == k and (a == g).all(), (j, int(np.count_nonzero(a["hash"] != g["hash"])))
    for i, window in samples:  # hash and length from cut_gear restarted at the chunk
        assert O.cut_gear(O.Params(*P16), window) == (int(g["hash"][i]), int(g["length"][i]))


def test_configs3_80k_small_files(ctx):
    rng = np.random.default_rng(20251016)  # bench.py small_files
    nfiles = 80_000
    sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, nfiles)).astype(np.uint64) + 1, 64 << 20)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    n = int(sizes.sum())
    p = _lib.params(*P16)
    arena = ctx.device_alloc(n + 16)
    cap = int(sum(int(s) // (P16[0] - 1) + 2 for s in sizes))
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(arena, n, SEED ^ 0x5F)
        total, counts = ctx.chunk_batch_device_to_device(p, arena, offs, sizes, d_out, cap)
        got = ctx.d2h_chunks(d_out, total)
    finally:
        ctx.device_free(d_out)
        ctx.device_free(arena)
    host = O.random_bytes(n, SEED ^ 0x5F)
    ref, rc = O.chunk_files(O.Params(*P16), [host[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)], threads=8)
    assert counts.size == nfiles and (counts == rc).all()
    assert len(got) == len(ref)
    bad = np.nonzero((got["offset"] != ref["offset"]) | (got["length"] != ref["length"]) |
                     (got["hash"] != ref["hash"]))[0]
    assert bad.size == 0, f"first mismatch at chunk {bad[0]}"
