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
* configs[2]: 10 000 independent 8 MiB files (78 GiB) in one batched device
  call (bench.py batch_files' arena: file i = bytes [8 MiB i, 8 MiB (i+1)) of
  the stream of SEED ^ 0xB0): every file's count, boundary digest and hash
  digest against oracle.random_files_digest, which regenerates each file on 16
  host threads (the host never holds the 78 GiB).
* configs[4], one rank's slice: 8192 files of 8 MiB (file i = the stream of
  SEED ^ (i + 1), bench.py corpus_sharded) through shard.chunk_sharded at
  world 1, every file and the corpus digest (shard.corpus_digest) against the
  oracle's.
* configs[3] stand-in: the bench's 80 000-file log-normal mix (median 8 KiB,
  1.34 GB; bench.py small_files), one batched device call, every file's
  boundary list and count against oracle.chunk_files.
"""
import numpy as np
import pytest

from mapache_amd import _lib, shard
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


def _per_file(g, counts):
    """(count, boundary digest, hash digest) of every file of a batch result."""
    starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return [(int(counts[k]), _lib.digest(g[starts[k]:starts[k + 1]]), O.hash_digest(g[starts[k]:starts[k + 1]]))
            for k in range(len(counts))]


def test_configs2_10000_files_full(ctx):
    nfiles, size = 10_000, 8 << 20
    n = nfiles * size
    p = _lib.params(*P16)
    offs = np.arange(nfiles, dtype=np.uint64) * np.uint64(size)
    lens = np.full(nfiles, size, dtype=np.uint64)
    big = _lib.Context(0, nfiles * size)
    try:
        arena = big.device_alloc(n)
        cap = nfiles * (size // (P16[0] - 1) + 2)
        d_out = big.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
        try:
            big.fill_random(arena, n, SEED ^ 0xB0)
            total, counts = big.chunk_batch_device_to_device(p, arena, offs, lens, d_out, cap)
            g = big.d2h_chunks(d_out, total)
        finally:
            big.device_free(d_out)
            big.device_free(arena)
    finally:
        big.close()
    assert counts.size == nfiles and int(counts.sum()) == total
    got = _per_file(g, counts)
    rc, rd, rh = O.random_files_digest(O.Params(*P16), SEED ^ 0xB0, offs, lens, threads=16)
    bad = [i for i in range(nfiles) if got[i] != (int(rc[i]), int(rd[i]), int(rh[i]))]
    assert not bad, (len(bad), bad[:8])
    # size-independent invariants over the whole list
    starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    assert (g["offset"][starts[:-1]] == 0).all()
    assert int(g["length"].sum()) == n


def test_configs4_rank_slice_8192_files(ctx):
    nfiles, size = 8192, 8 << 20
    p = _lib.params(*P16)
    sizes = [size] * nfiles
    big = _lib.Context(0, nfiles * size)
    try:
        arena = big.device_alloc(nfiles * size)
        cap = nfiles * (size // (P16[0] - 1) + 2)
        d_out = big.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
        try:
            def chunk_indices(idx):
                for k, i in enumerate(idx):
                    big.fill_random(arena + k * size, size, SEED ^ (i + 1))
                offs = np.arange(len(idx), dtype=np.uint64) * np.uint64(size)
                total, counts = big.chunk_batch_device_to_device(p, arena, offs, np.full(len(idx), size, np.uint64),
                                                                 d_out, cap)
                return big.d2h_chunks(d_out, total), counts
            per_file = shard.chunk_sharded(sizes, chunk_indices)
        finally:
            big.device_free(d_out)
            big.device_free(arena)
    finally:
        big.close()
    assert len(per_file) == nfiles
    cnt = [len(c) for c in per_file]
    dig = [_lib.digest(c) for c in per_file]
    rc, rd, rh = O.random_files_digest(O.Params(*P16), [SEED ^ (i + 1) for i in range(nfiles)], 0, sizes,
                                       threads=16)
    assert shard.corpus_digest(cnt, dig) == shard.corpus_digest(rc, rd)
    bad = [i for i in range(nfiles) if (cnt[i], dig[i], O.hash_digest(per_file[i])) !=
           (int(rc[i]), int(rd[i]), int(rh[i]))]
    assert not bad, (len(bad), bad[:8])
