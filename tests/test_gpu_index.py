"""GPU dedup index (mcdc_index_add) against the save_blob restatement
(oracle.DedupIndex, repository_v1.rs:169-180): which IDs of a batch are
stored — the first of equal IDs in processing order, within a batch and
across batches — bit-exact flags, compacted chunk records and index sizes."""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu
SEED = 0x1D5


def _rand_ids(rng, n):
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


def test_distinct_then_repeated_batches(ctx):
    rng = np.random.default_rng(SEED)
    pool = _rand_ids(rng, 5000)
    ref = O.DedupIndex()
    with ctx.index_create() as ix:
        a = _rand_ids(rng, 100_000)
        assert ix.add(a).all() and ref.add(a).all()
        for _ in range(3):  # batches drawn from a pool: repeats within and across batches
            b = pool[rng.integers(0, pool.shape[0], 40_000)]
            b = np.concatenate([b, a[rng.integers(0, a.shape[0], 1000)]])
            assert (ix.add(b) == ref.add(b)).all()
        assert len(ix) == len(ref)


def test_all_identical_and_empty(ctx):
    one = np.tile(np.arange(32, dtype=np.uint8), (200_000, 1))
    with ctx.index_create() as ix:
        f = ix.add(one)
        assert f[0] and not f[1:].any()
        assert not ix.add(one[:10]).any()
        assert ix.add(np.zeros((0, 32), np.uint8)).size == 0
        assert len(ix) == 1


def test_prefix_collisions(ctx):
    """IDs sharing their first 8 bytes (the sort key) but differing later:
    full 32-byte compares inside equal-prefix runs, in the batch and in the index."""
    rng = np.random.default_rng(SEED + 1)
    ids = _rand_ids(rng, 3000)
    ids[:, :8] = rng.integers(0, 4, (3000, 1), dtype=np.uint8)  # only 4 distinct prefixes
    ids[::3, 8:] = ids[0, 8:]  # and many full duplicates among them
    ref = O.DedupIndex()
    with ctx.index_create() as ix:
        for part in np.array_split(ids, 4):
            part = np.concatenate([part, part[::-1]])
            assert (ix.add(part) == ref.add(part)).all()
        assert len(ix) == len(ref)


def test_new_chunks_compacted_in_order(ctx):
    rng = np.random.default_rng(SEED + 2)
    pool = _rand_ids(rng, 700)
    ids = pool[rng.integers(0, 700, 5000)]
    ch = np.zeros(5000, dtype=_lib.CHUNK_DTYPE)
    ch["offset"] = np.arange(5000) * 1000
    ch["length"] = rng.integers(1, 1000, 5000)
    with ctx.index_create() as ix:
        f, new = ix.add(ids, chunks=ch)
    ref = O.DedupIndex().add(ids)
    assert (f == ref).all()
    assert (new == ch[ref]).all()


def test_device_pipeline_repeated_content(ctx):
    """chunk -> IDs -> dedup, all in HBM: a stream made of one random block
    repeated (the chunker resynchronises, so later copies yield the same
    chunks) plus a changed copy; flags vs the oracle's chunks, IDs and index."""
    base = O.random_bytes(24 << 20, SEED + 3)
    changed = base.copy()
    changed[5 << 20] ^= 0xFF
    data = np.concatenate([base, base, changed, base])
    p = _lib.params(16384, 65536, 262144, 1)
    n = data.size
    dp = ctx.device_alloc(n + 16)
    cap = n // (16384 - 1) + 2
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    d_ids = ctx.device_alloc(cap * 32)
    try:
        ctx.h2d(dp, data)
        k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
        ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)
        with ctx.index_create() as ix:
            f = ix.add(None, d_ids=d_ids, n=k)
            assert len(ix) == int(f.sum())
        chunks = ctx.d2h_chunks(d_out, k)
    finally:
        ctx.device_free(d_ids)
        ctx.device_free(d_out)
        ctx.device_free(dp)
    rc = O.chunk(O.Params(16384, 65536, 262144, 1), data)
    assert len(rc) == k and (chunks["offset"] == rc["offset"]).all()
    ref = O.DedupIndex().add(O.chunk_ids(data, rc, threads=8))
    assert (f == ref).all()
    assert ref.sum() < 0.5 * k  # the repeats were found


def test_incremental_save_path_in_hbm(ctx):
    """Second snapshot with a few changed bytes: chunk -> IDs -> dedup against
    the first snapshot's index -> seal only the new chunks, all in HBM; the new
    chunks are those the oracle's chunks/IDs/index give, sealed as the RFC 8452
    oracle seals them."""
    n = 40 << 20
    data = O.random_bytes(n, SEED + 4)
    changed = data.copy()
    pos = np.array([3 << 20, (17 << 20) + 5, (33 << 20) + 77])
    changed[pos] ^= 0x5A
    p = _lib.params(16384, 65536, 262144, 1)
    cap = n // (16384 - 1) + 2
    dp = ctx.device_alloc(n + 16)
    d_ch = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    d_new = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    d_ids = ctx.device_alloc(cap * 32)
    key = bytes(range(32))
    try:
        with ctx.index_create() as ix:
            ctx.h2d(dp, data)
            k0 = ctx.chunk_device_to_device(p, dp, n, d_ch, cap)
            ctx.chunk_ids(dp, n, (d_ch, k0), ids=d_ids)
            assert ix.add_device(d_ids, k0, d_ch, d_new) == k0
            ctx.h2d(dp, changed)
            k1 = ctx.chunk_device_to_device(p, dp, n, d_ch, cap)
            ctx.chunk_ids(dp, n, (d_ch, k1), ids=d_ids)
            m = ix.add_device(d_ids, k1, d_ch, d_new)
            new = ctx.d2h_chunks(d_new, m)
            nonces = np.arange(12 * m, dtype=np.uint32).astype(np.uint8).reshape(m, 12)
            cap_s = int(new["length"].sum()) + 28 * m
            d_s = ctx.device_alloc(cap_s)
            try:
                oo = ctx.seal_chunks(key, dp, n, new, nonces, d_s, cap_s)
                sealed = ctx.d2h_bytes(d_s, int(oo[-1]))
            finally:
                ctx.device_free(d_s)
    finally:
        for x in (d_ids, d_new, d_ch, dp):
            ctx.device_free(x)
    P = O.Params(16384, 65536, 262144, 1)
    r0, r1 = O.chunk(P, data), O.chunk(P, changed)
    ix_ref = O.DedupIndex()
    ix_ref.add(O.chunk_ids(data, r0, threads=8))
    flags = ix_ref.add(O.chunk_ids(changed, r1, threads=8))
    ref_new = r1[flags]
    assert 0 < m == len(ref_new) and (new["offset"] == ref_new["offset"]).all()
    assert (new["length"] == ref_new["length"]).all()
    ref, _ = O.seal_blobs(key, changed, ref_new["offset"], ref_new["length"], nonces)
    assert sealed.tobytes() == ref.tobytes()
