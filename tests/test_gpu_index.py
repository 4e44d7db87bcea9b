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
