"""GPU chunk IDs (BLAKE3 of every chunk, libmcdc.so mcdc_chunk_ids_device)
against the oracle restatement (oracle/blake3_oracle.c), byte for byte.

The reference computes one ID per chunk at
/root/reference/src/archiver/processor.rs:184 (ID::from_content ->
src/utils/mod.rs:62-68).  Covers the reference KAT bytes placed in HBM, every
leaf/block edge length, unaligned chunk offsets, chunks of <= 16 leaves
(finished in k_b3_leaves) and of many groups (k_b3_tree), the P16 and P512
chunkers' real boundary lists, device- and host-resident chunk lists and ID
arrays, and out-of-range chunks.
"""
import json
import os

import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x6d61706163686521


def _chunks(pairs):
    c = np.zeros(len(pairs), dtype=_lib.CHUNK_DTYPE)
    for i, (o, n) in enumerate(pairs):
        c[i]["offset"], c[i]["length"] = o, n
    return c


def _device_bytes(ctx, data: np.ndarray, pad: int = 0):
    dp = ctx.device_alloc(data.size + pad + 16)
    ctx.h2d(dp, data)
    return dp


def test_reference_kat_on_device(ctx):
    kats = json.load(open(os.path.join(HERE, "golden", "blake3_kat.json")))
    blobs = []
    for k in kats:
        blobs.append(bytes(i % 251 for i in range(k["pattern_i_mod_251"])) if "pattern_i_mod_251" in k
                     else bytes.fromhex(k["input_hex"]))
    data = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum([len(b) for b in blobs])[:-1]])
    dp = _device_bytes(ctx, data)
    try:
        ids = ctx.chunk_ids(dp, data.size, _chunks(list(zip(offs, map(len, blobs)))))
    finally:
        ctx.device_free(dp)
    for k, h in zip(kats, ids):
        assert bytes(h).hex() == k["blake3"], k["source"]


def test_edge_lengths_and_alignments(ctx):
    lens = [0, 1, 3, 4, 5, 63, 64, 65, 127, 128, 1023, 1024, 1025, 2047, 2048, 2049, 3071, 3073, 15 * 1024,
            16 * 1024 - 1, 16 * 1024, 16 * 1024 + 1, 17 * 1024, 31 * 1024 + 5, 32 * 1024, 33 * 1024 + 63,
            48 * 1024, 64 * 1024 + 1, 100_000, 262_144, 300_001]
    pairs, pos = [], 0
    for i, n in enumerate(lens):
        pos += i % 7  # gaps -> every offset alignment mod 16
        pairs.append((pos, n))
        pos += n
    data = O.random_bytes(pos, SEED + 1)
    dp = _device_bytes(ctx, data)
    try:
        got = ctx.chunk_ids(dp, data.size, _chunks(pairs))
    finally:
        ctx.device_free(dp)
    ref = O.chunk_ids(data, _chunks(pairs), threads=8)
    bad = [i for i in range(len(pairs)) if not (got[i] == ref[i]).all()]
    assert not bad, [(lens[i], pairs[i][0] % 16) for i in bad]


@pytest.mark.parametrize("p", [(16384, 65536, 262144, 1), (524288, 1048576, 8388608, 1), (64, 256, 1024, 1)],
                         ids=lambda p: "/".join(map(str, p)))
def test_chunker_boundaries_device_resident(ctx, p):
    """The real pipeline: chunk in HBM, boundary list stays in HBM, IDs in HBM."""
    n = (96 << 20) + 4321
    prm = _lib.params(*p)
    dp = ctx.device_alloc(n + 16)
    cap = n // (p[0] - 1) + 2
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    d_ids = ctx.device_alloc(cap * 32)
    try:
        ctx.fill_random(dp, n, SEED + 2)
        k = ctx.chunk_device_to_device(prm, dp, n, d_out, cap)
        ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)
        got = ctx.d2h_bytes(d_ids, 32 * k).reshape(k, 32)
        chunks = ctx.d2h_chunks(d_out, k)
    finally:
        ctx.device_free(d_ids)
        ctx.device_free(d_out)
        ctx.device_free(dp)
    host = O.random_bytes(n, SEED + 2)
    ref = O.chunk_ids(host, O.chunk(O.Params(*p), host), threads=8)
    assert len(chunks) == len(ref)
    assert (got == ref).all()


def test_host_chunk_list_and_host_ids(ctx):
    n = 20 << 20
    data = O.random_bytes(n, SEED + 3)
    dp = _device_bytes(ctx, data)
    try:
        c = O.chunk(O.P16, data)
        got = ctx.chunk_ids(dp, n, c)
    finally:
        ctx.device_free(dp)
    assert (got == O.chunk_ids(data, c, threads=8)).all()


def test_out_of_range_chunk_rejected(ctx):
    dp = ctx.device_alloc(4096)
    try:
        with pytest.raises(_lib.McdcError) as ei:
            ctx.chunk_ids(dp, 4096, _chunks([(0, 100), (4000, 200)]))
        assert ei.value.code == _lib.MCDC_E_INVALID
        ids = ctx.chunk_ids(dp, 4096, _chunks([]))
        assert ids.shape == (0, 32)
    finally:
        ctx.device_free(dp)


def test_overlapping_and_repeated_chunks(ctx):
    """A list whose chunks overlap or repeat (not a chunker output, but the
    header allows it): its 16-KiB leaf groups exceed the disjoint-chunk bound
    the grid is sized by; the kernels write nothing over the bound and the
    call re-hashes with the exact group count — every ID still exact."""
    n = 6 << 20
    data = O.random_bytes(n, SEED + 9)
    pairs = [(0, n)] * 5 + [(17, n - 17), (1 << 20, 3 << 20), (1 << 20, 3 << 20), (5, 70_000), (5, 70_000)]
    pairs += [(o, 300_000) for o in range(0, n - 300_000, 99_991)]
    c = _chunks(pairs)
    dp = _device_bytes(ctx, data)
    try:
        got = ctx.chunk_ids(dp, n, c)
        again = ctx.chunk_ids(dp, n, c)  # the grown workspace is reused
    finally:
        ctx.device_free(dp)
    ref = O.chunk_ids(data, c, threads=8)
    assert (got == ref).all() and (again == ref).all()


def test_many_tail_lengths_in_list_order(ctx):
    """Thousands of chunks whose last 16-KiB groups have every block count,
    listed out of offset order: the tail groups are counting-sorted across
    many workgroups (per-block bin reservations), full groups come first,
    and waves whose lanes have unequal loops still hash every lane exactly."""
    rng = np.random.default_rng(SEED + 11)
    lens = np.concatenate([rng.integers(0, 70_000, 5000), np.arange(0, 16385, 64), 16384 * rng.integers(1, 5, 200),
                           np.array([0, 1, 63, 64, 65, 16383, 16385])]).astype(np.int64)
    gaps = rng.integers(0, 16, lens.size)
    offs = np.cumsum(np.concatenate([[0], lens[:-1] + gaps[:-1]])) + gaps[0]
    n = int(offs[-1] + lens[-1])
    perm = rng.permutation(lens.size)
    c = _chunks(list(zip(offs[perm].tolist(), lens[perm].tolist())))
    data = O.random_bytes(n, SEED + 11)
    dp = _device_bytes(ctx, data)
    try:
        got = ctx.chunk_ids(dp, n, c)
    finally:
        ctx.device_free(dp)
    ref = O.chunk_ids(data, c, threads=8)
    bad = np.nonzero(~(got == ref).all(axis=1))[0]
    assert bad.size == 0, [(int(c["offset"][i]), int(c["length"][i])) for i in bad[:10]]


def test_large_chunks_tree_paths(ctx):
    """Chunks of more than 16 groups go to the wave-parallel tree
    (k_b3_tree_wide, mcdc_blake3.hip): up to kTreeWaveMax = 512 nodes in LDS,
    the levels above that in place in HBM first.  256 KiB + 1 (17 groups),
    1 MiB, 8 MiB - 16 KiB + 1 (512 groups, an odd last group), 8 MiB
    (mapache's max, 512 groups: all in LDS), 8 MiB + 1 (513 groups: one HBM
    level, an odd one), 16 MiB + 1 (a pack's size: 1025 groups), 16 MiB (1024,
    even levels), 24 MiB, 40 MiB + 3 and 64 MiB + 16 KiB + 5 (3-4 HBM levels,
    odd counts), at odd offsets; the IDs equal the specification's tree
    (the pack ID is calculate_hash of the pack, src/utils/mod.rs:62-68)."""
    lens = [(256 << 10) + 1, 1 << 20, (8 << 20) - (16 << 10) + 1, 8 << 20, (8 << 20) + 1, (16 << 20) + 1,
            16 << 20, 24 << 20, (40 << 20) + 3, (64 << 20) + (16 << 10) + 5]
    pairs, pos = [], 5
    for n_ in lens:
        pairs.append((pos, n_))
        pos += n_ + 3
    data = O.random_bytes(pos, SEED + 12)
    dp = _device_bytes(ctx, data)
    try:
        got = ctx.chunk_ids(dp, data.size, _chunks(pairs))
    finally:
        ctx.device_free(dp)
    ref = O.chunk_ids(data, _chunks(pairs), threads=8)
    bad = [lens[i] for i in range(len(pairs)) if not (got[i] == ref[i]).all()]
    assert not bad, bad
