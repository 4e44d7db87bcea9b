"""GPU parity: the MI355X path (libmcdc.so through the C ABI) against the
oracle restatement, bit for bit (offsets, lengths, ChunkData.hash).

Covers the edge cases the reference's call semantics imply
(/root/reference/src/archiver/processor.rs:160-205: per-file restart, tail
chunk, empty input) and every internal path of the GPU pipeline: the
windowed-candidate scan, run overflow (dense candidates -> on-the-fly
rescans), speculative segment chains that merge, skip a segment, or never
merge (serial fallback), unaligned device pointers and batches.
"""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x6d61706163686521
PARAMS = [(16384, 65536, 262144, 1), (524288, 1048576, 8388608, 1), (64, 256, 1024, 1),
          (4096, 16384, 65536, 2), (65, 300, 1111, 3), (1024, 4096, 16384, 0), (4095, 8191, 65535, 1)]


def _same(g, r):
    assert len(g) == len(r), (len(g), len(r))
    if len(g):
        bad = np.nonzero((g["offset"] != r["offset"]) | (g["length"] != r["length"]) | (g["hash"] != r["hash"]))[0]
        assert bad.size == 0, f"first mismatch at {bad[0]}: gpu {g[bad[0]]} ref {r[bad[0]]}"


@pytest.mark.parametrize("p", PARAMS, ids=lambda p: "/".join(map(str, p)))
def test_random_sizes(ctx, p):
    for n in [0, 1, 2, 47, 48, 4095, 4096, 4097, 65535, 65536, 262145, (1 << 20) + 3, (7 << 20) + 1,
              2 * p[2] + 1, 3 * p[2]]:
        d = O.random_bytes(n, SEED + n)
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


def test_large_random_host(ctx):
    d = O.random_bytes(300 << 20, SEED)
    for p in PARAMS[:2]:
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


@pytest.mark.parametrize("misalign", [0, 1, 3, 7, 8, 13, 15])
def test_device_pointer_any_alignment(ctx, misalign):
    n = (64 << 20) + 12345
    dp = ctx.device_alloc(n + 64)
    try:
        ctx.fill_random(dp, n + 64, SEED)
        h = O.random_bytes(n, SEED, pos=misalign)
        p = PARAMS[0]
        _same(ctx.chunk_device(_lib.params(*p), dp + misalign, n), O.chunk(O.Params(*p), h))
    finally:
        ctx.device_free(dp)


def test_batch_many_files(ctx):
    rng = np.random.default_rng(3)
    sizes = [0, 1, 5, 16383, 16384, 16385, 100_000, 262_144, 262_145, 1 << 20, (3 << 20) + 7, 9 << 20]
    sizes += rng.integers(0, 2 << 20, 200).tolist()
    files = [O.random_bytes(int(s), 1000 + i) for i, s in enumerate(sizes)]
    for p in PARAMS[:4]:
        g, gc = ctx.chunk_batch(_lib.params(*p), files)
        r, rc = O.chunk_files(O.Params(*p), files, threads=4)
        assert (gc == rc).all()
        _same(g, r)


def test_batch_device_arena(ctx):
    sizes = [70_000, 0, 5 << 20, 123, (2 << 20) + 1, 262_144]
    gaps = [0, 16, 1, 4095, 0, 7]
    offs, pos = [], 0
    for s, gp in zip(sizes, gaps):
        pos += gp
        offs.append(pos)
        pos += s
    dp = ctx.device_alloc(pos + 64)
    try:
        ctx.fill_random(dp, pos + 64, SEED)
        p = PARAMS[0]
        g, gc = ctx.chunk_batch_device(_lib.params(*p), dp, offs, sizes)
        files = [O.random_bytes(s, SEED, pos=o) for o, s in zip(offs, sizes)]
        r, rc = O.chunk_files(O.Params(*p), files)
        assert (gc == rc).all()
        _same(g, r)
    finally:
        ctx.device_free(dp)


def _find_dense_byte(p):
    """A constant byte whose windowed hash passes mask_l: every position becomes a candidate."""
    _, _, masks = O.tables()
    g = O.gear_md5()
    import math
    ml = masks[round(math.log2(p[1])) - p[3]]
    for b in range(256):
        w = sum(g[b] << k for k in range(48)) & ((1 << 48) - 1)
        if w & ml == 0:
            return b
    return None


@pytest.mark.parametrize("p", PARAMS, ids=lambda p: "/".join(map(str, p)))
def test_adversarial_patterns(ctx, p):
    rng = np.random.default_rng(7)
    pats = [np.zeros(6 << 20, np.uint8),                                     # forced cuts only
            np.full(3 << 20, 0xa5, np.uint8),
            np.tile(rng.integers(0, 256, 13, dtype=np.uint8), 300_000),     # periodic, dense or empty
            np.tile(rng.integers(0, 256, 5000, dtype=np.uint8), 900),
            np.frombuffer(b"all work and no play makes jack a dull boy\n" * 90_000, np.uint8)]
    b = _find_dense_byte(p)
    if b is not None:  # every position a candidate -> every run overflows -> on-the-fly rescans
        pats.append(np.full(2 << 20, b, np.uint8))
    for d in pats:
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


def test_forced_stretch_crossed_by_the_continuation(ctx):
    """Random prefix sets a forced-cut phase the segment-start speculation never
    matches; the continuation takes the 48 MiB zero run in a few repeated
    entries (forced_run) and merges in the random data behind it."""
    p = PARAMS[0]
    d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(48 << 20, np.uint8), O.random_bytes(3 << 20, 10)])
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    assert ctx.timing()["fallback_files"] == 0


@pytest.mark.parametrize("p", PARAMS, ids=lambda p: "/".join(map(str, p)))
def test_long_forced_stretch_emitted_by_the_grid(ctx, p):
    """A continuation of more than kEmitInline (256) chunks: 80 MiB (16/64/256)
    or 2.2 GiB (512K/1M/8M) of zeros out of phase, emitted by k_emit_long; and
    the same stretch twice in one file with random data between and behind."""
    z = (80 << 20) if p[2] <= (256 << 10) else (2200 << 20)
    d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(z, np.uint8), O.random_bytes(3 << 20, 10)])
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    assert ctx.timing()["fallback_files"] == 0
    if p[2] <= (256 << 10):
        d = np.concatenate([O.random_bytes(777_777, 3), np.zeros(z, np.uint8), O.random_bytes(5 << 20, 4),
                            np.zeros(z + 12345, np.uint8), O.random_bytes(1 << 20, 5)])
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


def test_stretch_beyond_link_reach_takes_the_serial_fallback(ctx):
    """1.2 GiB of zeros out of phase: more than 64 continuation entries of at
    most 16 MiB each, so the file is walked by k_fallback (which takes forced
    stretches whole as well)."""
    p = PARAMS[0]
    d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(1200 << 20, np.uint8), O.random_bytes(3 << 20, 10)])
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    assert ctx.timing()["fallback_files"] == 1


@pytest.mark.parametrize("p", PARAMS, ids=lambda p: "/".join(map(str, p)))
def test_mixed_zero_extents_and_runs(ctx, p):
    """Disk-image-like layouts: random and zero extents alternating (1 and 9 MiB),
    runs of one byte value (1 B .. 64 KiB), sparse random extents."""
    rng = np.random.default_rng(21)
    n = 96 << 20
    for k in (1 << 20, 9 << 20):
        d = O.random_bytes(n, 31)
        for b in range(k, n, 2 * k):
            d[b:b + k] = 0
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    lens = rng.integers(1, 65536, n // 32768 * 2)
    vals = rng.integers(0, 256, len(lens)).astype(np.uint8)
    d = np.repeat(vals, lens)[:n]
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    d = np.zeros(n, np.uint8)
    for b in range(12345, n, 24 << 20):
        d[b:b + (1 << 20)] = O.random_bytes(1 << 20, b)[: len(d[b:b + (1 << 20)])]
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


def test_skipped_segment_walk(ctx):
    """A zero run about one segment long: the continuation crosses a whole
    segment before merging (k_walk's serial link-following)."""
    p = PARAMS[0]
    for zlen in [1_310_720 - 5000, 1_310_720 + 70_000, 2 * 1_310_720 + 1]:
        d = np.concatenate([O.random_bytes(1_000_001, 11), np.zeros(zlen, np.uint8), O.random_bytes(5 << 20, 12)])
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


def test_full_size_digest_and_invariants(ctx):
    """8 GiB device-resident stream: digest of (offset, length) equals the
    oracle's over the regenerated bytes; every chunk within [min, max] except
    the tail; lengths sum to n."""
    n = 8 << 30
    dp = ctx.device_alloc(n)
    try:
        ctx.fill_random(dp, n, SEED)
        p = PARAMS[0]
        g = ctx.chunk_device(_lib.params(*p), dp, n)
    finally:
        ctx.device_free(dp)
    assert int(g["length"].sum()) == n
    assert (g["offset"][1:] == np.cumsum(g["length"])[:-1]).all()
    assert g["length"][:-1].min() >= p[0] and g["length"].max() <= p[2]
    h = O.random_bytes(n, SEED)
    k, dig = O.chunk_digest(O.Params(*p), h)
    assert k == len(g)
    assert _lib.digest(g) == dig
    # spot-check hashes on a sample of chunks against cut_gear restarted at the chunk
    for i in np.linspace(0, len(g) - 2, 64).astype(int):
        o = int(g["offset"][i])
        hh, cc = O.cut_gear(O.Params(*p), h[o:o + p[2] + 1])
        assert (hh, cc) == (int(g["hash"][i]), int(g["length"][i]))


def test_python_mirror_fastcdc_and_streamcdc(ctx):
    import io
    from mapache_amd import FastCDC, StreamCDC
    d = O.random_bytes(50 << 20, 21)
    ref = O.chunk(O.P512, d)
    got = list(FastCDC(d, 524288, 1048576, 8388608, ctx=ctx))
    assert [(c.offset, c.length, c.hash) for c in got] == list(zip(ref["offset"].tolist(), ref["length"].tolist(),
                                                                  ref["hash"].tolist()))
    stream = list(StreamCDC(io.BytesIO(d.tobytes()), 524288, 1048576, 8388608, window=20 << 20, ctx=ctx))
    assert [(c.offset, c.length, c.hash) for c in stream] == [(c.offset, c.length, c.hash) for c in got]
    assert b"".join(c.data for c in stream) == d.tobytes()


def test_cpp_host_api_gpu():
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "test_host_api")
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def test_timing_reported(ctx):
    d = O.random_bytes(64 << 20, 5)
    ctx.chunk_host(_lib.params(*PARAMS[0]), d)
    t = ctx.timing()
    assert t["bytes"] == d.size and t["chunks"] > 0
    assert 0 < t["scan_ms"] <= t["device_ms"] and t["h2d_ms"] > 0


@pytest.fixture
def knob_ctx(monkeypatch):
    """A fresh context created after the test sets its MCDC_* switches (a
    context reads them once, at mcdc_ctx_create)."""
    made = []

    def make(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, str(v))
        c = _lib.Context(0, 4 << 30)
        made.append(c)
        return c
    yield make
    for c in made:
        c.close()


@pytest.mark.parametrize("direct", [1, 0])
def test_pinned_output_written_directly(knob_ctx, direct):
    """A pinned caller array is written by k_emit over PCIe (no staging copy;
    MCDC_PINNED_DIRECT=0: emitted into HBM and copied by one DMA): same result
    as the pageable path; a too-small pinned array reports MCDC_E_CAPACITY
    with the required count."""
    ctx = knob_ctx(MCDC_PINNED_DIRECT=direct)
    n = (96 << 20) + 777
    dp = ctx.device_alloc(n)
    try:
        ctx.fill_random(dp, n, SEED + 3)
        p = _lib.params(*PARAMS[0])
        ref = ctx.chunk_device(p, dp, n)
        pin = ctx.pinned_out(len(ref) + 8)
        got = ctx.chunk_device(p, dp, n, out=pin)
        assert len(got) == len(ref) and (got == ref).all()
        small = pin[: len(ref) - 1]
        with pytest.raises(_lib.McdcError) as ei:
            ctx.chunk_device(p, dp, n, out=small)
        assert ei.value.code == -3
        _same(ref, O.chunk(O.Params(*PARAMS[0]), O.random_bytes(n, SEED + 3)))
    finally:
        ctx.device_free(dp)


def test_device_output_stays_in_hbm(ctx):
    """A device `out` array: k_emit writes the boundary list in HBM (the
    bench's headline configuration); identical to the host-output path and the
    oracle; a too-small device array reports MCDC_E_CAPACITY with the count."""
    n = (80 << 20) + 4321
    p = _lib.params(*PARAMS[0])
    dp = ctx.device_alloc(n)
    cap = n // (p.min_size - 1) + 2
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(dp, n, SEED + 4)
        k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
        got = ctx.d2h_chunks(d_out, k)
        ref = O.chunk(O.Params(*PARAMS[0]), O.random_bytes(n, SEED + 4))
        _same(got, ref)
        _same(ctx.chunk_device(p, dp, n), ref)
        with pytest.raises(_lib.McdcError) as ei:
            ctx.chunk_device_to_device(p, dp, n, d_out, k - 1)
        assert ei.value.code == -3
    finally:
        ctx.device_free(d_out)
        ctx.device_free(dp)


def test_batch_device_to_device(ctx):
    sizes = [0, 17, 16385, 300_000, 5 << 20, 1, (2 << 20) + 9]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64) + 3
    n = int(sum(sizes)) + 64
    p = _lib.params(*PARAMS[0])
    arena = ctx.device_alloc(n)
    cap = sum(s // (p.min_size - 1) + 2 for s in sizes)
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(arena, n, SEED + 5)
        total, counts = ctx.chunk_batch_device_to_device(p, arena, offs, sizes, d_out, cap)
        host = O.random_bytes(n, SEED + 5)
        ref, rc = O.chunk_files(O.Params(*PARAMS[0]), [host[int(o):int(o) + s] for o, s in zip(offs, sizes)])
        _same(ctx.d2h_chunks(d_out, total), ref)
        assert (counts == rc).all()
    finally:
        ctx.device_free(d_out)
        ctx.device_free(arena)


def test_plan_reuse_across_layouts(ctx):
    """The segment plan is cached per (file ranges, params): alternating
    lengths and parameter sets must re-plan, repeats must reuse it."""
    n = 40 << 20
    dp = ctx.device_alloc(n)
    try:
        ctx.fill_random(dp, n, SEED + 6)
        h = O.random_bytes(n, SEED + 6)
        for ln, pi in [(n, 0), (n, 0), (n - 999, 0), (n, 1), (n, 0), (n - 999, 3), (n - 999, 3), (n, 2)]:
            _same(ctx.chunk_device(_lib.params(*PARAMS[pi]), dp, ln), O.chunk(O.Params(*PARAMS[pi]), h[:ln]))
    finally:
        ctx.device_free(dp)


@pytest.fixture(scope="module")
def staged():
    """A context forced into the staged pipeline (scan in 4 parts, resolution
    of the scanned prefix overlapping the next part) on small inputs: a round =
    16 tiles (4 MiB), parts of 1, 3 and 9 rounds at the end."""
    mp = pytest.MonkeyPatch()
    for k, v in (("MCDC_PARTS", 4), ("MCDC_TAIL_ROUNDS", 1), ("MCDC_PART_TILES", 16), ("MCDC_MIN_ROUNDS", 0)):
        mp.setenv(k, str(v))
    c = _lib.Context(0, 4 << 30)
    mp.undo()  # the context keeps the switches; later contexts do not see them
    yield c
    c.close()


@pytest.mark.parametrize("p", PARAMS, ids=lambda p: "/".join(map(str, p)))
def test_staged_pipeline_random(staged, p):
    ctx = staged
    n = (200 << 20) + 12345
    d = O.random_bytes(n, SEED + 7)
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    assert ctx.timing()["scan_launches"] == 4


def test_staged_pipeline_dirty_paths(staged):
    ctx = staged
    """Skipped segments and never-merging chains inside a staged call: the
    incremental pass flags them and the general resolution redoes the call."""
    p = PARAMS[0]
    d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(48 << 20, np.uint8), O.random_bytes(90 << 20, 10)])
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    assert ctx.timing()["fallback_files"] == 1
    for zlen in [1_310_720 - 5000, 1_310_720 + 70_000, 2 * 1_310_720 + 1]:
        d = np.concatenate([O.random_bytes(150 << 20, 11), np.zeros(zlen, np.uint8), O.random_bytes(60 << 20, 12)])
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))


def test_staged_pipeline_batch(staged):
    ctx = staged
    rng = np.random.default_rng(8)
    sizes = [int(x) for x in rng.integers(0, 3 << 20, 150)] + [0, 1, 16384, 40 << 20]
    files = [O.random_bytes(s, 500 + i) for i, s in enumerate(sizes)]
    out, counts = ctx.chunk_batch(_lib.params(*PARAMS[0]), files)
    ref, rc = O.chunk_files(O.Params(*PARAMS[0]), files)
    _same(out, ref)
    assert (counts == rc).all()


def test_call_larger_than_context_fails_loudly():
    """A context bounds the bytes of one call (max_bytes sizes its workspace):
    a larger call reports MCDC_E_TOOBIG instead of allocating past it; a
    call within the bound on the same context still works."""
    small = _lib.Context(0, 1 << 20)
    try:
        d = O.random_bytes((1 << 20) + 1, 41)
        with pytest.raises(_lib.McdcError) as e:
            small.chunk_host(_lib.params(*PARAMS[2]), d)
        assert e.value.code == -6
        _same(small.chunk_host(_lib.params(*PARAMS[2]), d[:1 << 20]), O.chunk(O.Params(*PARAMS[2]), d[:1 << 20]))
    finally:
        small.close()


@pytest.mark.parametrize("pieces,cold", [(1, 0), (2, 0), (2, 1), (4, 0), (4, 1)])
def test_scan_lane_pieces(knob_ctx, pieces, cold):
    """Every lane-piece variant of the scan (a 4 KiB run hashed by 1, 2 or 4
    lanes; the library picks by call size), warm (each piece re-reads the 48
    bytes before it) and cold (first 48 positions re-walked at tile end from
    the previous lane's hash), on the same inputs: edge sizes around the tile
    and run grid, a partial last tile, overflowed runs whose candidates come
    from several lanes, and a batch of ragged files."""
    ctx = knob_ctx(MCDC_SCAN_PIECES=pieces, MCDC_SCAN_COLD=cold)
    for p in [PARAMS[0], PARAMS[2], PARAMS[6]]:
        for n in [47, 1023, 1024, 1025, 4097, (256 << 10) + 1, (64 << 20) + 4096 * 17 + 3, (200 << 20) + 12345]:
            d = O.random_bytes(n, SEED + 31 * n)
            _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
        b = _find_dense_byte(p)
        if b is not None:
            d = np.full((5 << 20) + 77, b, np.uint8)
            _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    rng = np.random.default_rng(11)
    files = [O.random_bytes(int(s), 500 + i) for i, s in enumerate(rng.integers(0, 3 << 20, 120))]
    p = PARAMS[0]
    g, gc = ctx.chunk_batch(_lib.params(*p), files)
    r, rc = O.chunk_files(O.Params(*p), files, threads=4)
    assert (gc == rc).all()
    _same(g, r)


def _segment_bytes(p):
    """The library's segment size (mcdc_api.hip segment_bytes): ~4 expected
    chunks on the lane walk (max <= 64 runs of 4 KiB), 16 on the group walk."""
    k = 4 if p[2] <= 64 * 4096 else 16
    z = max(2 * p[2], k * (p[0] + p[1]))
    return (z + 4095) // 4096 * 4096


@pytest.mark.parametrize("p", [PARAMS[0], PARAMS[2], PARAMS[3], PARAMS[6]], ids=lambda p: "/".join(map(str, p)))
def test_short_last_segment(ctx, p):
    """Files of k segments plus a short remainder: the previous segment's
    continuation often runs to the end of the file without meeting the last
    segment's speculative chain; the clean path then takes the last segment
    off the chain (count 0) instead of re-resolving the whole call."""
    z = _segment_bytes(p)
    rems = sorted({1, 47, 100, 5000, p[0] - 1, p[0], p[0] + 1, p[1], p[2] - 1, p[2] + 1, 3 * p[2]})
    files = []
    for k in (1, 2):
        for r in rems:
            d = O.random_bytes(k * z + r, SEED + 97 * r + k)
            _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
            files.append(d)
    g, gc = ctx.chunk_batch(_lib.params(*p), files)
    r_, rc = O.chunk_files(O.Params(*p), files, threads=4)
    assert (gc == rc).all()
    _same(g, r_)


@pytest.mark.parametrize("walk", [0, 2])
def test_walk_variants(knob_ctx, walk):
    """Both chain walks on the same inputs: the group walk (MCDC_LANE_WALK=0,
    16 lanes per chain) where the library would take the lane walk, and the
    lane walk forced (=2) where it would not (mapache's 512K/1M/8M): sizes,
    adversarial patterns (overflowed runs hand segments back to the group
    walk, forced stretches run into kContMax) and batches of ragged files."""
    ctx = knob_ctx(MCDC_LANE_WALK=walk)
    rng = np.random.default_rng(23)
    for p in PARAMS:
        for n in [0, 47, 4097, (1 << 20) + 3, 2 * p[2] + 1, 5 * p[2] + 77, (90 << 20) + 5]:
            d = O.random_bytes(n, SEED + 3 * n + walk)
            _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
            if n:
                assert ctx.timing()["lane_walk"] == (1 if walk == 2 else 0)
        pats = [np.zeros(6 << 20, np.uint8), np.tile(rng.integers(0, 256, 13, dtype=np.uint8), 300_000),
                np.concatenate([O.random_bytes(3 << 20, 5), np.zeros(9 << 20, np.uint8), O.random_bytes(1 << 20, 6)])]
        b = _find_dense_byte(p)
        if b is not None:
            pats.append(np.full(2 << 20, b, np.uint8))
        for d in pats:
            _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    files = [O.random_bytes(int(s), 900 + i) for i, s in enumerate(rng.integers(0, 3 << 20, 90))]
    for p in PARAMS[:3]:
        g, gc = ctx.chunk_batch(_lib.params(*p), files)
        r, rc = O.chunk_files(O.Params(*p), files, threads=4)
        assert (gc == rc).all()
        _same(g, r)


def test_lane_walk_is_the_default(ctx):
    """At max <= 256 KiB a single-part call walks chains one lane per chain;
    on random data no segment is handed back to the group walk."""
    p = PARAMS[0]
    d = O.random_bytes(64 << 20, SEED + 99)
    _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    t = ctx.timing()
    assert t["lane_walk"] == 1 and t["handed_back"] == 0, t
    ctx.chunk_host(_lib.params(*PARAMS[1]), d)
    assert ctx.timing()["lane_walk"] == 0


def test_long_stretch_hashes_repeated(ctx):
    """The reproducer of the LDS-table item: 80 MiB of zeros
    after a random prefix at 64/256/1024, whose ~80 000 forced chunks are
    emitted by k_emit_long, chunked 60 times in one process.  With GEAR read
    from an LDS copy this sequence lost whole waves of ChunkData.hash values
    in 1.5-5 % of calls (19-44 % under a rocprofv3 --pmc pass); the product
    reads the global table and must be exact in every call."""
    p = (64, 256, 1024, 1)
    d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(80 << 20, np.uint8), O.random_bytes(3 << 20, 10)])
    ref = O.chunk(O.Params(*p), d)
    n = d.size
    dp = ctx.device_alloc(n + 64)
    cap = n // (p[0] - 1) + 2
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.h2d(dp, d)
        bad_calls = []
        for k in range(60):
            c = ctx.chunk_device_to_device(_lib.params(*p), dp, n, d_out, cap)
            g = ctx.d2h_chunks(d_out, c)
            if not (len(g) == len(ref) and (g == ref).all()):
                bad_calls.append(k)
    finally:
        ctx.device_free(d_out)
        ctx.device_free(dp)
    assert not bad_calls, f"calls with wrong output: {bad_calls}"


def test_batch_device_ranges_validated(ctx):
    """mcdc_chunk_batch_device: files in any order are fine, including a last
    file that does not end furthest (the scan is enqueued on the last file's
    end before the ranges are read; the call then restarts with the true
    span); overlapping ranges, offset + length overflow and an arena span
    beyond the context's max_bytes are rejected (MCDC_E_INVALID /
    MCDC_E_TOOBIG)."""
    n = 8 << 20
    dp = ctx.device_alloc(n)
    p = _lib.params(*PARAMS[0])
    try:
        ctx.fill_random(dp, n, SEED + 12)
        host = O.random_bytes(n, SEED + 12)
        offs, lens = [5 << 20, 0, 1 << 20, 7 << 20], [1 << 20, 1 << 20, 0, 1 << 20]
        g, gc = ctx.chunk_batch_device(p, dp, offs, lens)
        r, rc = O.chunk_files(O.Params(*PARAMS[0]), [host[o:o + ln] for o, ln in zip(offs, lens)])
        assert (gc == rc).all()
        _same(g, r)
        for offs, lens in (([6 << 20, 0, 2 << 20], [2 << 20, 1 << 20, (1 << 20) + 3]),  # the last ends at 3 MiB
                           ([(7 << 20) + 5, 11, 3 << 20, 0], [(1 << 20) - 5, 2 << 20, 1 << 20, 0])):
            for _ in range(2):  # (twice: the second call repeats the layout)
                g, gc = ctx.chunk_batch_device(p, dp, offs, lens)
                r, rc = O.chunk_files(O.Params(*PARAMS[0]), [host[o:o + ln] for o, ln in zip(offs, lens)])
                assert (gc == rc).all()
                _same(g, r)
        for offs, lens in (([0, 1 << 20], [(1 << 20) + 1, 5]), ([100, 50], [100, 100])):
            with pytest.raises(_lib.McdcError) as ei:
                ctx.chunk_batch_device(p, dp, offs, lens)
            assert ei.value.code == _lib.MCDC_E_INVALID
        with pytest.raises(_lib.McdcError) as ei:
            ctx.chunk_batch_device(p, dp, [2**64 - 10], [100])
        assert ei.value.code == _lib.MCDC_E_INVALID
    finally:
        ctx.device_free(dp)
    small = _lib.Context(0, 1 << 20)
    try:  # two 256 KiB files 4 MiB apart: 512 KiB of data, a 4.25 MiB span
        dq = small.device_alloc(5 << 20)
        try:
            with pytest.raises(_lib.McdcError) as ei:
                small.chunk_batch_device(p, dq, [0, 4 << 20], [256 << 10, 256 << 10])
            assert ei.value.code == _lib.MCDC_E_TOOBIG
            with pytest.raises(_lib.McdcError) as ei:  # (the last file ends first: found after the scan's launch)
                small.chunk_batch_device(p, dq, [4 << 20, 0], [256 << 10, 256 << 10])
            assert ei.value.code == _lib.MCDC_E_TOOBIG
            g, gc = small.chunk_batch_device(p, dq, [0], [256 << 10])  # (the context still works)
            assert gc.sum() == len(g) > 0
        finally:
            small.device_free(dq)
    finally:
        small.close()


def test_pageable_staging_sizes(ctx):
    """Host entry points from pageable memory: the staging copy is split over
    the copy pool's threads and two pinned slabs; every byte must arrive for
    sizes whose per-thread shares do not divide evenly (8 044 034 lost its
    last 2 bytes to a rounding error once), around the 4 MiB hand-off
    threshold, across the 256 MiB slab edge, and for batches of many files."""
    p = PARAMS[2]
    for n in [(4 << 20) - 1, 4 << 20, (4 << 20) + 1, 8_044_034, 8 * 1_005_504 + 7, (256 << 20) + 3, (512 << 20) - 5]:
        d = O.random_bytes(n, SEED + n)
        _same(ctx.chunk_host(_lib.params(*p), d), O.chunk(O.Params(*p), d))
    rng = np.random.default_rng(19)
    files = [O.random_bytes(int(s), 700 + i) for i, s in enumerate(rng.integers(0, 9 << 20, 70))]
    g, gc = ctx.chunk_batch(_lib.params(*p), files)
    r, rc = O.chunk_files(O.Params(*p), files, threads=8)
    assert (gc == rc).all()
    _same(g, r)


def _arena_files(rng, sizes, gaps):
    """Host bytes of files laid out in one arena with the given gaps before
    each; returns (arena bytes, offsets, lengths, per-file arrays)."""
    parts, offs, at = [], [], 0
    files = []
    for i, (s, g) in enumerate(zip(sizes, gaps)):
        if g:
            parts.append(rng.integers(0, 256, int(g), dtype=np.uint8))
            at += int(g)
        d = O.random_bytes(int(s), SEED + 7919 * i + int(s))
        files.append(d)
        parts.append(d)
        offs.append(at)
        at += int(s)
    arena = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return arena, np.array(offs, np.uint64), np.array([int(s) for s in sizes], np.uint64), files


def _batch_device_calls(ctx, p, arena, offs, lens, calls):
    """`calls` calls of mcdc_chunk_batch_device on one uploaded arena."""
    dp = ctx.device_alloc(arena.size + 16)
    try:
        ctx.h2d(dp, arena)
        return [ctx.chunk_batch_device(_lib.params(*p), dp, offs, lens) for _ in range(calls)]
    finally:
        ctx.device_free(dp)


@pytest.mark.parametrize("mode", [0, 2])
def test_run_list_scan(knob_ctx, mode):
    """The list-mode scan (MCDC_RUN_LIST=2: whenever the files ascend; 0: the
    flat scan) of device batches: only the runs some chunk window reaches (a
    file's first min_size bytes are never hashed by cut_gear) are scanned,
    through a run list built on a call whose layout repeats the previous one
    and used by the calls after it.  Every layout three times (flat, flat +
    list built, list scan) against the oracle, file by file: sizes around
    min_size and its window warm-up, files crossing run edges, gaps, a partial
    last run, every file at most min_size (a list of no runs), tiny parameters
    whose files share runs (ranges merged), a dense-byte file (overflowed
    runs), descending offsets (no list), mapache's 512K/1M/8M (group walk);
    then a layout change of the same span after a list was built (the
    speculative list scan replaced by the flat scan)."""
    ctx = knob_ctx(MCDC_RUN_LIST=mode)
    rng = np.random.default_rng(77 + mode)

    def check(p, arena, offs, lens, files, calls=3):
        r, rc = O.chunk_files(O.Params(*p), files, threads=4)
        for g, gc in _batch_device_calls(ctx, p, arena, offs, lens, calls):
            assert (gc == rc).all()
            _same(g, r)

    for p in [PARAMS[0], PARAMS[2], PARAMS[1], PARAMS[3], PARAMS[4]]:
        mn = p[0]
        edge = [mn - 1, mn, mn + 1, mn + 47, mn + 48, mn + 64, mn + 4096, 2 * mn + 5, 3 * p[2] + 11]
        layouts = [
            (edge * 3, [0] * len(edge) * 3),
            (list(rng.integers(1, 4 * mn + 2, 300)), list(rng.integers(0, 9000, 300) * (rng.random(300) < 0.3))),
            ([min(mn, 50000)] * 40, [0] * 40),  # every file <= min_size: nothing listed
            ([int(x) for x in np.minimum(np.exp(rng.normal(np.log(max(mn // 2, 64)), 1.2, 500)).astype(np.int64) + 1,
                                         40 * mn)], [0] * 500),
        ]
        for sizes, gaps in layouts:
            arena, offs, lens, files = _arena_files(rng, sizes, gaps)
            check(p, arena, offs, lens, files)
    # a dense-byte file among random ones (runs whose entry lists overflow)
    p = PARAMS[2]
    b = _find_dense_byte(p)
    if b is not None:
        files = [O.random_bytes(3000, 5), np.full(700_000, b, np.uint8), O.random_bytes(1 << 20, 6)]
        check(p, np.concatenate(files), np.array([0, 3000, 703000], np.uint64),
              np.array([f.size for f in files], np.uint64), files)
    # descending offsets (no list), then the same files ascending
    p = PARAMS[0]
    sizes = [int(x) for x in rng.integers(1, 200_000, 64)]
    arena, offs, lens, files = _arena_files(rng, sizes, [0] * 64)
    for order in (np.arange(64)[::-1], np.arange(64)):
        check(p, arena, offs[order], lens[order], [files[i] for i in order])
    # a list built for layout A, then layout B of the same span (one boundary
    # moved): B's first call scans A's runs speculatively and re-scans flat
    sizes = [int(x) for x in rng.integers(20_000, 120_000, 400)]
    arena, offs, lens, files = _arena_files(rng, sizes, [0] * 400)
    lens_b = lens.copy()
    lens_b[10] -= np.uint64(30_000)
    lens_b[11] += np.uint64(30_000)
    offs_b = offs.copy()
    offs_b[11] -= np.uint64(30_000)
    files_b = [arena[int(o):int(o) + int(n)] for o, n in zip(offs_b, lens_b)]
    ra, rca = O.chunk_files(O.Params(*p), files, threads=4)
    rb, rcb = O.chunk_files(O.Params(*p), files_b, threads=4)
    dp = ctx.device_alloc(arena.size + 16)
    try:
        ctx.h2d(dp, arena)
        for o, n, r, rc in [(offs, lens, ra, rca)] * 3 + [(offs_b, lens_b, rb, rcb)] * 3 + [(offs, lens, ra, rca)]:
            g, gc = ctx.chunk_batch_device(_lib.params(*p), dp, o, n)
            assert (gc == rc).all()
            _same(g, r)
    finally:
        ctx.device_free(dp)


@pytest.mark.parametrize("p", [PARAMS[0], PARAMS[1], PARAMS[2], PARAMS[3]], ids=lambda p: "/".join(map(str, p)))
def test_gpu_plan_many_files(ctx, p):
    """A single-part batch of >= 2048 files is planned on the GPU (k_plan_count
    / k_plan_write: files, segments, node offsets from the uploaded extents):
    empty files, files of exactly k segments and one byte either side,
    multi-segment files, gaps; a new layout every call (offsets shifted by 16
    bytes) and the same layout again (the kept plan), against the oracle."""
    z = _segment_bytes(p)
    rng = np.random.default_rng(4242)
    special = [0, 1, p[0], p[0] + 1, z - 1, z, z + 1, 2 * z, 2 * z + 1, 3 * z - 1]
    sizes = [int(x) for x in rng.integers(0, 3 * p[0] + 5, 2600)]
    for k, s in enumerate(special * 12):
        sizes[(k * 211) % len(sizes)] = s
    gaps = [int(g) * (k % 7 == 0) for k, g in enumerate(rng.integers(1, 5000, len(sizes)))]
    arena, offs, lens, files = _arena_files(rng, sizes, gaps)
    arena = np.concatenate([arena, np.zeros(64, np.uint8)])
    shifted = [np.concatenate([arena[int(o) + 16:int(o) + 16 + int(n)]]) for o, n in zip(offs, lens)]
    r0, rc0 = O.chunk_files(O.Params(*p), files, threads=4)
    r1, rc1 = O.chunk_files(O.Params(*p), shifted, threads=4)
    dp = ctx.device_alloc(arena.size + 16)
    try:
        ctx.h2d(dp, arena)
        for c in range(6):  # new, new, new, new, same, same
            sh = 16 * (c % 2) if c < 4 else 0
            g, gc = ctx.chunk_batch_device(_lib.params(*p), dp, offs + np.uint64(sh), lens)
            r, rc = (r1, rc1) if sh else (r0, rc0)
            assert (gc == rc).all()
            _same(g, r)
    finally:
        ctx.device_free(dp)


def test_gpu_plan_falls_back_for_huge_files(ctx):
    """A batch of >= 2048 files holding a file of more than 1024 segments is
    planned on the host (k_plan_write writes a file's segments on one lane):
    same boundaries as the oracle, then the same batch without that file
    (planned on the GPU)."""
    p = PARAMS[2]
    z = _segment_bytes(p)
    rng = np.random.default_rng(99)
    sizes = [int(x) for x in rng.integers(0, 3000, 2100)]
    sizes[777] = 1100 * z + 5
    arena, offs, lens, files = _arena_files(rng, sizes, [0] * len(sizes))
    r, rc = O.chunk_files(O.Params(*p), files, threads=4)
    keep = [i for i in range(len(sizes)) if i != 777]
    r2, rc2 = O.chunk_files(O.Params(*p), [files[i] for i in keep], threads=4)
    dp = ctx.device_alloc(arena.size + 16)
    try:
        ctx.h2d(dp, arena)
        for _ in range(2):
            g, gc = ctx.chunk_batch_device(_lib.params(*p), dp, offs, lens)
            assert (gc == rc).all()
            _same(g, r)
            g, gc = ctx.chunk_batch_device(_lib.params(*p), dp, offs[keep], lens[keep])
            assert (gc == rc2).all()
            _same(g, r2)
    finally:
        ctx.device_free(dp)
