"""GPU SecureStorage sealing (mcdc_seal_device / mcdc_open_device) against the
AES-256-GCM-SIV oracle (oracle/aead_oracle.c, pinned by tests/test_aead_oracle.py).

The reference seals each blob with encrypt_with_key (/root/reference/src/
repository/storage.rs:97-118: nonce || ciphertext || tag, no AAD) and opens
with decrypt_with_key (:128-144); its own test only round trips
(:235-247), so byte parity is against the RFC 8452 restatement ("unpinned by
reference", pinned by the RFC's vectors) and the round trip is checked too.
Bit-exact throughout.
"""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu

h = bytes.fromhex
K256, N3 = h("01") + bytes(31), h("030000000000000000000000")


def _dev(ctx, data, pad=64, shift=0):
    """Device copy of `data` at byte offset `shift` of a fresh allocation."""
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    p = ctx.device_alloc(a.size + pad + shift)
    if a.size:
        ctx.h2d(p + shift, a)
    return p


def _seal_gpu(ctx, key, data, offs, lens, nonces, out_shift=0):
    din = _dev(ctx, data)
    cap = int(np.sum(np.asarray(lens, dtype=np.uint64))) + 28 * len(lens)
    dout = ctx.device_alloc(cap + 64 + out_shift)
    try:
        oo = ctx.seal(key, din, len(data), offs, lens, nonces, dout + out_shift, cap)
        got = ctx.d2h_bytes(dout + out_shift, int(oo[-1]))
    finally:
        ctx.device_free(dout)
        ctx.device_free(din)
    return got, oo


def test_rfc8452_vectors_on_gpu(ctx):
    """RFC 8452 appendix C AES-256 vectors without AAD, as one batch; and the
    two counter-wrap vectors (C.3)."""
    pts = [b"", h("0100000000000000"), h("010000000000000000000000"), h("01000000000000000000000000000000")]
    cts = ["07f5f4169bbf55a8400cd47ea6fd400f", "c2ef328e5c71c83b843122130f7364b761e0b97427e3df28",
           "9aab2aeb3faa0a34aea8e2b18ca50da9ae6559e48fd10f6e5c9ca17e",
           "85a01b63025ba19b7fd3ddfc033b3e76c9eac6fa700942702e90862383c6c366"]
    data = b"".join(pts)
    offs = np.cumsum([0] + [len(p) for p in pts[:-1]])
    got, oo = _seal_gpu(ctx, K256, data, offs, [len(p) for p in pts], np.frombuffer(N3 * 4, np.uint8))
    for i, c in enumerate(cts):
        assert got[oo[i]:oo[i + 1]].tobytes() == N3 + h(c), i
    pts = [h("000000000000000000000000000000004db923dc793ee6497c76dcc03a98e108"),
           h("eb3640277c7ffd1303c7a542d02d3e4c0000000000000000")]
    cts = ["f3f80f2cf0cb2dd9c5984fcda908456cc537703b5ba70324a6793a7bf218d3eaffffffff000000000000000000000000",
           "18ce4f0b8cb4d0cac65fea8f79257b20888e53e72299e56dffffffff000000000000000000000000"]
    got, oo = _seal_gpu(ctx, bytes(32), b"".join(pts), [0, 32], [32, 24], np.zeros(24, np.uint8))
    for i, c in enumerate(cts):
        assert got[oo[i] + 12:oo[i + 1]].tobytes() == h(c), i


SIZES = [0, 1, 11, 12, 15, 16, 17, 27, 28, 31, 32, 33, 63, 64, 65, 1023, 1024, 1025, 1040, 4095, 4096, 4097,
         16383, 16384, 16385, 65535, 65536, 65537, 65536 + 1024, 3 * 65536 + 5, (1 << 20) + 7]


@pytest.mark.parametrize("out_shift", [0, 3, 4, 9])
def test_blobs_vs_oracle(ctx, out_shift):
    rng = np.random.default_rng(100 + out_shift)
    lens = np.array(SIZES + list(rng.integers(0, 300_000, 40)), dtype=np.uint64)
    rng.shuffle(lens)
    gaps = rng.integers(0, 40, len(lens))  # blobs at arbitrary byte offsets
    offs = np.cumsum(np.concatenate([[5], (lens + gaps)[:-1]])).astype(np.uint64)
    data = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 13, dtype=np.uint8)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonces = rng.integers(0, 256, (len(lens), 12), dtype=np.uint8)
    got, oo = _seal_gpu(ctx, key, data, offs, lens, nonces, out_shift=out_shift)
    ref, roo = O.seal_blobs(key, data, offs, lens, nonces, threads=8)
    assert (oo[:-1] == roo).all() and int(oo[-1]) == ref.size
    bad = [i for i in range(len(lens)) if got[oo[i]:oo[i + 1]].tobytes() != ref[roo[i]:roo[i] + lens[i] + 28].tobytes()]
    assert not bad, [(i, int(lens[i])) for i in bad[:5]]


def test_overlapping_and_repeated_extents(ctx):
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 300_001, dtype=np.uint8)
    offs = np.array([0, 0, 100, 5, 299_990, 150_000, 7], dtype=np.uint64)
    lens = np.array([300_001, 300_001, 1000, 70_000, 11, 0, 65_536], dtype=np.uint64)
    nonces = rng.integers(0, 256, (len(lens), 12), dtype=np.uint8)
    nonces[1] = nonces[0]
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    got, oo = _seal_gpu(ctx, key, data, offs, lens, nonces)
    ref, roo = O.seal_blobs(key, data, offs, lens, nonces)
    assert got.tobytes() == ref.tobytes()
    assert got[oo[0]:oo[1]].tobytes() == got[oo[1]:oo[2]].tobytes()  # same nonce, same blob


def test_large_blob_tile_combination(ctx):
    """A 20 MiB + 3 blob: 321 POLYVAL tiles joined with H^4096."""
    n = (20 << 20) + 3
    data = O.random_bytes(n, 77)
    nonce = np.arange(12, dtype=np.uint8)
    key = bytes(range(32))
    got, oo = _seal_gpu(ctx, key, data, [0], [n], nonce)
    assert got.tobytes() == O.encrypt_with_key(key, nonce, data)


def _roundtrip(ctx, key, data, offs, lens, nonces, tamper=()):
    din = _dev(ctx, data)
    cap = int(np.sum(lens)) + 28 * len(lens)
    dseal = ctx.device_alloc(cap + 64)
    dopen = ctx.device_alloc(cap + 64)
    try:
        oo = ctx.seal(key, din, len(data), offs, lens, nonces, dseal, cap)
        for i, byte in tamper:  # flip one bit of a sealed blob in HBM
            pos = int(oo[i]) + byte
            b = ctx.d2h_bytes(dseal + pos, 1)
            ctx.h2d(dseal + pos, np.array([b[0] ^ 0x10], np.uint8))
        po, st = ctx.open(key, dseal, int(oo[-1]), oo[:-1], np.diff(oo), dopen, cap, raise_on_auth=False)
        plain = ctx.d2h_bytes(dopen, int(po[-1]))
    finally:
        for p in (dopen, dseal, din):
            ctx.device_free(p)
    return po, st, plain


def test_open_round_trip(ctx):
    rng = np.random.default_rng(5)
    lens = np.array(SIZES + list(rng.integers(0, 200_000, 30)), dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonces = rng.integers(0, 256, (len(lens), 12), dtype=np.uint8)
    po, st, plain = _roundtrip(ctx, key, data, offs, lens, nonces)
    assert (st == 0).all()
    assert (np.diff(po) == lens).all()
    assert plain.tobytes() == data[: int(lens.sum())].tobytes()


def test_open_rejects_tampered_blobs(ctx):
    rng = np.random.default_rng(6)
    lens = np.array([0, 5, 16, 1000, 70_000, 4096, 33, 250_000], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonces = rng.integers(0, 256, (len(lens), 12), dtype=np.uint8)
    tamper = [(0, 3), (2, 12 + 7), (4, 12 + 65_000), (5, 12 + 4096 + 15), (7, 5)]  # nonce, data, tag bytes
    po, st, plain = _roundtrip(ctx, key, data, offs, lens, nonces, tamper)
    bad = {i for i, _ in tamper}
    assert [int(x) for x in st] == [-1 if i in bad else 0 for i in range(len(lens))]
    for i in range(len(lens)):
        seg = plain[po[i]:po[i + 1]]
        want = np.zeros(int(lens[i]), np.uint8) if i in bad else data[offs[i]:offs[i] + lens[i]]
        assert seg.tobytes() == want.tobytes(), i
    with pytest.raises(_lib.McdcError) as ei:
        din = _dev(ctx, bytes(40))
        try:
            ctx.open(bytes(32), din, 40, [0], [27], din, 0)
        finally:
            ctx.device_free(din)
    assert ei.value.code == _lib.MCDC_E_AUTH


def test_open_matches_oracle_decrypt(ctx):
    """Sealed by the oracle, opened on the GPU; short extents fail like the crate."""
    rng = np.random.default_rng(8)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pts = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in (0, 1, 100, 65_536, 123_457)]
    blobs = [O.encrypt_with_key(key, rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), p) for p in pts]
    blobs.append(bytes(27))  # shorter than nonce + tag
    data = b"".join(blobs)
    offs = np.cumsum([0] + [len(b) for b in blobs[:-1]])
    din = _dev(ctx, data)
    dout = ctx.device_alloc(len(data) + 64)
    try:
        po, st = ctx.open(key, din, len(data), offs, [len(b) for b in blobs], dout, len(data), raise_on_auth=False)
        plain = ctx.d2h_bytes(dout, int(po[-1]))
    finally:
        ctx.device_free(dout)
        ctx.device_free(din)
    assert [int(x) for x in st] == [0] * len(pts) + [-1]
    assert plain.tobytes() == b"".join(pts)


def test_errors(ctx):
    din = _dev(ctx, bytes(100))
    dout = ctx.device_alloc(256)
    try:
        with pytest.raises(_lib.McdcError) as ei:  # extent outside the input
            ctx.seal(bytes(32), din, 100, [90], [11], np.zeros(12, np.uint8), dout, 256)
        assert ei.value.code == _lib.MCDC_E_INVALID
        with pytest.raises(_lib.McdcError) as ei:  # output too small
            ctx.seal(bytes(32), din, 100, [0, 0], [100, 100], np.zeros(24, np.uint8), dout, 255)
        assert ei.value.code == _lib.MCDC_E_CAPACITY
        assert (ctx.seal(bytes(32), din, 100, [], [], np.zeros(0, np.uint8), dout, 0) == [0]).all()
        with pytest.raises(ValueError):
            ctx.seal(bytes(31), din, 100, [0], [1], np.zeros(12, np.uint8), dout, 256)
    finally:
        ctx.device_free(dout)
        ctx.device_free(din)


def test_seal_chunks_of_a_stream(ctx):
    """The chunker's device-resident boundary list sealed in place of the
    compressed blobs (random data: zstd would store it raw): 256 MiB, every
    sealed blob against the oracle."""
    n = 256 << 20
    p = _lib.params(16384, 65536, 262144, 1)
    dp = ctx.device_alloc(n + 64)
    try:
        ctx.fill_random(dp, n, 31337)
        ch = ctx.chunk_device(p, dp, n)
        key = bytes(range(100, 132))
        nonces = np.frombuffer(np.arange(len(ch) * 3, dtype=np.uint32).tobytes(), np.uint8)
        cap = n + 28 * len(ch)
        dout = ctx.device_alloc(cap + 64)
        try:
            oo = ctx.seal(key, dp, n, ch["offset"], ch["length"], nonces, dout, cap)
            got = ctx.d2h_bytes(dout, int(oo[-1]))
        finally:
            ctx.device_free(dout)
    finally:
        ctx.device_free(dp)
    ref, roo = O.seal_blobs(key, O.random_bytes(n, 31337), ch["offset"], ch["length"], nonces, threads=8)
    assert got.tobytes() == ref.tobytes()


def test_seal_chunks_device_list(ctx):
    """mcdc_seal_chunks_device with the chunker's device-resident boundary list
    (and with a host list, and with device nonces / device offsets) gives
    exactly mcdc_seal_device's output."""
    n = 64 << 20
    p = _lib.params(16384, 65536, 262144, 1)
    dp = ctx.device_alloc(n + 64)
    cap_c = n // (16384 - 1) + 2
    d_ch = ctx.device_alloc(cap_c * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(dp, n, 4242)
        k = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
        ch = ctx.d2h_chunks(d_ch, k)
        key = bytes(range(7, 39))
        nonces = np.random.default_rng(1).integers(0, 256, (k, 12), dtype=np.uint8)
        d_nonce = _dev(ctx, nonces.reshape(-1))
        d_offs = ctx.device_alloc(8 * (k + 1))
        cap = n + 28 * k
        outs = [ctx.device_alloc(cap) for _ in range(3)]
        try:
            oo = ctx.seal(key, dp, n, ch["offset"], ch["length"], nonces, outs[0], cap)
            oo2 = ctx.seal_chunks(key, dp, n, ch, nonces, outs[1], cap)
            assert ctx.seal_chunks(key, dp, n, (d_ch, k), d_nonce, outs[2], cap, offsets_out=d_offs) is None
            got = [ctx.d2h_bytes(o, int(oo[-1])) for o in outs]
            oo3 = np.frombuffer(ctx.d2h_bytes(d_offs, 8 * (k + 1)).tobytes(), np.uint64)
        finally:
            for o in outs + [d_offs, d_nonce]:
                ctx.device_free(o)
    finally:
        ctx.device_free(d_ch)
        ctx.device_free(dp)
    assert (oo == oo2).all() and (oo == oo3).all()
    assert got[0].tobytes() == got[1].tobytes() == got[2].tobytes()
    host = O.random_bytes(n, 4242)
    for i in (0, 1, k // 2, k - 1):
        assert got[0][oo[i]:oo[i + 1]].tobytes() == O.encrypt_with_key(
            key, nonces[i], host[ch["offset"][i]:ch["offset"][i] + ch["length"][i]])
