"""GPU-assisted packer (mcdc_pack_blobs: Packer::add_blob + flush, packer.rs:
101-186) against the restatement (oracle.pack_plan / pack_header): pack
boundaries, the blobs back to back, the encoded header (opened by the RFC 8452
oracle, decompressed by libzstd, equal to the restated header bytes incl. the
random padding entries), the le32 length trailer, the parse_header view of it,
and the pack ID = BLAKE3 of the pack (oracle/blake3_oracle.c)."""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu
KEY = bytes(range(0x60, 0x80))


def _inputs(nblobs, seed, maxlen=300_000):
    rng = np.random.default_rng(seed)
    lens = rng.integers(28, maxlen, nblobs)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = O.random_bytes(int(lens.sum()) + 1, seed)
    ids = rng.integers(0, 256, (nblobs, 32), dtype=np.uint8)
    types = rng.integers(0, 2, nblobs).astype(np.uint8)
    return data, offs, lens.astype(np.uint64), ids, types, rng


def _check(ctx, data, offs, lens, ids, types, maxp, rng):
    plan = O.pack_plan(lens, maxp)
    nonces = rng.integers(0, 256, (max(len(plan), 1), 12), dtype=np.uint8)
    padding = rng.integers(0, 256, (63 * max(len(plan), 1), 36), dtype=np.uint8)
    out, packs = ctx.pack_blobs(KEY, data, offs, lens, ids, types, maxp, nonces, padding)
    assert [(int(p["nblobs"])) for p in packs] == [e - f for f, e in plan]
    z, used = O.Zstd(), 0
    at = 0
    for k, (f, e) in enumerate(plan):
        p = packs[k]
        assert int(p["offset"]) == at
        pack = out[at:at + int(p["length"])].tobytes()
        at += len(pack)
        body = b"".join(data[int(offs[i]):int(offs[i] + lens[i])].tobytes() for i in range(f, e))
        assert pack[:len(body)] == body
        hl = int.from_bytes(pack[-4:], "little")
        assert hl + 4 == int(p["meta_size"]) and len(body) + hl + 4 == len(pack)
        enc = pack[len(body):len(body) + hl]
        assert enc[:12] == nonces[k].tobytes()
        cnt = e - f
        pad = (64 - cnt % 64) % 64
        ref_hdr = O.pack_header(ids[f:e], lens[f:e], types[f:e], padding[used:used + pad])
        used += pad
        hdr = z.decompress(O.decrypt_with_key(KEY, enc), len(ref_hdr))
        assert hdr == ref_hdr
        # parse_header (packer.rs:214-285): non-padding entries, offsets by running sum
        entries = [hdr[j:j + 37] for j in range(0, len(hdr), 37)]
        real = [x for x in entries if x[36] != 0xFF]
        assert [x[:32] for x in real] == [ids[i].tobytes() for i in range(f, e)]
        assert [int.from_bytes(x[32:36], "little") for x in real] == [int(lens[i]) for i in range(f, e)]
        assert bytes(p["id"]) == O.blake3(np.frombuffer(pack, np.uint8))
    assert at == out.size
    return packs


def test_many_packs(ctx):
    data, offs, lens, ids, types, rng = _inputs(700, 31)
    packs = _check(ctx, data, offs, lens, ids, types, 4 << 20, rng)
    assert len(packs) > 20


def test_edge_shapes(ctx):
    # one blob over the limit; exactly 64 entries (no padding); a single small blob
    for nb, maxp, mx in ((1, 1000, 300_000), (64, 1 << 40, 5000), (1, 1 << 24, 100), (129, 200_000, 9000)):
        data, offs, lens, ids, types, rng = _inputs(nb, 40 + nb, mx)
        _check(ctx, data, offs, lens, ids, types, maxp, rng)


def test_empty_and_argument_errors(ctx):
    data, offs, lens, ids, types, rng = _inputs(10, 50, 1000)
    out, packs = ctx.pack_blobs(KEY, data, offs[:0], lens[:0], ids[:0], types[:0], 1 << 24,
                                np.zeros((1, 12), np.uint8), np.zeros((1, 36), np.uint8))
    assert out.size == 0 and packs.size == 0
    with pytest.raises(_lib.McdcError) as ei:  # 10 entries need 54 padding entries, the pool holds 3
        ctx.pack_blobs(KEY, data, offs, lens, ids, types, 1 << 24, np.zeros((1, 12), np.uint8),
                       np.zeros((3, 36), np.uint8))
    assert ei.value.code == _lib.MCDC_E_INVALID
    with pytest.raises(_lib.McdcError) as ei:  # 10 packs, one nonce
        ctx.pack_blobs(KEY, data, offs, lens, ids, types, 1, np.zeros((1, 12), np.uint8),
                       np.zeros((700, 36), np.uint8))
    assert ei.value.code == _lib.MCDC_E_INVALID


def _kat():
    blobs = [b"mapache", b"backup", b"rust"]
    data = np.frombuffer(b"".join(blobs), np.uint8)
    lens = np.array([len(b) for b in blobs], np.uint64)
    offs = np.array([0, 7, 13], np.uint64)
    ids = np.stack([np.frombuffer(O.blake3(np.frombuffer(b, np.uint8)), np.uint8) for b in blobs])
    rng = np.random.default_rng(5)
    padding = rng.integers(0, 256, (61, 36), dtype=np.uint8)
    return blobs, data, offs, lens, ids, padding


def test_reference_pack_flush_kat(ctx):
    """packer.rs:345-378 (test_pack_flush) through the C ABI: three blobs,
    SecureStorage::build() (key None), one flush -> a 2398-byte pack whose
    header holds 64 entries of which parse_header keeps 3; byte-identical to
    the restatement (oracle.pack_flush) given the same padding draws; pack ID =
    BLAKE3 of the pack."""
    blobs, data, offs, lens, ids, padding = _kat()
    out, packs = ctx.pack_blobs(None, data, offs, lens, ids, np.zeros(3, np.uint8), 16 << 20, None, padding)
    assert len(packs) == 1 and out.size == 2398 and int(packs[0]["length"]) == 2398
    assert int(packs[0]["nblobs"]) == 3 and int(packs[0]["meta_size"]) == 2398 - 17
    pack = out.tobytes()
    pad = [(p[:32].tobytes(), 0, int.from_bytes(p[32:].tobytes(), "little")) for p in padding]
    ref, desc = O.pack_flush(blobs, [i.tobytes() for i in ids], [0, 0, 0], pad)
    assert pack == ref and len(desc) == 64
    hdr = O.parse_header(pack)
    assert [(h[2], h[3]) for h in hdr] == [(0, 7), (7, 6), (13, 4)] and [h[0] for h in hdr] == [i.tobytes() for i in ids]
    assert bytes(packs[0]["id"]) == O.blake3(out)


def test_reference_empty_pack_flush(ctx):
    """packer.rs:380-395 (test_empty_pack_flush): nothing added, nothing flushed."""
    out, packs = ctx.pack_blobs(None, np.zeros(0, np.uint8), [], [], np.zeros((0, 32), np.uint8),
                                np.zeros(0, np.uint8), 16 << 20, None, np.zeros((0, 36), np.uint8))
    assert len(packs) == 0 and out.size == 0


def test_keyless_packs_match_the_restatement(ctx):
    """Many packs without a key: every pack byte-identical to oracle.pack_flush
    over its blobs (flush rule oracle.pack_plan), headers parsed back."""
    data, offs, lens, ids, types, rng = _inputs(300, 41, maxlen=200_000)
    maxp = 4 << 20
    plan = O.pack_plan(lens, maxp)
    padding = rng.integers(0, 256, (63 * len(plan), 36), dtype=np.uint8)
    out, packs = ctx.pack_blobs(None, data, offs, lens, ids, types, maxp, None, padding)
    assert len(packs) == len(plan)
    used = 0
    for k, (f, e) in enumerate(plan):
        npad = (64 - (e - f) % 64) % 64
        pad = [(p[:32].tobytes(), 0, int.from_bytes(p[32:].tobytes(), "little")) for p in padding[used:used + npad]]
        used += npad
        blobs = [data[int(offs[i]):int(offs[i] + lens[i])].tobytes() for i in range(f, e)]
        ref, _ = O.pack_flush(blobs, [ids[i].tobytes() for i in range(f, e)], types[f:e], pad)
        p = packs[k]
        got = out[int(p["offset"]):int(p["offset"] + p["length"])].tobytes()
        assert got == ref, k
        assert [(h[3], h[1]) for h in O.parse_header(got)] == [(int(lens[i]), int(types[i])) for i in range(f, e)]
