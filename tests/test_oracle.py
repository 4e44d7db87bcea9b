"""The oracle (CPU restatement of fastcdc 3.2.1 v2020) against everything that
can pin it offline: the MD5 derivation of GEAR, MASKS popcounts, the crate's
recalled ``test_all_zeros`` KAT, three independent statements of cut_gear
(C 2-byte loop, C 1-byte loop, pure Python), StreamCDC buffer semantics, and
the analytic mean chunk size.  Parity with the crate itself is unpinned by the
reference (no reference test reaches the chunker)."""
import hashlib
import struct

import numpy as np
import pytest

from oracle import oracle as O

SEED = 0x6d61706163686521


def test_gear_md5_derivation_and_known_values():
    g, gls, _ = O.tables()
    assert g == O.gear_md5()
    assert [hex(x) for x in g[:8]] == ["0x3b5d3c7d207e37dc", "0x784d68ba91123086", "0xcd52880f882e7298",
                                      "0xeacf8e4e19fdcca7", "0xc31f385dfbd1632b", "0x1d5f27001e25abe6",
                                      "0x83130bde3c9ad991", "0xc4b225676e9b7649"]
    assert g[128] == 0xc0ce47f889336346 and g[255] == 0xaabd2b2a451504e1
    assert len(set(g)) == 256
    blob = b"".join(struct.pack("<Q", x) for x in g)
    assert hashlib.sha256(blob).hexdigest() == "91a3061015ae351cd3701852712bcd6aa4a1ce26c8a231d3969432b00f028f88"
    blob_ls = b"".join(struct.pack("<Q", x) for x in gls)
    assert hashlib.sha256(blob_ls).hexdigest() == "7d105f0bf349dc8a92b8c0d7cf22ea7a998d61673ff02b9cc5ad308b522e146f"
    assert gls[0] == 0x76ba78fa40fc6fb8


def test_masks_popcount_and_span():
    _, _, m = O.tables()
    assert m[:5] == [0] * 5
    for k in range(5, 26):
        assert bin(m[k]).count("1") == k
    for k in range(11, 26):
        assert m[k] >> 47 == 1 and m[k] < (1 << 48)  # highest bit 47: 48-byte window locality


def test_crate_kat_all_zeros():
    """fastcdc v2020 test_all_zeros (recalled): 10 x 1024, hash 14169102344523991076."""
    c = O.chunk(O.Params(64, 256, 1024), bytes(10240))
    assert len(c) == 10
    assert set(c["length"].tolist()) == {1024}
    assert set(c["hash"].tolist()) == {14169102344523991076}


@pytest.mark.parametrize("bad", [(63, 256, 1024), (1048577, 2097152, 4194304), (64, 255, 1024),
                                 (64, 4194305, 16777216), (64, 256, 1023), (64, 256, 16777217)])
def test_crate_param_asserts(bad):
    with pytest.raises(ValueError):
        O.Params(*bad).c()


def test_masks_selected_like_crate_test_masks():
    _, _, m = O.tables()
    for (mn, av, mx), (l, s) in [((64, 256, 1024), (7, 9)), ((8192, 16384, 32768), (13, 15)),
                                 ((1048576, 4194304, 16777216), (21, 23))]:
        p = O.Params(mn, av, mx).c()
        assert p.mask_l == m[l] and p.mask_s == m[s]


PARAMS = [O.P16, O.P512, O.Params(64, 256, 1024), O.Params(100, 1000, 5000, 2),
          O.Params(65, 300, 1111, 3), O.Params(1024, 4096, 16384, 0), O.Params(4095, 8191, 65535, 1)]


def _adversarial():
    rng = np.random.default_rng(1)
    yield "random", O.random_bytes(3 << 20, SEED)
    yield "zeros", np.zeros(1 << 20, np.uint8)
    yield "ones", np.full(1 << 20, 0xff, np.uint8)
    yield "period7", np.tile(rng.integers(0, 256, 7, dtype=np.uint8), 150000)
    yield "period4096", np.tile(rng.integers(0, 256, 4096, dtype=np.uint8), 300)
    yield "text", np.frombuffer((b"the quick brown fox jumps over the lazy dog. " * 40000), np.uint8)
    yield "odd", O.random_bytes(1_000_003, 5)


@pytest.mark.parametrize("p", PARAMS, ids=str)
def test_two_byte_equals_one_byte_and_stream(p):
    for name, d in _adversarial():
        a = O.chunk(p, d)
        b = O.chunk(p, d, one_byte=True)
        assert (a == b).all(), name
        s = O.chunk_stream(p, d, 65537)
        assert (a == s).all(), name
        assert int(a["length"].sum()) == len(d)


@pytest.mark.parametrize("p", [O.P16, O.Params(64, 256, 1024), O.Params(65, 300, 1111, 3)], ids=str)
def test_c_matches_pure_python(p):
    for seed in range(4):
        d = bytes(O.random_bytes(int(p.max_size * 2.5) + seed, 1000 + seed))
        off = 0
        while off < len(d):
            h, c = O.cut_gear_py(p, d[off:off + p.max_size + 1])
            h2, c2 = O.cut_gear(p, np.frombuffer(d[off:off + p.max_size + 1], np.uint8))
            assert (h, c) == (h2, c2)
            off += c


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 16383, 16384, 16385, 65535, 65536, 65537, 262143,
                               262144, 262145, 2 * 262144 + 1])
def test_edge_lengths(n):
    d = O.random_bytes(n, 42 + n)
    for p in (O.P16, O.Params(65, 300, 1111, 3)):
        c = O.chunk(p, d)
        assert int(c["length"].sum()) == n
        if n == 0:
            assert len(c) == 0
        for i, ln in enumerate(c["length"].tolist()):
            assert ln <= p.max_size
            if i + 1 < len(c):
                assert ln >= 2 * (p.min_size // 2)


def test_mean_chunk_size_matches_analytic():
    """Uniform random bytes at 16/64/256 KiB L1: E[len] = 79 836 B."""
    d = O.random_bytes(512 << 20, SEED)
    k, _ = O.chunk_digest(O.P16, d)
    mean = d.size / k
    assert abs(mean - 79836) / 79836 < 0.02, mean


def test_prng_matches_definition():
    d = O.random_bytes(64, 7, pos=3)

    def mix(z):
        M = (1 << 64) - 1
        z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M
        z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M
        return z ^ (z >> 31)
    ref = bytes(((mix((7 + (((p >> 3) + 1) * 0x9e3779b97f4a7c15)) & ((1 << 64) - 1)) >> (8 * (p & 7))) & 0xff)
                for p in range(3, 67))
    assert bytes(d) == ref


@pytest.mark.parametrize("p", [(16384, 65536, 262144, 1), (64, 256, 1024, 1), (524288, 1048576, 8388608, 1)])
def test_streamed_random_digest_equals_in_memory(p):
    """oc_random_stream_digest (slabs regenerated, window carried across them)
    gives the in-memory whole-slice result, for slabs smaller and larger than
    max and stream lengths not a multiple of the slab."""
    n = (40 << 20) + 12345
    d = O.random_bytes(n, 77)
    k, dig = O.chunk_digest(O.Params(*p), d)
    hd = O.hash_digest(O.chunk(O.Params(*p), d))
    for slab in (4096, 1 << 20, 5_000_000, 64 << 20):
        assert O.random_stream_digest(O.Params(*p), 77, n, slab) == (k, dig, n)
        assert O.random_stream_digest(O.Params(*p), 77, n, slab, hashes=True) == (k, dig, n, hd)


def test_random_files_digest_equals_in_memory():
    """oracle.random_files_digest (files regenerated per thread, the full-size
    many-file parity of tests/test_gpu_configs.py) equals chunking each file in
    memory: counts, boundary digests (the library's mcdc_digest over
    file-relative records) and hash digests; positional and per-file seeds,
    empty and sub-min files, several threads."""
    from mapache_amd import _lib, shard
    p = O.Params(16384, 65536, 262144, 1)
    seeds = [0x5EED ^ (i + 1) for i in range(12)]
    lens = [0, 1, 16383, 16384, 16385, 3 << 20, (1 << 20) + 7, 262145, 5, 2 << 20, 777_777, 1 << 16]
    pos = [i * 1000 + (i % 3) for i in range(12)]
    c, d, h = O.random_files_digest(p, seeds, pos, lens, threads=3)
    for i in range(12):
        ch = O.chunk(p, O.random_bytes(lens[i], seeds[i], pos=pos[i]))
        assert (int(c[i]), int(d[i]), int(h[i])) == (len(ch), _lib.digest(ch), O.hash_digest(ch)), i
    assert shard.corpus_digest(c, d) == shard.corpus_digest([int(x) for x in c], [int(x) for x in d])
    assert shard.corpus_digest(c, d) != shard.corpus_digest(c[::-1], d[::-1])
