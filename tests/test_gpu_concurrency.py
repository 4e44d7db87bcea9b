"""The deployment's concurrency shape on the GPU: mapache chunks files on
`read_concurrency` rayon workers at once (/root/reference/src/archiver/
mod.rs:162-215, default 4: src/global/defaults.rs:22), each with its own
StreamCDC per file (src/archiver/processor.rs:173).

* 4 host threads, each with its own mcdc context on device 0 (the Rust
  adapter's thread_local context), chunk different files at
  the same time — four LDS-filling scans on one GPU concurrently;
* 8 threads sharing ONE Python Context (calls serialise on its lock);
* 16 threads submitting through the batching front-end (mcdc_batcher_*),
  whose batches serve many callers per call;
every result against the oracle, bit for bit.
"""
import threading

import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu

P16 = (16384, 65536, 262144, 1)
P512 = (524288, 1048576, 8388608, 1)


def _same(g, r):
    return len(g) == len(r) and bool((g["offset"] == r["offset"]).all() and (g["length"] == r["length"]).all()
                                      and (g["hash"] == r["hash"]).all())


def _threads(n, fn):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # reported by the main thread
            errs.append((i, repr(e)))
    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a worker thread hung"
    assert not errs, errs


def test_four_workers_own_contexts():
    rng = np.random.default_rng(41)
    files = [[O.random_bytes(int(s), 7000 + 10 * w + k) for k, s in enumerate(rng.integers(1, 40 << 20, 6))]
             for w in range(4)]
    refs = [[O.chunk(O.Params(*(P16 if k % 2 == 0 else P512)), d) for k, d in enumerate(fs)] for fs in files]
    bad = []

    def worker(w):
        with _lib.Context(0, 64 << 20) as ctx:
            for rep in range(3):
                for k, d in enumerate(files[w]):
                    p = P16 if k % 2 == 0 else P512
                    if not _same(ctx.chunk_host(_lib.params(*p), d), refs[w][k]):
                        bad.append((w, rep, k))
    _threads(4, worker)
    assert not bad, bad


def test_eight_threads_share_one_context(ctx):
    rng = np.random.default_rng(43)
    files = [O.random_bytes(int(s), 8000 + i) for i, s in enumerate(rng.integers(0, 12 << 20, 24))]
    refs = [O.chunk(O.Params(*P16), d) for d in files]
    bad = []

    def worker(w):
        for k in range(w, len(files), 8):
            if not _same(ctx.chunk_host(_lib.params(*P16), files[k]), refs[k]):
                bad.append(k)
    _threads(8, worker)
    assert not bad, bad


@pytest.mark.parametrize("threads", [4, 16])
def test_batcher_many_submitters(threads):
    rng = np.random.default_rng(47 + threads)
    nfiles = 12 * threads
    sizes = rng.integers(0, 6 << 20, nfiles)
    sizes[::9] = 0
    sizes[1::11] = P16[0] - 1  # below min: one whole chunk
    files = [O.random_bytes(int(s), 9000 + i) for i, s in enumerate(sizes)]
    refs = [O.chunk(O.Params(*P16), d) for d in files]
    bad = []
    with _lib.Batcher(_lib.params(*P16), max_batch_bytes=256 << 20, max_batch_files=64, gather_us=500) as b:
        def worker(w):
            for k in range(w, nfiles, threads):
                if not _same(b.chunk(files[k]), refs[k]):
                    bad.append(k)
        _threads(threads, worker)
        st = b.stats()
        with pytest.raises(_lib.McdcError) as ei:  # larger than max_batch_bytes
            b.chunk(np.zeros((256 << 20) + 1, np.uint8))
        assert ei.value.code == _lib.MCDC_E_TOOBIG
    assert not bad, bad
    assert st["files"] == nfiles and st["bytes"] == int(sizes.sum())
    assert st["batches"] < nfiles and st["max_batch_files"] > 1, st


def test_two_contexts_24gib_streams_concurrently():
    """Two worker threads, each with its own context (INTEGRATION.md §2's
    per-worker context), chunk a distinct 24 GiB device-resident stream at the
    same time, three calls each, so the two LDS-filling scans share the CUs
    with each other's resolution waves (k_spec_lane / k_emit) -- the
    co-residence the round-3 exact-fill exemption of k_scan_q assumed never
    happened.  Every call's whole boundary list and every
    ChunkData.hash against the oracle's streamed digest of its stream."""
    n = 24 << 30
    seeds = [0x6d61706163686521 ^ 0x24A, 0x6d61706163686521 ^ 0x24B]
    ref = [None, None]

    def oracle_digest(i):
        ref[i] = O.random_stream_digest(O.Params(*P16), seeds[i], n, hashes=True)
    oth = [threading.Thread(target=oracle_digest, args=(i,)) for i in range(2)]
    for t in oth:  # the oracle digests run on the host while the GPU works
        t.start()
    got = [[], []]
    cap = n // (P16[0] - 1) + 2

    def worker(i):
        with _lib.Context(0, n) as c:
            dp = c.device_alloc(n)
            d_out = c.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
            try:
                c.fill_random(dp, n, seeds[i])
                for _ in range(3):
                    k = c.chunk_device_to_device(_lib.params(*P16), dp, n, d_out, cap)
                    g = c.d2h_chunks(d_out, k)
                    got[i].append((k, _lib.digest(g), int(g["length"].sum()), O.hash_digest(g)))
            finally:
                c.device_free(d_out)
                c.device_free(dp)
    _threads(2, worker)
    for t in oth:
        t.join()
    for i in range(2):
        assert len(got[i]) == 3
        for j, r in enumerate(got[i]):
            assert r == ref[i], (i, j, r, ref[i])
