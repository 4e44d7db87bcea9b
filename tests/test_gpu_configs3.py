"""BASELINE configs[3] ("extracted Linux kernel source tree, ~80 k small files,
dedup-heavy realistic mix") through the composed save path at mapache's own
parameters: processor::save_file's whole-file branch for the files below
MIN_CHUNK_SIZE (/root/reference/src/archiver/processor.rs:144-153), StreamCDC
512K/1M/8M for the rest (:160-205, defaults.rs:35-40), ID::from_content,
Repository::save_blob's dedup (repository_v1.rs:169-180), SecureStorage::encode
with a key and the packer (:182-192).  No kernel tree exists here or on the
GPU box: tests/corpora.kernel_tree is a deterministic stand-in (80 000 files,
log-normal sizes with median 8 KiB, C-like text, ~10 % duplicate files).

* host zstd: every per-file ID list, every is_new flag and every pack byte
  equal oracle.save_files (the composed restatement);
* GPU compression: the same IDs and decisions; every pack parses and every
  blob decodes (SecureStorage::decode) to bytes whose BLAKE3 is its ID, in
  storing order; the ratio beside the host encoder's."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O
from tests import corpora
from tests.test_gpu_save import _check

pytestmark = pytest.mark.gpu
P512 = (524288, 1048576, 8388608, 1)
KEY = bytes(range(0x40, 0x60))


def _rand(seed, n, width):
    return np.random.default_rng(seed).integers(0, 256, (n, width), dtype=np.uint8)


@pytest.fixture(scope="module")
def tree():
    data, offs, lens, dup = corpora.kernel_tree(80000)
    nonces, hn, pad = _rand(1, 100_000, 12), _rand(2, 4096, 12), _rand(3, 4096 * 63, 36)
    files = [data[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]
    ref = O.save_files(O.Params(*P512), files, None, KEY, nonces, hn, pad)
    return data, offs, lens, dup, nonces, hn, pad, ref


def _save(ctx, tree, gpu):
    data, offs, lens, _, nonces, hn, pad, _ = tree
    dp = ctx.device_alloc(data.size)
    try:
        ctx.h2d(dp, data)
        with ctx.index_create() as ix:
            got = ctx.save_files(_lib.params(*P512), ix, dp, offs, lens, KEY, nonces, hn, pad, n=data.size,
                                 gpu_compress=gpu)
            assert len(ix) == int(got[1].sum())
    finally:
        ctx.device_free(dp)
    return got


@pytest.mark.timeout(900)
def test_kernel_tree_host_zstd_every_pack_byte(ctx, tree):
    data, offs, lens, dup, *_, ref = tree
    got = _save(ctx, tree, False)
    _check(got, ref)
    ids, new = got[0], got[1]
    assert sum(len(x) == 1 for x in ids) > 0.99 * len(ids)  # save_file's whole-file branch
    assert sum(len(x) > 1 for x in ids) >= 5  # and chunked files
    for f in np.nonzero(dup >= 0)[0]:
        assert ids[f].shape == ids[dup[f]].shape and (ids[f] == ids[dup[f]]).all(), f
    distinct = {x.tobytes() for f in ids for x in f}
    assert int(new.sum()) == len(distinct) < sum(len(f) for f in ids)  # every duplicate stored once


@pytest.mark.timeout(900)
def test_kernel_tree_gpu_compress_decodes(ctx, tree):
    *_, ref = tree
    ids, new, out, packs = _save(ctx, tree, True)
    r_ids, r_new, r_packs = ref
    assert len(ids) == len(r_ids) and all((a == b).all() for a, b in zip(ids, r_ids))
    assert (new == r_new).all()
    stored = [x.tobytes() for x in np.concatenate(ids)[new]]
    hdrs, at = [], 0
    for pk in packs:
        assert int(pk["offset"]) == at
        body = out[at:at + int(pk["length"])].tobytes()
        assert bytes(pk["id"]) == O.blake3(np.frombuffer(body, np.uint8))
        hdrs += [(body, h) for h in O.parse_header(body, KEY)]
        at += int(pk["length"])
    assert at == out.size and len(hdrs) == len(stored)

    def check(i):
        body, (bid, typ, off, ln) = hdrs[i]
        dec = O.storage_decode(body[off:off + ln], KEY, size_hint=16 << 20)
        return bid == stored[i] and typ == 0 and O.blake3(np.frombuffer(dec, np.uint8)) == bid

    with ThreadPoolExecutor(8) as ex:
        assert all(ex.map(check, range(len(hdrs))))
    host_bytes = sum(len(p) for p, _ in r_packs)
    assert out.size <= host_bytes / 0.95, (out.size, host_bytes)  # ratio >= 0.95 x the host level 3's
