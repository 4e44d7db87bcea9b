"""GPU SecureStorage::encode / decode of host blobs (mcdc_encode_blobs /
mcdc_decode_blobs: zstd on host threads, AES-256-GCM-SIV on the GPU) against
the RFC 8452 restatement (oracle/aead_oracle.c) and the system libzstd driven
directly from the test (storage.rs:61-94: level 3, window log 20, no
checksum).  The compressed bytes depend on the libzstd version (the crate's is
1.5.7, this image's 1.4.8), so parity is on what decodes: every sealed blob
opened by the oracle and decompressed within a 2^20 window equals its input,
frames carry no checksum, and frames the library did not write (no content
size, as the crate's streaming encoder leaves them) decode too."""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu
KEY = bytes(range(0x20, 0x40))


Zstd = O.Zstd  # the system libzstd through ctypes (oracle/oracle.py)


def _blobs():
    rng = np.random.default_rng(77)
    words = [b"mapache", b"backup", b"snapshot", b"chunk", b"blob", b"pack", b"index", b"tree"]
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 400_000))
    parts = [text[:300_000], O.random_bytes(200_000, 5).tobytes(), bytes(150_000), b"", b"x",
             text[:3 << 20], O.random_bytes(70_001, 6).tobytes(), bytes(range(256)) * 4000]
    data, offs, lens, at = bytearray(), [], [], 0
    for i, p in enumerate(parts):
        data += bytes(i % 5)  # gaps: every blob at another alignment
        at += i % 5
        offs.append(at)
        lens.append(len(p))
        data += p
        at += len(p)
    return np.frombuffer(bytes(data), np.uint8), np.array(offs, np.uint64), np.array(lens, np.uint64), parts


def _nonces(n):
    nz = np.zeros((n, 12), np.uint8)
    nz[:, 0] = np.arange(n)
    nz[:, 4:] = np.frombuffer(b"encode!!", np.uint8)
    return nz


@pytest.fixture(scope="module")
def zstd():
    return Zstd()


def test_encode_opens_with_the_oracle_and_decompresses(ctx, zstd):
    data, offs, lens, parts = _blobs()
    nz = _nonces(len(parts))
    enc, oo = ctx.encode_blobs(KEY, data, offs, lens, nz)
    assert int(oo[-1]) == enc.size
    for i, p in enumerate(parts):
        blob = enc[int(oo[i]):int(oo[i + 1])].tobytes()
        assert blob[:12] == nz[i].tobytes()
        frame = O.decrypt_with_key(KEY, blob)
        assert frame is not None, f"blob {i}: tag rejected by the oracle"
        assert frame[4] & 0x04 == 0, f"blob {i}: frame carries a checksum"  # Frame_Header_Descriptor bit 2
        assert zstd.decompress(frame, len(p)) == p, f"blob {i}: decoded bytes differ"
    assert len(enc) < data.size  # the text and zero blobs compressed


def test_decode_round_trip_and_foreign_frames(ctx, zstd):
    data, offs, lens, parts = _blobs()
    nz = _nonces(len(parts))
    enc, oo = ctx.encode_blobs(KEY, data, offs, lens, nz)
    dec, do, st = ctx.decode_blobs(KEY, enc, oo[:-1], np.diff(oo), int(lens.sum()) + 16)
    assert (st == 0).all()
    assert [dec[int(do[i]):int(do[i + 1])].tobytes() for i in range(len(parts))] == parts
    # blobs sealed by the restatement around frames without a content size (the
    # crate's streaming encoder) decode the same way
    foreign = [O.encrypt_with_key(KEY, nz[i], zstd.compress(p, content_size=False)) for i, p in enumerate(parts)]
    arr = np.frombuffer(b"".join(foreign), np.uint8)
    fo = np.cumsum([0] + [len(b) for b in foreign]).astype(np.uint64)
    dec2, do2, st2 = ctx.decode_blobs(KEY, arr, fo[:-1], np.diff(fo), int(lens.sum()) + 16)
    assert (st2 == 0).all()
    assert [dec2[int(do2[i]):int(do2[i + 1])].tobytes() for i in range(len(parts))] == parts


def test_decode_failures_per_blob(ctx):
    data, offs, lens, parts = _blobs()
    nz = _nonces(len(parts))
    enc, oo = ctx.encode_blobs(KEY, data, offs, lens, nz)
    bad = enc.copy()
    bad[int(oo[1]) + 20] ^= 1  # ciphertext of blob 1: authentication fails
    # blob 2: authentic, but its plaintext is not a zstd frame
    junk = O.encrypt_with_key(KEY, nz[2], b"not a zstd frame at all")
    pieces = [bad[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(len(parts))]
    pieces[2] = junk
    arr = np.frombuffer(b"".join(pieces), np.uint8)
    fo = np.cumsum([0] + [len(b) for b in pieces]).astype(np.uint64)
    dec, do, st = ctx.decode_blobs(KEY, arr, fo[:-1], np.diff(fo), int(lens.sum()) + 16)
    assert st[1] == -1 and st[2] == -2
    assert all(st[i] == 0 for i in range(len(parts)) if i not in (1, 2))
    for i in range(len(parts)):
        if i not in (1, 2):
            assert dec[int(do[i]):int(do[i + 1])].tobytes() == parts[i]
        else:
            assert do[i + 1] == do[i]  # failed blobs yield no bytes


def test_encode_capacity_and_range_errors(ctx):
    from mapache_amd._lib import load
    data, offs, lens, parts = _blobs()
    nz = _nonces(len(parts))
    ext = np.stack([offs, lens], axis=1).astype(np.uint64)
    oo = np.zeros(len(parts) + 1, np.uint64)
    out = np.empty(16, np.uint8)
    rc = load().mcdc_encode_blobs(ctx._h, KEY, data.ctypes.data, data.size, ext.ctypes.data, len(parts),
                                  nz.ctypes.data, out.ctypes.data, out.size, oo.ctypes.data)
    assert rc == _lib.MCDC_E_CAPACITY and oo[-1] > 16
    ext[3, 0] = data.size  # offset past the end with a non-zero length elsewhere
    ext[3, 1] = 1
    rc = load().mcdc_encode_blobs(ctx._h, KEY, data.ctypes.data, data.size, ext.ctypes.data, len(parts),
                                  nz.ctypes.data, out.ctypes.data, out.size, oo.ctypes.data)
    assert rc == _lib.MCDC_E_INVALID


def test_keyless_storage_is_the_crates_bytes(ctx):
    """SecureStorage::build() (key None: storage.rs:40-46, encrypt / decrypt the
    identity): every encoded blob is byte-for-byte the frame the crate's
    streaming encoder writes with this libzstd (oracle.storage_encode: no
    content size, 2^20 window descriptor), and decode(None) returns the blobs.
    With a key, the opened frames are the same bytes."""
    data, offs, lens, parts = _blobs()
    enc, oo = ctx.encode_blobs(None, data, offs, lens, None)
    got = [enc[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(len(parts))]
    assert got == [O.storage_encode(p) for p in parts]
    for g in got:
        assert g[4] == 0x00 and g[5] == 0x50  # no content size / checksum; window 2^20
    dec, do, st = ctx.decode_blobs(None, enc, oo[:-1], np.diff(oo), int(lens.sum()) + 16)
    assert (st == 0).all()
    assert [dec[int(do[i]):int(do[i + 1])].tobytes() for i in range(len(parts))] == parts
    nz = _nonces(len(parts))
    enc_k, ok = ctx.encode_blobs(KEY, data, offs, lens, nz)
    assert [O.decrypt_with_key(KEY, enc_k[int(ok[i]):int(ok[i + 1])].tobytes()) for i in range(len(parts))] == got
