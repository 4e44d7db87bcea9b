"""GPU zstd raw-block frames (mcdc_zstd_frames_device) against the RFC 8878
restatement (oracle.zstd_raw_frame, bit-exact) and the system libzstd (every
frame decodes to its chunk within the 2^20 window mapache's decoder allows,
storage.rs:87-94), and chunk -> frame -> seal -> mcdc_decode_blobs in HBM."""
import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _frames(ctx, data, chunks):
    dp = ctx.device_alloc(data.size + 16)
    try:
        ctx.h2d(dp, data)
        cap = int(sum(int(x) + 6 + 3 * (int(x) // 131072 + 1) + 16 for x in chunks["length"])) + 16
        d_out = ctx.device_alloc(cap)
        try:
            fr, span = ctx.zstd_frames(dp, data.size, chunks, d_out, cap)
            out = ctx.d2h_bytes(d_out, span)
        finally:
            ctx.device_free(d_out)
    finally:
        ctx.device_free(dp)
    return fr, out


@pytest.mark.parametrize("p", [(16384, 65536, 262144, 1), (524288, 1048576, 8388608, 1)], ids=["P16", "P512"])
def test_frames_of_a_stream(ctx, p):
    data = O.random_bytes((48 << 20) + 11, 0xF7)
    ch = O.chunk(O.Params(*p), data)
    fr, out = _frames(ctx, data, ch)
    z = O.Zstd()
    for i in range(len(ch)):
        o, n = int(fr[i, 0]), int(fr[i, 1])
        assert o % 16 == 0
        chunk = data[int(ch["offset"][i]):int(ch["offset"][i] + ch["length"][i])].tobytes()
        frame = out[o:o + n].tobytes()
        assert frame == O.zstd_raw_frame(chunk)
        if i < 40 or i == len(ch) - 1:  # (libzstd on a sample; includes 8 MiB chunks at P512)
            assert z.decompress(frame, len(chunk)) == chunk


def test_edge_lengths_and_alignments(ctx):
    lens = [0, 1, 15, 16, 17, 131069, 131072, 131073, 262144, 262147, 400_001]
    pairs, pos = [], 0
    for i, n in enumerate(lens):
        pos += i % 7
        pairs.append((pos, n))
        pos += n
    data = O.random_bytes(pos + 3, 0xF8)
    ch = np.zeros(len(pairs), dtype=_lib.CHUNK_DTYPE)
    ch["offset"], ch["length"] = [x[0] for x in pairs], [x[1] for x in pairs]
    fr, out = _frames(ctx, data, ch)
    z = O.Zstd()
    for i, (o_, n_) in enumerate(pairs):
        frame = out[int(fr[i, 0]):int(fr[i, 0] + fr[i, 1])].tobytes()
        chunk = data[o_:o_ + n_].tobytes()
        assert frame == O.zstd_raw_frame(chunk), lens[i]
        assert z.decompress(frame, len(chunk)) == chunk


def test_frame_seal_decode_in_hbm(ctx):
    """chunk -> frame -> seal on the GPU; mcdc_decode_blobs (GPU open + zstd)
    returns the chunks: blobs the reference's decoder reads."""
    n = (20 << 20) + 5
    data = O.random_bytes(n, 0xF9)
    p = _lib.params(16384, 65536, 262144, 1)
    dp = ctx.device_alloc(n + 16)
    cap_c = n // 16383 + 2
    d_ch = ctx.device_alloc(cap_c * 24)
    try:
        ctx.h2d(dp, data)
        k = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
        cap_f = n + 32 * k + 64
        d_f = ctx.device_alloc(cap_f)
        try:
            fr, span = ctx.zstd_frames(dp, n, (d_ch, k), d_f, cap_f)
            nonces = np.arange(12 * k, dtype=np.uint32).astype(np.uint8).reshape(k, 12)
            cap_s = int(fr[:, 1].sum()) + 28 * k
            d_s = ctx.device_alloc(cap_s)
            try:
                oo = ctx.seal(bytes(range(32)), d_f, span, fr[:, 0], fr[:, 1], nonces, d_s, cap_s)
                sealed = ctx.d2h_bytes(d_s, int(oo[-1]))
            finally:
                ctx.device_free(d_s)
        finally:
            ctx.device_free(d_f)
        chunks = ctx.d2h_chunks(d_ch, k)
    finally:
        ctx.device_free(d_ch)
        ctx.device_free(dp)
    dec, do, st = ctx.decode_blobs(bytes(range(32)), sealed, oo[:-1], np.diff(oo), n + 64)
    assert (st == 0).all() and dec.size == n and (dec == data).all()
    assert (np.diff(do) == chunks["length"]).all()


def test_capacity_error(ctx):
    data = O.random_bytes(1 << 20, 1)
    ch = np.zeros(1, dtype=_lib.CHUNK_DTYPE)
    ch["length"] = 1 << 20
    dp = ctx.device_alloc(data.size)
    d_out = ctx.device_alloc(1024)
    try:
        ctx.h2d(dp, data)
        with pytest.raises(_lib.McdcError) as ei:
            ctx.zstd_frames(dp, data.size, ch, d_out, 1024)
        assert ei.value.code == _lib.MCDC_E_CAPACITY
    finally:
        ctx.device_free(d_out)
        ctx.device_free(dp)


def test_misaligned_output_rejected(ctx):
    """k_zframe_write stores 16-byte quads: an output pointer off the 16-byte
    grid is refused up front (MCDC_E_INVALID), an aligned sub-buffer works."""
    data = O.random_bytes(100_003, 2)
    ch = np.zeros(1, dtype=_lib.CHUNK_DTYPE)
    ch["length"] = data.size
    dp = ctx.device_alloc(data.size)
    d_out = ctx.device_alloc(data.size + 4096)
    try:
        ctx.h2d(dp, data)
        for shift in (1, 4, 8):
            with pytest.raises(_lib.McdcError) as ei:
                ctx.zstd_frames(dp, data.size, ch, d_out + shift, data.size + 1024)
            assert ei.value.code == _lib.MCDC_E_INVALID
        fr, _ = ctx.zstd_frames(dp, data.size, ch, d_out + 32, data.size + 1024)
        got = ctx.d2h_bytes(d_out + 32 + int(fr[0, 0]), int(fr[0, 1]))
        assert got.tobytes() == O.zstd_raw_frame(data.tobytes())
    finally:
        ctx.device_free(d_out)
        ctx.device_free(dp)
