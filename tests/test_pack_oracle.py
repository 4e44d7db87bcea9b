"""The packer restatement (oracle.pack_flush / parse_header / pack_header,
restating /root/reference/src/repository/packer.rs:113-285) pinned by the
reference's own packer tests:

* test_pack_flush (packer.rs:345-378): blobs b"mapache", b"backup", b"rust"
  (IDs = ID::from_content, BlobType::Data), flushed with
  SecureStorage::build() (no key, compression level 0 = zstd's default):
  the pack is exactly 2398 bytes, flush returns 64 descriptors (3 + 61
  padding), parse_header returns 3, and the two lists differ;
* test_empty_pack_flush (packer.rs:380-395): an empty packer flushes to None.

2398 = 17 bytes of blobs + the encoded header + 4: the header is 64 x 37 =
2368 bytes of mostly random bytes, which zstd stores as one raw block in a
frame without a content size (the crate's streaming encoder) -- 6 + 3 + 2368
= 2377 -- so the KAT also pins the frame layout the GPU store mode writes
(oracle.zstd_raw_frame)."""
import numpy as np

from oracle import oracle as O


def _kat_inputs(seed=1):
    blobs = [b"mapache", b"backup", b"rust"]
    ids = [O.blake3(np.frombuffer(b, np.uint8)) for b in blobs]
    rng = np.random.default_rng(seed)
    padding = [(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), int(rng.integers(0, 2**32)),
                int(rng.integers(0, 2**32))) for _ in range(61)]
    return blobs, ids, padding


def test_reference_pack_flush_kat():
    blobs, ids, padding = _kat_inputs()
    data, desc = O.pack_flush(blobs, ids, [0, 0, 0], padding)
    assert len(data) == 2398  # packer.rs:368
    assert len(desc) == 64  # :372
    hdr = O.parse_header(data)
    assert len(hdr) == 3  # :373
    assert hdr != desc  # :374
    assert hdr == [(ids[0], 0, 0, 7), (ids[1], 0, 7, 6), (ids[2], 0, 13, 4)]
    # the encoded header is a raw-block frame without content size: exactly
    # the GPU store mode's frame of the header bytes
    enc = data[17:-4]
    header = O.pack_header(ids, [7, 6, 4], [0, 0, 0],
                           [p[0] + p[2].to_bytes(4, "little") for p in padding])
    assert len(header) == 64 * 37
    assert enc == O.zstd_raw_frame(header)


def test_reference_pack_flush_kat_any_padding():
    """The size does not depend on the random padding draws."""
    for seed in range(2, 6):
        blobs, ids, padding = _kat_inputs(seed)
        assert len(O.pack_flush(blobs, ids, [0, 0, 0], padding)[0]) == 2398


def test_reference_empty_pack_flush():
    assert O.pack_flush([], [], [], []) is None  # packer.rs:380-395


def test_pack_flush_with_key_round_trips():
    """With a key the header is sealed (28 more bytes: nonce + tag) and
    parse_header with the same key recovers the real descriptors."""
    blobs, ids, padding = _kat_inputs()
    key, nonce = bytes(range(32)), bytes(range(12))
    data, desc = O.pack_flush(blobs, ids, [0, 1, 0], padding, key, nonce)
    assert len(data) == 2398 + 28
    assert O.parse_header(data, key) == [(ids[0], 0, 0, 7), (ids[1], 1, 7, 6), (ids[2], 0, 13, 4)]
