"""ctypes front-end of the FastCDC v2020 CPU restatement (oracle/fastcdc_oracle.c).

TEST INFRASTRUCTURE ONLY — the parity checker and the timed CPU baseline.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  The product path
(``mapache_amd``) never does.

Provenance: see ``fastcdc_oracle.h``.  The reference's chunker is the
un-vendored crate ``fastcdc`` 3.2.1 (``/root/reference/Cargo.lock:449-452``)
called at ``/root/reference/src/archiver/processor.rs:173-179``; parity is
"vs this restatement" (pinned by the GEAR derivation, the MASKS popcounts and
the crate's recalled ``test_all_zeros`` KAT).  Also holds a pure-Python loop
(``cut_gear_py``) used as a third, independent statement on small inputs.
"""
from __future__ import annotations

import ctypes
import hashlib
import math
import os
import subprocess
import threading
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

MINIMUM_MIN, MINIMUM_MAX = 64, 1_048_576
AVERAGE_MIN, AVERAGE_MAX = 256, 4_194_304
MAXIMUM_MIN, MAXIMUM_MAX = 1024, 16_777_216


class OcParams(ctypes.Structure):
    _fields_ = [
        ("min_size", ctypes.c_uint32), ("avg_size", ctypes.c_uint32),
        ("max_size", ctypes.c_uint32), ("level", ctypes.c_uint32),
        ("mask_s", ctypes.c_uint64), ("mask_l", ctypes.c_uint64),
        ("mask_s_ls", ctypes.c_uint64), ("mask_l_ls", ctypes.c_uint64),
    ]


CHUNK_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("hash", "<u8")])


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oc_params_init.argtypes = [ctypes.POINTER(OcParams), ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32]
        L.oc_params_init.restype = ctypes.c_int
        for name in ("oc_gear", "oc_gear_ls", "oc_masks"):
            getattr(L, name).argtypes = [u64p]
            getattr(L, name).restype = None
        L.oc_logarithm2.argtypes = [ctypes.c_uint32]
        L.oc_logarithm2.restype = ctypes.c_uint32
        for name in ("oc_cut_gear", "oc_cut_gear_1byte"):
            getattr(L, name).argtypes = [ctypes.POINTER(OcParams), ctypes.c_void_p, ctypes.c_size_t,
                                         u64p, ctypes.POINTER(ctypes.c_size_t)]
            getattr(L, name).restype = None
        for name in ("oc_chunk_slice", "oc_chunk_slice_1byte"):
            getattr(L, name).argtypes = [ctypes.POINTER(OcParams), ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_size_t]
            getattr(L, name).restype = ctypes.c_size_t
        L.oc_chunk_stream.argtypes = [ctypes.POINTER(OcParams), ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        L.oc_chunk_stream.restype = ctypes.c_size_t
        L.oc_chunk_files.argtypes = [ctypes.POINTER(OcParams), ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p]
        L.oc_chunk_files.restype = ctypes.c_size_t
        L.oc_chunk_digest.argtypes = [ctypes.POINTER(OcParams), ctypes.c_void_p, ctypes.c_size_t, u64p]
        L.oc_chunk_digest.restype = ctypes.c_size_t
        L.oc_random_stream_digest.argtypes = [ctypes.POINTER(OcParams), ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_size_t, u64p, u64p]
        L.oc_random_stream_digest.restype = ctypes.c_size_t
        L.oc_random_stream_digest_h.argtypes = [ctypes.POINTER(OcParams), ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_size_t, u64p, u64p, u64p]
        L.oc_random_stream_digest_h.restype = ctypes.c_size_t
        L.oc_random_files_digest.argtypes = [ctypes.POINTER(OcParams), ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]
        L.oc_random_files_digest.restype = ctypes.c_int
        L.oc_hash_digest.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oc_hash_digest.restype = ctypes.c_uint64
        L.oc_fill_random.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint64]
        L.oc_fill_random.restype = None
        L.oc_file_seed.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oc_file_seed.restype = ctypes.c_uint64
        L.oc_digest_step.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oc_digest_step.restype = ctypes.c_uint64
        L.ob_hash.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.ob_hash.restype = None
        L.ob_chunk_ids.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
        L.ob_chunk_ids.restype = None
        vp = ctypes.c_void_p
        L.oa_sbox.argtypes = [vp]
        L.oa_aes_encrypt_block.argtypes = [vp, ctypes.c_int, vp, vp]
        L.oa_aes_encrypt_block.restype = ctypes.c_int
        L.oa_dot.argtypes = [vp, vp, vp]
        L.oa_polyval.argtypes = [vp, vp, ctypes.c_size_t, vp]
        L.oa_siv_derive.argtypes = [vp, vp, vp, vp]
        for name in ("oa_siv_encrypt", "oa_siv_decrypt"):
            getattr(L, name).argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp]
            getattr(L, name).restype = ctypes.c_int
        L.oa_seal_blobs.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp, vp, ctypes.c_int]
        L.oa_seal_blobs.restype = None
        _lib = L
    return _lib


# ----------------------------------------------------------------- params --
@dataclass(frozen=True)
class Params:
    min_size: int
    avg_size: int
    max_size: int
    level: int = 1

    def c(self) -> OcParams:
        p = OcParams()
        if lib().oc_params_init(ctypes.byref(p), self.min_size, self.avg_size, self.max_size, self.level) != 0:
            raise ValueError(f"invalid FastCDC params {self}")
        return p


P16 = Params(16 * 1024, 64 * 1024, 256 * 1024, 1)      # BASELINE.json configs
P512 = Params(512 * 1024, 1024 * 1024, 8 * 1024 * 1024, 1)  # reference defaults.rs:35-40


def tables():
    g = (ctypes.c_uint64 * 256)()
    gl = (ctypes.c_uint64 * 256)()
    m = (ctypes.c_uint64 * 26)()
    lib().oc_gear(g)
    lib().oc_gear_ls(gl)
    lib().oc_masks(m)
    return list(g), list(gl), list(m)


def gear_md5() -> list[int]:
    """Independent derivation with Python's hashlib."""
    return [int.from_bytes(hashlib.md5(bytes([i]) * 64).digest()[:8], "big") for i in range(256)]


# -------------------------------------------------------------- chunking --
def _buf(data):
    a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data,
                             dtype=np.uint8)
    return a, a.ctypes.data


def cut_gear(params: Params, data, one_byte: bool = False):
    a, ptr = _buf(data)
    h = ctypes.c_uint64()
    c = ctypes.c_size_t()
    fn = lib().oc_cut_gear_1byte if one_byte else lib().oc_cut_gear
    fn(ctypes.byref(params.c()), ptr, a.size, ctypes.byref(h), ctypes.byref(c))
    return h.value, c.value


def chunk(params: Params, data, one_byte: bool = False) -> np.ndarray:
    """FastCDC over a whole slice -> structured array (offset, length, hash)."""
    a, ptr = _buf(data)
    cap = a.size // max(params.min_size - 1, 1) + 2
    out = np.zeros(cap, dtype=CHUNK_DTYPE)
    fn = lib().oc_chunk_slice_1byte if one_byte else lib().oc_chunk_slice
    k = fn(ctypes.byref(params.c()), ptr, a.size, out.ctypes.data, cap)
    assert k <= cap
    return out[:k].copy()


def chunk_stream(params: Params, data, read_quantum: int) -> np.ndarray:
    a, ptr = _buf(data)
    cap = a.size // max(params.min_size - 1, 1) + 2
    out = np.zeros(cap, dtype=CHUNK_DTYPE)
    k = lib().oc_chunk_stream(ctypes.byref(params.c()), ptr, a.size, read_quantum, out.ctypes.data, cap)
    return out[:k].copy()


def chunk_files(params: Params, files, threads: int = 1):
    arrs = [np.ascontiguousarray(np.frombuffer(f, dtype=np.uint8) if not isinstance(f, np.ndarray) else f,
                                 dtype=np.uint8) for f in files]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[x.ctypes.data for x in arrs])
    lens = (ctypes.c_size_t * max(n, 1))(*[x.size for x in arrs])
    cap = sum(x.size // max(params.min_size - 1, 1) + 2 for x in arrs)
    out = np.zeros(max(cap, 1), dtype=CHUNK_DTYPE)
    counts = np.zeros(max(n, 1), dtype=np.uint64)
    k = lib().oc_chunk_files(ctypes.byref(params.c()), ptrs, lens, n, threads, out.ctypes.data, cap,
                             counts.ctypes.data)
    if k == ctypes.c_size_t(-1).value:
        raise RuntimeError("oc_chunk_files failed")
    return out[:k].copy(), counts[:n].astype(np.int64)


def chunk_digest(params: Params, data):
    a, ptr = _buf(data)
    d = ctypes.c_uint64()
    k = lib().oc_chunk_digest(ctypes.byref(params.c()), ptr, a.size, ctypes.byref(d))
    return k, d.value


def random_stream_digest(params: Params, seed: int, n: int, slab: int = 256 << 20, hashes: bool = False):
    """(count, digest, sum of lengths) of the counter-based stream [0, n) chunked
    as one file, regenerated slab by slab (no n-byte buffer): full-size parity.
    hashes=True appends the hash digest (hash_digest of every ChunkData.hash)."""
    d, sm, hd = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    k = lib().oc_random_stream_digest_h(ctypes.byref(params.c()), seed, n, slab, ctypes.byref(d), ctypes.byref(sm),
                                        ctypes.byref(hd))
    return (k, d.value, sm.value, hd.value) if hashes else (k, d.value, sm.value)


def random_files_digest(params: Params, seeds, pos, lens, threads: int = 16):
    """(counts, digests, hash digests) per file; file i = bytes [pos[i], pos[i] +
    lens[i]) of the counter-based stream of seeds[i], chunked as one file
    (oc_random_files_digest: regenerated per file on `threads` threads, so the
    host never holds the corpus).  digests[i] == mcdc digest of the file's
    boundary list (file-relative offsets), hash digests == hash_digest."""
    n = len(lens)
    a = [np.ascontiguousarray(np.broadcast_to(np.asarray(x, dtype=np.uint64), (n,))) for x in (seeds, pos, lens)]
    counts, dig, hd = (np.zeros(max(n, 1), np.uint64) for _ in range(3))
    rc = lib().oc_random_files_digest(ctypes.byref(params.c()), a[0].ctypes.data, a[1].ctypes.data,
                                      a[2].ctypes.data, n, threads, counts.ctypes.data, dig.ctypes.data,
                                      hd.ctypes.data)
    if rc:
        raise RuntimeError("oc_random_files_digest failed")
    return counts[:n], dig[:n], hd[:n]


def hash_digest(chunks: np.ndarray) -> int:
    """Order-sensitive digest of a boundary list's hash column (oc_hash_digest)."""
    h = np.ascontiguousarray(chunks["hash"], dtype=np.uint64)
    return int(lib().oc_hash_digest(h.ctypes.data, h.size))


def digest_of(chunks: np.ndarray) -> int:
    d = 0
    step = lib().oc_digest_step
    for off, ln in zip(chunks["offset"].tolist(), chunks["length"].tolist()):
        d = step(d, off, ln)
    return d


def random_bytes(n: int, seed: int, pos: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    lib().oc_fill_random(out.ctypes.data, pos, n, seed)
    return out


def file_seed(seed: int, index: int) -> int:
    return lib().oc_file_seed(seed, index)


# ------------------------------------------------- pure-Python statement --
_M64 = (1 << 64) - 1


def cut_gear_py(params: Params, src: bytes):
    """Third statement of crate cut_gear (2-byte loop), pure Python, small inputs only."""
    g = gear_md5()
    gls = [(x << 1) & _M64 for x in g]
    _, _, masks = tables()
    bits = round(math.log2(params.avg_size))
    ms, ml = masks[bits + params.level], masks[bits - params.level]
    msl, mll = (ms << 1) & _M64, (ml << 1) & _M64
    remaining = len(src)
    if remaining <= params.min_size:
        return 0, remaining
    center = params.avg_size
    if remaining > params.max_size:
        remaining = params.max_size
    elif remaining < center:
        center = remaining
    index, h = params.min_size // 2, 0
    while index < center // 2:
        a = 2 * index
        h = ((h << 2) + gls[src[a]]) & _M64
        if h & msl == 0:
            return h, a
        h = (h + g[src[a + 1]]) & _M64
        if h & ms == 0:
            return h, a + 1
        index += 1
    while index < remaining // 2:
        a = 2 * index
        h = ((h << 2) + gls[src[a]]) & _M64
        if h & mll == 0:
            return h, a
        h = (h + g[src[a + 1]]) & _M64
        if h & ml == 0:
            return h, a + 1
        index += 1
    return h, remaining


# --------------------------------------------------------------- BLAKE3 --
# Chunk IDs: ID::from_content = blake3::Hasher (unkeyed, 32-byte output)
# over each chunk's bytes (/root/reference/src/global/mod.rs:86-88,
# src/utils/mod.rs:62-68, used at src/archiver/processor.rs:184).
def blake3(data) -> bytes:
    """BLAKE3 of `data` by the C restatement (oracle/blake3_oracle.c)."""
    a, ptr = _buf(data)
    out = ctypes.create_string_buffer(32)
    lib().ob_hash(ptr, a.size, out)
    return out.raw


def chunk_ids(data, chunks: np.ndarray, threads: int = 1) -> np.ndarray:
    """(n, 32) uint8: BLAKE3 of every chunk [offset, offset + length) of `data`."""
    a, ptr = _buf(data)
    off = np.ascontiguousarray(chunks["offset"], dtype=np.uint64)
    ln = np.ascontiguousarray(chunks["length"], dtype=np.uint64)
    out = np.zeros((max(len(off), 1), 32), dtype=np.uint8)
    lib().ob_chunk_ids(ptr, off.ctypes.data, ln.ctypes.data, len(off), threads, out.ctypes.data)
    return out[: len(off)]


_B3_IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19)
_B3_PERM = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
_M32 = 0xFFFFFFFF


def _b3_compress(cv, m, counter, block_len, flags):
    def rotr(x, n):
        return ((x >> n) | (x << (32 - n))) & _M32
    s = list(cv) + list(_B3_IV[:4]) + [counter & _M32, counter >> 32, block_len, flags]
    m = list(m)
    for r in range(7):
        for (a, b, c, d), (x, y) in zip(((0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15),
                                         (0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)),
                                        ((0, 1), (2, 3), (4, 5), (6, 7), (8, 9), (10, 11), (12, 13), (14, 15))):
            s[a] = (s[a] + s[b] + m[x]) & _M32
            s[d] = rotr(s[d] ^ s[a], 16)
            s[c] = (s[c] + s[d]) & _M32
            s[b] = rotr(s[b] ^ s[c], 12)
            s[a] = (s[a] + s[b] + m[y]) & _M32
            s[d] = rotr(s[d] ^ s[a], 8)
            s[c] = (s[c] + s[d]) & _M32
            s[b] = rotr(s[b] ^ s[c], 7)
        m = [m[_B3_PERM[i]] for i in range(16)]
    return [s[i] ^ s[i + 8] for i in range(8)]


def blake3_py(data: bytes) -> bytes:
    """Second, independent statement (pure Python, small inputs): the tree by
    its recursive definition — the left subtree holds the largest power-of-two
    number of 1024-byte chunks that leaves at least one chunk on the right."""
    def chunk(p, counter, root):
        cv = list(_B3_IV)
        blocks = [p[i:i + 64] for i in range(0, len(p), 64)] or [b""]
        for i, b in enumerate(blocks):
            m = [int.from_bytes((b + bytes(64 - len(b)))[4 * k:4 * k + 4], "little") for k in range(16)]
            fl = (1 if i == 0 else 0) | (2 if i == len(blocks) - 1 else 0) | (8 if root and i == len(blocks) - 1 else 0)
            cv = _b3_compress(cv, m, counter, len(b), fl)
        return cv

    def node(p, c0, root):
        n = max(1, -(-len(p) // 1024))
        if n == 1:
            return chunk(p, c0, root)
        left = 1 << ((n - 1).bit_length() - 1)
        lcv, rcv = node(p[:1024 * left], c0, False), node(p[1024 * left:], c0 + left, False)
        return _b3_compress(_B3_IV, lcv + rcv, 0, 64, 4 | (8 if root else 0))

    return b"".join(w.to_bytes(4, "little") for w in node(bytes(data), 0, True))


# ---------------------------------------------------------- AES-GCM-SIV --
# SecureStorage's encryption: AES-256-GCM-SIV (crate aes-gcm-siv 0.11.1), no
# AAD, random 12-byte nonce, blob = nonce || ciphertext || tag
# (/root/reference/src/repository/storage.rs:97-118).  C restatement in
# oracle/aead_oracle.c (RFC 8452 over FIPS-197).
NONCE_BYTES, TAG_BYTES = 12, 16
SEAL_OVERHEAD = NONCE_BYTES + TAG_BYTES


def _bytes(x) -> bytes:
    return bytes(x) if not isinstance(x, np.ndarray) else x.tobytes()


def aes_sbox() -> bytes:
    out = ctypes.create_string_buffer(256)
    lib().oa_sbox(out)
    return out.raw


def aes_encrypt_block(key, block) -> bytes:
    key, block = _bytes(key), _bytes(block)
    assert len(block) == 16
    out = ctypes.create_string_buffer(16)
    if lib().oa_aes_encrypt_block(key, len(key), block, out) != 0:
        raise ValueError("AES key must be 16 or 32 bytes")
    return out.raw


def polyval_dot(a, b) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().oa_dot(_bytes(a), _bytes(b), out)
    return out.raw


def polyval(h, x) -> bytes:
    x = _bytes(x)
    assert len(x) % 16 == 0
    out = ctypes.create_string_buffer(16)
    lib().oa_polyval(_bytes(h), x, len(x) // 16, out)
    return out.raw


def siv_derive(key, nonce):
    """(message-authentication key, message-encryption key) of RFC 8452 §4."""
    a, e = ctypes.create_string_buffer(16), ctypes.create_string_buffer(32)
    lib().oa_siv_derive(_bytes(key), _bytes(nonce), a, e)
    return a.raw, e.raw


def siv_encrypt(key, nonce, plaintext, aad=b"") -> bytes:
    """ciphertext || tag (RFC 8452 §4); key 16 or 32 bytes."""
    key, nonce, pt, aad = _bytes(key), _bytes(nonce), _bytes(plaintext), _bytes(aad)
    assert len(nonce) == NONCE_BYTES
    out = ctypes.create_string_buffer(len(pt) + TAG_BYTES)
    if lib().oa_siv_encrypt(key, len(key), nonce, aad, len(aad), pt, len(pt), out) != 0:
        raise ValueError("bad key length")
    return out.raw


def siv_decrypt(key, nonce, ct_tag, aad=b""):
    """plaintext, or None when the tag does not verify (RFC 8452 §5)."""
    key, nonce, ct, aad = _bytes(key), _bytes(nonce), _bytes(ct_tag), _bytes(aad)
    if len(ct) < TAG_BYTES:
        return None
    out = ctypes.create_string_buffer(max(len(ct) - TAG_BYTES, 1))
    if lib().oa_siv_decrypt(key, len(key), nonce, aad, len(aad), ct, len(ct), out) != 0:
        return None
    return out.raw[: len(ct) - TAG_BYTES]


def encrypt_with_key(key, nonce, data) -> bytes:
    """storage.rs:97-118 with the nonce made explicit: nonce || ct || tag."""
    return _bytes(nonce) + siv_encrypt(key, nonce, data)


def decrypt_with_key(key, blob):
    """storage.rs:120-139: split the nonce off, open; None on failure."""
    blob = _bytes(blob)
    if len(blob) < SEAL_OVERHEAD:
        return None
    return siv_decrypt(key, blob[:NONCE_BYTES], blob[NONCE_BYTES:])


def seal_blobs(key, data, offsets, lengths, nonces, threads: int = 1):
    """Every blob [offsets[i], +lengths[i]) of `data` sealed as nonce || ct ||
    tag, packed back to back -> (out bytes as uint8 array, out offsets)."""
    a, ptr = _buf(data)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint64)
    nz = np.ascontiguousarray(nonces, dtype=np.uint8).reshape(-1, NONCE_BYTES)
    assert len(off) == len(ln) == len(nz)
    out_off = np.concatenate([[0], np.cumsum(ln + SEAL_OVERHEAD)]).astype(np.uint64)
    out = np.zeros(max(int(out_off[-1]), 1), dtype=np.uint8)
    lib().oa_seal_blobs(_bytes(key), ptr, off.ctypes.data, ln.ctypes.data, len(off), nz.ctypes.data,
                        out.ctypes.data, out_off.ctypes.data, threads)
    return out[: int(out_off[-1])], out_off[:-1]


# ------------------------------------------------------------ dedup index --
class DedupIndex:
    """Restates the blob-exists check of Repository::save_blob
    (/root/reference/src/repository/repository_v1.rs:169-180):
        blob_exists = index.contains(&id) || !index.add_pending_blob(id)
    in processing order: an ID is stored (new) the first time it is seen,
    within a batch and across batches; later equal IDs are only referenced."""

    def __init__(self):
        self.seen = set()

    def __len__(self):
        return len(self.seen)

    def add(self, ids) -> np.ndarray:
        a = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 32)
        out = np.zeros(a.shape[0], dtype=bool)
        for i in range(a.shape[0]):
            k = a[i].tobytes()
            if k not in self.seen:
                self.seen.add(k)
                out[i] = True
        return out


# ----------------------------------------------------------------- packer --
HEADER_BLOB_LEN, HEADER_BLOB_MULTIPLE = 37, 64  # packer.rs:30, defaults.rs:32


def pack_plan(lengths, max_pack_size: int):
    """Restates Repository::save_blob's flush rule (repository_v1.rs:185-193:
    add the blob, then flush once the packer holds more than max_pack_size
    bytes) plus the final flush: [(first, end)) blob ranges per pack."""
    plan, size, first = [], 0, None
    for i, n in enumerate(lengths):
        if first is None:
            first = i
        size += int(n)
        if size > max_pack_size:
            plan.append((first, i + 1))
            size, first = 0, None
    if first is not None:
        plan.append((first, len(lengths)))
    return plan


def pack_header(ids, lengths, types, padding36) -> bytes:
    """Packer::generate_header (packer.rs:156-186): per blob ID || le32 length ||
    type, padded to a multiple of 64 entries with (36 random bytes, 0xff);
    padding36: the random bytes of the padding entries, in order."""
    out = bytearray()
    for i in range(len(lengths)):
        out += bytes(ids[i]) + int(lengths[i]).to_bytes(4, "little") + bytes([int(types[i])])
    for p in padding36:
        out += bytes(p) + b"\xff"
    return bytes(out)


# ------------------------------------------------------- zstd raw frames --
def zstd_raw_frame(data) -> bytes:
    """RFC 8878 frame in raw-block mode, as mcdc_zstd_frames_device writes it:
    magic, Frame_Header_Descriptor 0 (no content size, not single-segment, no
    checksum, no dictionary), Window_Descriptor 0x50 (2^20, storage.rs:31),
    raw blocks of <= 128 KiB with 3-byte headers (Last_Block | Raw << 1 |
    Block_Size << 3); an empty input is one empty last block."""
    data = bytes(data)
    out = bytearray(b"\x28\xb5\x2f\xfd\x00\x50")
    blocks = [data[i:i + 131072] for i in range(0, len(data), 131072)] or [b""]
    for k, b in enumerate(blocks):
        h = (1 if k + 1 == len(blocks) else 0) | (len(b) << 3)
        out += h.to_bytes(3, "little") + b
    return bytes(out)


# ------------------------------------------------------------ zstd codec --
class Zstd:
    """The system libzstd (1.4.8 here; the crate links 1.5.7) through ctypes:
    the test-side reference codec for SecureStorage's compression
    (storage.rs:74-94: level 3, window log 20, no checksum; decoded with
    window_log_max 20).  Compressed bytes depend on the version: parity on
    compressed data is decode-equality."""

    _lib = None  # (the loaded library, set up once per process)

    def __init__(self):
        import ctypes
        if Zstd._lib is not None:
            self.z, self.ct = Zstd._lib, ctypes
            return
        z = ctypes.CDLL("libzstd.so.1")
        z.ZSTD_createCCtx.restype = ctypes.c_void_p
        z.ZSTD_createDCtx.restype = ctypes.c_void_p
        z.ZSTD_compressBound.restype = ctypes.c_size_t
        z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
        z.ZSTD_compress2.restype = ctypes.c_size_t
        z.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                     ctypes.c_size_t]
        z.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        z.ZSTD_DCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        z.ZSTD_decompressDCtx.restype = ctypes.c_size_t
        z.ZSTD_decompressDCtx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_size_t]
        z.ZSTD_compressStream2.restype = ctypes.c_size_t
        z.ZSTD_compressStream2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        z.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong
        z.ZSTD_getFrameContentSize.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        z.ZSTD_isError.argtypes = [ctypes.c_size_t]
        z.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
        z.ZSTD_freeDCtx.argtypes = [ctypes.c_void_p]
        self.z, self.ct = z, ctypes
        Zstd._lib = z

    def compress(self, data: bytes, content_size: bool, level: int = 3) -> bytes:
        """content_size=True: one-shot ZSTD_compress2 (size known: content size in
        the frame, window fitted to the input).  False: the crate's streaming
        encoder (ZstdEncoder::write_all + finish, storage.rs:75-83): the data
        is passed with ZSTD_e_continue, then ZSTD_e_end flushes -- the size is
        never pledged, so the frame has no content size and keeps the 2^20
        window descriptor."""
        z, ct = self.z, self.ct
        c = z.ZSTD_createCCtx()
        z.ZSTD_CCtx_setParameter(c, 100, level)  # level (0: zstd's default, 3)
        z.ZSTD_CCtx_setParameter(c, 101, 20)  # window log
        z.ZSTD_CCtx_setParameter(c, 201, 0)  # checksum off
        z.ZSTD_CCtx_setParameter(c, 200, 1 if content_size else 0)  # content size flag
        out = ct.create_string_buffer(z.ZSTD_compressBound(len(data)) + 64)
        if content_size:
            r = z.ZSTD_compress2(c, out, len(out), data, len(data))
            z.ZSTD_freeCCtx(c)
            assert not z.ZSTD_isError(r)
            return out.raw[:r]

        class Buf(ct.Structure):
            _fields_ = [("ptr", ct.c_void_p), ("size", ct.c_size_t), ("pos", ct.c_size_t)]
        src = ct.create_string_buffer(bytes(data), max(len(data), 1))
        ib, ob = Buf(ct.addressof(src), len(data), 0), Buf(ct.addressof(out), len(out), 0)
        r = z.ZSTD_compressStream2(c, ct.byref(ob), ct.byref(ib), 0)  # ZSTD_e_continue
        assert not z.ZSTD_isError(r) and ib.pos == len(data)
        while True:
            r = z.ZSTD_compressStream2(c, ct.byref(ob), ct.byref(ib), 2)  # ZSTD_e_end
            assert not z.ZSTD_isError(r)
            if r == 0:
                break
        z.ZSTD_freeCCtx(c)
        return out.raw[:ob.pos]

    _tls = threading.local()

    def decompress(self, frame: bytes, size: int) -> bytes:
        z = self.z
        d = z.ZSTD_createDCtx()
        z.ZSTD_DCtx_setParameter(d, 100, 20)  # window_log_max 20 (storage.rs:90)
        # (one output buffer per thread, reused: a fresh zero-filled buffer of
        # the size hint per frame, under the GIL, cost a 72 000-blob decode
        # minutes; only the r decoded bytes are copied out)
        out = getattr(Zstd._tls, "buf", None)
        if out is None or len(out) < max(size, 1):
            out = Zstd._tls.buf = self.ct.create_string_buffer(max(size, 1))
        r = z.ZSTD_decompressDCtx(d, out, max(size, 1), frame, len(frame))
        z.ZSTD_freeDCtx(d)
        assert not z.ZSTD_isError(r), "not a zstd frame within a 2^20 window"
        return self.ct.string_at(out, r)


# ------------------------------------------------- SecureStorage + Packer --
def storage_encode(data: bytes, key=None, nonce=None, level: int = 0) -> bytes:
    """SecureStorage::encode (storage.rs:61-65): compress as the crate's
    streaming encoder does (:74-84; no content size in the frame), then
    encrypt_with_key when there is a key (:120-125; the identity without one:
    SecureStorage::build())."""
    c = Zstd().compress(bytes(data), content_size=False, level=level)
    return c if key is None else encrypt_with_key(key, nonce, c)


def storage_decode(blob: bytes, key=None, size_hint: int = 1 << 24) -> bytes:
    """SecureStorage::decode (storage.rs:67-69): decrypt (identity without a
    key), then decompress within a 2^20 window."""
    if key is not None:
        blob = decrypt_with_key(key, blob)
        if blob is None:
            raise ValueError("Decryption failed")
    return Zstd().decompress(bytes(blob), size_hint)


def pack_flush(blobs, ids, types, padding, key=None, nonce=None):
    """Packer::flush (packer.rs:113-153) of the blobs added in order:
    None for an empty packer (:114-116); else (data, descriptors) with
    data = blobs back to back || encode(generate_header) || le32(len) and
    descriptors = (id, type, offset, length) of the blobs followed by the
    padding descriptors generate_header appends (:160-171).  padding: one
    (id32, offset, length) per padding entry the header needs (the crate
    draws them from its RNG)."""
    if not blobs:
        return None
    data, desc, off = bytearray(), [], 0
    for b, i, t in zip(blobs, ids, types):
        desc.append((bytes(i), int(t), off, len(b)))
        data += bytes(b)
        off += len(b)
    npad = (HEADER_BLOB_MULTIPLE - len(desc) % HEADER_BLOB_MULTIPLE) % HEADER_BLOB_MULTIPLE
    for j in range(npad):
        pid, poff, plen = padding[j]
        desc.append((bytes(pid), 0xFF, int(poff), int(plen)))
    header = b"".join(d[0] + (d[3] & 0xFFFFFFFF).to_bytes(4, "little") + bytes([d[1]]) for d in desc)
    enc = storage_encode(header, key, nonce)
    data += enc + len(enc).to_bytes(4, "little")
    return bytes(data), desc


def parse_header(header_data: bytes, key=None):
    """Packer::parse_header (packer.rs:214-285): the le32 length at the end, the
    encoded header before it, decoded; 37-byte entries; padding entries
    (type 0xff) skipped; offsets are the running sum of the real entries'
    lengths.  Returns [(id, type, offset, length)]."""
    if len(header_data) < 4:
        raise ValueError("Pack header is invalid: data too short for header length")
    hl = int.from_bytes(header_data[-4:], "little")
    if len(header_data) < hl:
        raise ValueError("Pack header is invalid: declared header_length exceeds total data length")
    info = storage_decode(header_data[len(header_data) - hl - 4:len(header_data) - 4], key)
    if len(info) % HEADER_BLOB_LEN:
        raise ValueError("Pack header is invalid: not a multiple of the descriptor size")
    out, cur = [], 0
    for j in range(len(info) // HEADER_BLOB_LEN):
        e = info[j * HEADER_BLOB_LEN:(j + 1) * HEADER_BLOB_LEN]
        if e[36] == 0xFF:
            continue
        ln = int.from_bytes(e[32:36], "little")
        out.append((bytes(e[:32]), e[36], cur, ln))
        cur += ln
    return out


MIN_CHUNK_SIZE = 512 << 10  # global::defaults::MIN_CHUNK_SIZE (/root/reference/src/global/defaults.rs:35)


def save_files(params: Params, files, index=None, key=None, nonces=None, header_nonces=None, padding=None,
               max_pack_size: int = 16 << 20, threads: int = 8, gate_bytes: int = MIN_CHUNK_SIZE):
    """The Archiver's save path for a run of files, in file order, restated
    (test infrastructure; the product is mcdc_save_files):

    * processor::save_file (processor.rs:138-157): a file smaller than
      MIN_CHUNK_SIZE (the constant, :144-145, whatever the chunker's min;
      gate_bytes, default 512 KiB) is one blob, ID = ID::from_content of
      the whole file (SaveID::CalculateID); otherwise chunk_and_save_blobs
      (:160-205): StreamCDC chunks, ID::from_content per chunk, in order;
    * Repository::save_blob (repository_v1.rs:155-195) per blob: skip it when
      index.contains(id) || !add_pending_blob(id) (:173-180, DedupIndex), else
      SecureStorage::encode (:182; storage_encode: nonces[k] for the k-th
      stored blob) and Packer::add_blob, flushing once the packer holds more
      than max_pack_size bytes (:185-192); one final flush at the end
      (Repository::flush at the end of the snapshot);
    * Packer::flush (pack_flush): header_nonces[j] for the j-th pack, padding
      entries drawn in order from `padding` (36 bytes each).

    Returns (ids_per_file: list of (k, 32) uint8 arrays, is_new: bool per blob
    in processing order, packs: list of (data, descriptors))."""
    index = DedupIndex() if index is None else index
    per_file, blob_bytes = [], []
    for f in files:
        a = np.ascontiguousarray(np.frombuffer(f, np.uint8) if not isinstance(f, np.ndarray) else f, np.uint8)
        if a.size < gate_bytes:
            ch = np.zeros(1, dtype=CHUNK_DTYPE)
            ch["length"] = a.size
        else:
            ch = chunk(params, a)
        ids = chunk_ids(a, ch, threads=threads if a.size >= (4 << 20) else 1)
        per_file.append(ids)
        blob_bytes += [a[int(o):int(o + n)].tobytes() for o, n in zip(ch["offset"], ch["length"])]
    all_ids = np.concatenate(per_file) if per_file else np.zeros((0, 32), np.uint8)
    is_new = index.add(all_ids) if len(all_ids) else np.zeros(0, bool)
    stored = [(all_ids[i].tobytes(), blob_bytes[i]) for i in np.nonzero(is_new)[0]]
    from concurrent.futures import ThreadPoolExecutor  # (libzstd and the AES oracle run outside the GIL)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        enc = list(ex.map(lambda kb: storage_encode(kb[1][1], key, None if key is None else bytes(nonces[kb[0]])),
                          enumerate(stored)))
    packs, pad_at = [], 0
    for j, (f0, f1) in enumerate(pack_plan([len(e) for e in enc], max_pack_size)):
        cnt = f1 - f0
        npad = (HEADER_BLOB_MULTIPLE - cnt % HEADER_BLOB_MULTIPLE) % HEADER_BLOB_MULTIPLE
        pad = [(bytes(padding[pad_at + t][:32]), 0, int.from_bytes(bytes(padding[pad_at + t][32:36]), "little"))
               for t in range(npad)]
        pad_at += npad
        packs.append(pack_flush(enc[f0:f1], [stored[i][0] for i in range(f0, f1)], [0] * cnt, pad, key,
                                None if key is None else bytes(header_nonces[j])))
    return per_file, is_new, packs
