"""Pins the AES-256-GCM-SIV restatement (oracle/aead_oracle.c) before any GPU
result is compared with it.

mapache seals every blob with AES-256-GCM-SIV (crate aes-gcm-siv 0.11.1,
/root/reference/Cargo.toml:13; storage.rs:97-118) and its own test only round
trips (storage.rs:235-247), so the reference holds no vectors: parity is
"unpinned by reference" and pinned instead by
  * FIPS-197 appendix C (AES-128, AES-256 example vectors),
  * RFC 8452 §A POLYVAL example and appendix C AEAD vectors (AES-128 and
    AES-256, with and without AAD, and the two counter-wrap vectors of C.3),
  * the system OpenSSL 3.0 libcrypto, an independent implementation: AES-128/
    256 blocks (ECB) on random keys, and POLYVAL through its GHASH relation
    (RFC 8452 appendix A) against AES-256-GCM tags over random AAD;
plus round trips, tamper rejection and the batch sealer vs the one-blob call.
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

from oracle import oracle as O

h = bytes.fromhex
K256 = h("01") + bytes(31)
K128 = h("01") + bytes(15)
N3 = h("030000000000000000000000")

# (key, nonce, aad, plaintext, ciphertext || tag)
RFC8452 = [
    (K128, N3, "", "", "dc20e2d83f25705bb49e439eca56de25"),
    (K128, N3, "", "0100000000000000", "b5d839330ac7b786578782fff6013b815b287c22493a364c"),
    (K128, N3, "01", "0200000000000000", "1e6daba35669f4273b0a1a2560969cdf790d99759abd1508"),
    (K256, N3, "", "", "07f5f4169bbf55a8400cd47ea6fd400f"),
    (K256, N3, "", "0100000000000000", "c2ef328e5c71c83b843122130f7364b761e0b97427e3df28"),
    (K256, N3, "", "010000000000000000000000", "9aab2aeb3faa0a34aea8e2b18ca50da9ae6559e48fd10f6e5c9ca17e"),
    (K256, N3, "", "01000000000000000000000000000000",
     "85a01b63025ba19b7fd3ddfc033b3e76c9eac6fa700942702e90862383c6c366"),
    (K256, N3, "01", "0200000000000000", "1de22967237a813291213f267e3b452f02d01ae33e4ec854"),
    (K256, N3, "01", "020000000000000000000000", "163d6f9cc1b346cd453a2e4cc1a4a19ae800941ccdc57cc8413c277f"),
    # C.3 counter wrap: the tag's first word is 0xffffffff, the le32 counter wraps
    (bytes(32), bytes(12), "", "000000000000000000000000000000004db923dc793ee6497c76dcc03a98e108",
     "f3f80f2cf0cb2dd9c5984fcda908456cc537703b5ba70324a6793a7bf218d3eaffffffff000000000000000000000000"),
    (bytes(32), bytes(12), "", "eb3640277c7ffd1303c7a542d02d3e4c0000000000000000",
     "18ce4f0b8cb4d0cac65fea8f79257b20888e53e72299e56dffffffff000000000000000000000000"),
]


def test_fips197_aes():
    pt = h("00112233445566778899aabbccddeeff")
    assert O.aes_encrypt_block(bytes(range(16)), pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert O.aes_encrypt_block(bytes(range(32)), pt).hex() == "8ea2b7ca516745bfeafc49904b496089"
    sb = O.aes_sbox()
    assert sb[0] == 0x63 and sb[0x53] == 0xED and sb[0xFF] == 0x16 and len(set(sb)) == 256


def test_rfc8452_polyval_example():
    H = h("25629347589242761d31f826ba4b757b")
    X = h("4f4f95668c83dfb6401762bb2d01a262") + h("d1a24ddd2721d006bbe45f20d3c9f362")
    assert O.polyval(H, X).hex() == "f7a3b47b846119fae5b7866cf5e5b77e"


def test_rfc8452_key_derivation():
    auth, enc = O.siv_derive(K256, N3)
    assert auth.hex() == "b5d3c529dfafac43136d2d11be284d7f"
    assert enc.hex() == "b914f4742be9e1d7a2f84addbf96dec3456e3c6c05ecc157cdbf0700fedad222"


@pytest.mark.parametrize("key,nonce,aad,pt,ct", RFC8452)
def test_rfc8452_vectors(key, nonce, aad, pt, ct):
    assert O.siv_encrypt(key, nonce, h(pt), aad=h(aad)).hex() == ct
    assert O.siv_decrypt(key, nonce, h(ct), aad=h(aad)) == h(pt)


# --------------------------------------------------------------- OpenSSL --
def _crypto():
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("libcrypto not present")
    L = ctypes.CDLL(name)
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    L.EVP_CIPHER_CTX_new.restype = vp
    L.EVP_CIPHER_CTX_free.argtypes = [vp]
    for c in ("EVP_aes_128_ecb", "EVP_aes_256_ecb", "EVP_aes_256_gcm"):
        getattr(L, c).restype = vp
    L.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, vp, vp]
    L.EVP_EncryptUpdate.argtypes = [vp, vp, ip, vp, ctypes.c_int]
    L.EVP_EncryptFinal_ex.argtypes = [vp, vp, ip]
    L.EVP_CIPHER_CTX_set_padding.argtypes = [vp, ctypes.c_int]
    L.EVP_CIPHER_CTX_ctrl.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    return L


def _ossl_ecb(L, key, data):
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        cipher = L.EVP_aes_256_ecb() if len(key) == 32 else L.EVP_aes_128_ecb()
        assert L.EVP_EncryptInit_ex(ctx, cipher, None, key, None) == 1
        L.EVP_CIPHER_CTX_set_padding(ctx, 0)
        out = ctypes.create_string_buffer(len(data) + 32)
        n = ctypes.c_int()
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), data, len(data)) == 1
        return out.raw[: n.value]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def _ossl_gcm_tag(L, key, iv, aad):
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_aes_256_gcm(), None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, 0x9, len(iv), None) == 1  # EVP_CTRL_GCM_SET_IVLEN
        assert L.EVP_EncryptInit_ex(ctx, None, None, key, iv) == 1
        n = ctypes.c_int()
        assert L.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
        buf = ctypes.create_string_buffer(32)
        assert L.EVP_EncryptFinal_ex(ctx, buf, ctypes.byref(n)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, tag) == 1  # EVP_CTRL_GCM_GET_TAG
        return tag.raw
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


@pytest.mark.parametrize("key_bytes", [16, 32])
def test_aes_blocks_vs_openssl(key_bytes):
    L = _crypto()
    rng = np.random.default_rng(8452 + key_bytes)
    for _ in range(64):
        key = rng.integers(0, 256, key_bytes, dtype=np.uint8).tobytes()
        blocks = rng.integers(0, 256, 16 * 8, dtype=np.uint8).tobytes()
        mine = b"".join(O.aes_encrypt_block(key, blocks[i:i + 16]) for i in range(0, len(blocks), 16))
        assert mine == _ossl_ecb(L, key, blocks)


def _mulx_polyval(x: bytes) -> bytes:
    v = int.from_bytes(x, "little") << 1
    if v >> 128:
        v ^= (1 << 128) | (1 << 127) | (1 << 126) | (1 << 121) | 1
    return v.to_bytes(16, "little")


def test_polyval_vs_openssl_ghash():
    """GHASH(H, X..) = ByteReverse(POLYVAL(mulX_POLYVAL(ByteReverse(H)), ByteReverse(X)..))
    (RFC 8452 appendix A); an AES-256-GCM tag over AAD only is E_K(J0) xor
    GHASH_{E_K(0)}(AAD blocks, be64(bitlen AAD) || be64(0))."""
    L = _crypto()
    rng = np.random.default_rng(1652)
    for nblk in (1, 2, 7, 64):
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        aad = rng.integers(0, 256, 16 * nblk, dtype=np.uint8).tobytes()
        hk = _ossl_ecb(L, key, bytes(16))
        ej0 = _ossl_ecb(L, key, iv + b"\x00\x00\x00\x01")
        ghash = bytes(a ^ b for a, b in zip(_ossl_gcm_tag(L, key, iv, aad), ej0))
        xs = [aad[i:i + 16] for i in range(0, len(aad), 16)] + [(8 * len(aad)).to_bytes(8, "big") + bytes(8)]
        pv = O.polyval(_mulx_polyval(hk[::-1]), b"".join(x[::-1] for x in xs))
        assert pv[::-1] == ghash


# ------------------------------------------------------------ properties --
def test_round_trip_and_tamper():
    rng = np.random.default_rng(3)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    for n in (0, 1, 15, 16, 17, 31, 32, 33, 255, 4096, 100_003):
        nonce = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        pt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        blob = O.encrypt_with_key(key, nonce, pt)
        assert len(blob) == n + O.SEAL_OVERHEAD and blob[:12] == nonce
        assert O.decrypt_with_key(key, blob) == pt
        bad = bytearray(blob)
        bad[rng.integers(0, len(bad))] ^= 1 << int(rng.integers(0, 8))
        assert O.decrypt_with_key(key, bytes(bad)) is None
    assert O.decrypt_with_key(key, bytes(27)) is None  # shorter than nonce + tag


@pytest.mark.parametrize("threads", [1, 4])
def test_seal_blobs_matches_single(threads):
    rng = np.random.default_rng(11 + threads)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    lens = rng.integers(0, 70_000, 40)
    lens[::7] = 0
    lens[3] = 16
    data = rng.integers(0, 256, int(lens.sum()) + 5, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    nonces = rng.integers(0, 256, (40, 12), dtype=np.uint8)
    out, oo = O.seal_blobs(key, data, offs, lens, nonces, threads=threads)
    for i in range(40):
        want = O.encrypt_with_key(key, nonces[i], data[offs[i]:offs[i] + lens[i]])
        assert out[oo[i]:oo[i] + len(want)].tobytes() == want
