"""ctypes binding of libmcdc.so (the C ABI in include/mcdc.h).

The library is built in-tree by ``mapache_amd.build`` (hipcc, gfx950).  There
is no CPU fallback: if the shared object or a HIP device is missing, every
entry point raises.
"""
from __future__ import annotations

import ctypes
import functools
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MCDC_LIBRARY overrides the in-tree build (A/B comparisons of kernel variants)
LIB_PATH = os.environ.get("MCDC_LIBRARY") or os.path.join(HERE, "libmcdc.so")

MCDC_OK = 0
MCDC_E_INVALID = -1
MCDC_E_PARAMS = -2
MCDC_E_CAPACITY = -3
MCDC_E_DEVICE = -4
MCDC_E_NOMEM = -5
MCDC_E_TOOBIG = -6
MCDC_E_INTERNAL = -7
MCDC_E_AUTH = -8
NONCE_BYTES, TAG_BYTES, SEAL_OVERHEAD = 12, 16, 28

# every symbol include/mcdc.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "mcdc_params_check", "mcdc_ctx_create", "mcdc_ctx_destroy", "mcdc_chunk_device",
    "mcdc_chunk_host", "mcdc_chunk_batch", "mcdc_chunk_batch_device", "mcdc_ctx_timing",
    "mcdc_last_error", "mcdc_device_alloc", "mcdc_device_free", "mcdc_host_alloc",
    "mcdc_host_free", "mcdc_memcpy_h2d", "mcdc_memcpy_d2h", "mcdc_fill_random_device", "mcdc_digest",
    "mcdc_abi_version", "mcdc_chunk_ids_device", "mcdc_batcher_create", "mcdc_batcher_destroy",
    "mcdc_batcher_chunk", "mcdc_batcher_stats", "mcdc_seal_device", "mcdc_open_device", "mcdc_seal_chunks_device",
    "mcdc_index_create", "mcdc_index_destroy", "mcdc_index_size", "mcdc_index_add",
    "mcdc_encode_blobs", "mcdc_decode_blobs", "mcdc_pack_blobs", "mcdc_zstd_frames_device", "mcdc_save_files",
    "mcdc_zstd_compress_device", "mcdc_ctx_synchronize", "mcdc_ctx_set_option", "mcdc_zstd_compress_scratch",
)


class McdcStore(ctypes.Structure):
    """mcdc_store (include/mcdc.h): SecureStorage key (None = build()), the
    repository's max pack size and the caller's randomness."""
    _fields_ = [("key", ctypes.c_void_p), ("max_pack_size", ctypes.c_uint64), ("nonces", ctypes.c_void_p),
                ("nnonces", ctypes.c_size_t), ("header_nonces", ctypes.c_void_p), ("nheader_nonces", ctypes.c_size_t),
                ("padding", ctypes.c_void_p), ("npadding", ctypes.c_size_t), ("gpu_compress", ctypes.c_uint32),
                ("gate_bytes", ctypes.c_uint64)]


PACK_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("nblobs", "<u8"), ("meta_size", "<u8"),
                       ("id", "u1", (32,))])


class McdcParams(ctypes.Structure):
    _fields_ = [("min_size", ctypes.c_uint32), ("avg_size", ctypes.c_uint32),
                ("max_size", ctypes.c_uint32), ("level", ctypes.c_uint32)]


class McdcChunk(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("length", ctypes.c_uint64), ("hash", ctypes.c_uint64)]


class McdcTiming(ctypes.Structure):
    _fields_ = [("scan_ms", ctypes.c_double), ("resolve_ms", ctypes.c_double),
                ("device_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("bytes", ctypes.c_uint64), ("chunks", ctypes.c_uint64),
                ("scan_launches", ctypes.c_uint64), ("fallback_files", ctypes.c_uint64),
                ("ids_ms", ctypes.c_double), ("aead_ms", ctypes.c_double),
                ("lane_walk", ctypes.c_uint64), ("handed_back", ctypes.c_uint64),
                ("host_pre_ms", ctypes.c_double), ("host_post_ms", ctypes.c_double)]


class McdcBatcherStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("files", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("max_batch_files", ctypes.c_uint64)]


CHUNK_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("hash", "<u8")])

_lib = None


class McdcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mcdc error {code}: {msg}")
        self.code = code


def load():
    """Load libmcdc.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python -m mapache_amd.build` (hipcc gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u64, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int
    P = ctypes.POINTER
    L.mcdc_params_check.argtypes = [P(McdcParams), P(u64), P(u64)]
    L.mcdc_ctx_create.argtypes = [i32, sz, P(vp)]
    L.mcdc_ctx_destroy.argtypes = [vp]
    L.mcdc_ctx_destroy.restype = None
    L.mcdc_chunk_device.argtypes = [vp, P(McdcParams), vp, sz, vp, sz, P(sz)]
    L.mcdc_chunk_host.argtypes = [vp, P(McdcParams), vp, sz, vp, sz, P(sz)]
    L.mcdc_chunk_batch.argtypes = [vp, P(McdcParams), vp, vp, sz, vp, sz, vp, P(sz)]
    L.mcdc_chunk_batch_device.argtypes = [vp, P(McdcParams), vp, vp, vp, sz, vp, sz, vp, P(sz)]
    L.mcdc_ctx_timing.argtypes = [vp, P(McdcTiming)]
    L.mcdc_last_error.argtypes = []
    L.mcdc_last_error.restype = ctypes.c_char_p
    L.mcdc_device_alloc.argtypes = [vp, sz, P(vp)]
    L.mcdc_device_free.argtypes = [vp, vp]
    L.mcdc_ctx_synchronize.argtypes = [vp]
    L.mcdc_ctx_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_longlong]
    L.mcdc_zstd_compress_scratch.argtypes = [vp, vp, sz, P(sz)]
    L.mcdc_host_alloc.argtypes = [vp, sz, P(vp)]
    L.mcdc_host_free.argtypes = [vp, vp]
    L.mcdc_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.mcdc_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.mcdc_fill_random_device.argtypes = [vp, vp, u64, sz, u64]
    L.mcdc_digest.argtypes = [vp, sz]
    L.mcdc_digest.restype = u64
    L.mcdc_abi_version.argtypes = []
    L.mcdc_chunk_ids_device.argtypes = [vp, vp, sz, vp, sz, vp]
    L.mcdc_batcher_create.argtypes = [i32, P(McdcParams), sz, sz, ctypes.c_uint32, P(vp)]
    L.mcdc_batcher_destroy.argtypes = [vp]
    L.mcdc_batcher_destroy.restype = None
    L.mcdc_batcher_chunk.argtypes = [vp, vp, sz, vp, sz, P(sz)]
    L.mcdc_batcher_stats.argtypes = [vp, P(McdcBatcherStats)]
    L.mcdc_seal_device.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, sz, vp]
    L.mcdc_open_device.argtypes = [vp, vp, vp, sz, vp, sz, vp, sz, vp, vp]
    L.mcdc_seal_chunks_device.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, sz, vp]
    L.mcdc_index_create.argtypes = [vp, P(vp)]
    L.mcdc_index_destroy.argtypes = [vp]
    L.mcdc_index_destroy.restype = None
    L.mcdc_index_size.argtypes = [vp]
    L.mcdc_index_size.restype = sz
    L.mcdc_index_add.argtypes = [vp, vp, vp, sz, vp, vp, vp, P(sz)]
    L.mcdc_encode_blobs.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, sz, vp]
    L.mcdc_decode_blobs.argtypes = [vp, vp, vp, sz, vp, sz, vp, sz, vp, vp]
    L.mcdc_zstd_frames_device.argtypes = [vp, vp, sz, vp, sz, vp, sz, P(sz), vp]
    L.mcdc_pack_blobs.argtypes = [vp, vp, vp, sz, vp, vp, vp, sz, u64, vp, sz, vp, sz, vp, sz, P(sz), vp, sz,
                                  P(sz)]
    # (an A/B library of older sources, MCDC_LIBRARY, may predate the save path)
    if hasattr(L, "mcdc_save_files"):
        L.mcdc_save_files.argtypes = [vp, P(McdcParams), vp, P(McdcStore), vp, sz, vp, sz, vp, vp, vp, sz, P(sz), vp,
                                      sz, P(sz), vp, sz, P(sz)]
    if hasattr(L, "mcdc_zstd_compress_device"):
        L.mcdc_zstd_compress_device.argtypes = [vp, vp, sz, vp, sz, vp, sz, P(sz), vp]
    for name in EXPORTS:  # fail loudly if the build is stale (the in-tree build)
        if not os.environ.get("MCDC_LIBRARY") or name not in ("mcdc_save_files", "mcdc_zstd_compress_device"):
            getattr(L, name)
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != MCDC_OK:
        raise McdcError(rc, load().mcdc_last_error().decode(errors="replace"))


def params(min_size: int, avg_size: int, max_size: int, level: int = 1) -> McdcParams:
    return McdcParams(min_size, avg_size, max_size, level)


def _locked(fn):
    """Serialise a Context method: mcdc.h forbids two threads in one context at
    once, and ctypes releases the GIL during every C call."""
    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        with self._lock:
            if not self._h:
                raise McdcError(MCDC_E_INVALID, "context is closed")
            return fn(self, *args, **kwargs)
    return wrapper


class Context:
    """One mcdc_ctx: a HIP device, a stream and its workspace.

    Thread-safe: every call holds the context's lock (the C context must not be
    entered by two threads at once), and close() waits for a call in flight.
    For concurrency, give each worker thread its own Context (as the Archiver
    adapter in INTEGRATION.md does) — calls on one context serialise."""

    def __init__(self, device: int = 0, max_bytes: int = 1 << 30):
        L = load()
        self._lock = threading.RLock()
        self._h = None
        h = ctypes.c_void_p()
        check(L.mcdc_ctx_create(device, max_bytes, ctypes.byref(h)))
        self._h = h
        self.device = device
        self.max_bytes = max_bytes
        self._out = None      # reusable pinned output buffer (np view) and its pointer
        self._out_ptr = None
        self._pinned = []     # pinned_bytes allocations, freed at close()

    def close(self):
        lock = getattr(self, "_lock", None)
        if lock is None:
            return
        with lock:
            if self._h:
                if self._out_ptr:
                    load().mcdc_host_free(self._h, ctypes.c_void_p(self._out_ptr))
                    self._out, self._out_ptr = None, None
                for ptr in self._pinned:
                    load().mcdc_host_free(self._h, ctypes.c_void_p(ptr))
                self._pinned = []
                load().mcdc_ctx_destroy(self._h)
                self._h = None

    @_locked
    def pinned_bytes(self, n: int) -> np.ndarray:
        """A pinned-host uint8 array of n bytes, valid until close()."""
        ptr = self.host_alloc(max(int(n), 1))
        self._pinned.append(ptr)
        return np.frombuffer((ctypes.c_uint8 * max(int(n), 1)).from_address(ptr), dtype=np.uint8)[:int(n)]

    @_locked
    def pinned_out(self, cap: int) -> np.ndarray:
        """A reusable pinned-host chunk array of at least `cap` entries (grown on demand).
        Results written into it are only valid until the next call that reuses it."""
        if self._out is None or self._out.size < cap:
            if self._out_ptr:
                check(load().mcdc_host_free(self._h, ctypes.c_void_p(self._out_ptr)))
            ptr = self.host_alloc(cap * CHUNK_DTYPE.itemsize)
            buf = (ctypes.c_uint8 * (cap * CHUNK_DTYPE.itemsize)).from_address(ptr)
            self._out = np.frombuffer(buf, dtype=CHUNK_DTYPE)
            self._out_ptr = ptr
        return self._out

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- chunking --
    @staticmethod
    def _bound(n: int, p: McdcParams) -> int:
        return n // max(p.min_size - 1, 1) + 2

    @_locked
    def _run(self, fn, p: McdcParams, *args, cap: int, out: np.ndarray | None = None):
        if out is None:
            out = np.empty(max(cap, 1), dtype=CHUNK_DTYPE)
            copy = True
        else:
            copy = False
            cap = min(cap, out.size)
        n_out = ctypes.c_size_t()
        rc = fn(self._h, ctypes.byref(p), *args, out.ctypes.data, cap, ctypes.byref(n_out))
        check(rc)
        return out[: n_out.value].copy() if copy else out[: n_out.value]

    def chunk_device(self, p: McdcParams, d_ptr: int, n: int, out: np.ndarray | None = None) -> np.ndarray:
        """Chunks of a device-resident buffer.  With `out` (e.g. ``pinned_out``) the
        result is a view into it (no allocation, pinned D2H)."""
        return self._run(load().mcdc_chunk_device, p, ctypes.c_void_p(d_ptr), n, cap=self._bound(n, p),
                         out=out)

    def chunk_host(self, p: McdcParams, data) -> np.ndarray:
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                                 else data.view(np.uint8).reshape(-1))
        return self._run(load().mcdc_chunk_host, p, ctypes.c_void_p(a.ctypes.data), a.size,
                         cap=self._bound(a.size, p))

    @_locked
    def chunk_batch(self, p: McdcParams, bufs):
        arrs = [np.ascontiguousarray(np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray)
                                     else b.view(np.uint8).reshape(-1)) for b in bufs]
        n = len(arrs)
        ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        lens = (ctypes.c_size_t * max(n, 1))(*[a.size for a in arrs])
        counts = np.empty(max(n, 1), dtype=np.uint64)  # (every entry written by the call)
        cap = sum(self._bound(a.size, p) for a in arrs) + 1
        out = np.zeros(cap, dtype=CHUNK_DTYPE)
        n_out = ctypes.c_size_t()
        check(load().mcdc_chunk_batch(self._h, ctypes.byref(p), ptrs, lens, n, out.ctypes.data, cap,
                                      counts.ctypes.data, ctypes.byref(n_out)))
        return out[: n_out.value].copy(), counts[:n].view(np.int64)  # (counts < 2^63: a view, no copy)

    @_locked
    def chunk_batch_device(self, p: McdcParams, d_arena: int, offsets, lens):
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        ls = np.ascontiguousarray(lens, dtype=np.uint64)
        n = offs.size
        counts = np.empty(max(n, 1), dtype=np.uint64)  # (every entry written by the call)
        cap = int(sum(self._bound(int(x), p) for x in ls)) + 1
        out = np.zeros(cap, dtype=CHUNK_DTYPE)
        n_out = ctypes.c_size_t()
        check(load().mcdc_chunk_batch_device(self._h, ctypes.byref(p), ctypes.c_void_p(d_arena),
                                             offs.ctypes.data, ls.ctypes.data, n, out.ctypes.data, cap,
                                             counts.ctypes.data, ctypes.byref(n_out)))
        return out[: n_out.value].copy(), counts[:n].view(np.int64)  # (counts < 2^63: a view, no copy)

    @_locked
    def chunk_device_to_device(self, p: McdcParams, d_ptr: int, n: int, d_out: int, cap: int) -> int:
        """Chunk a device-resident buffer into a device-resident boundary list
        (`cap` mcdc_chunk records at device pointer `d_out`); returns the count."""
        n_out = ctypes.c_size_t()
        check(load().mcdc_chunk_device(self._h, ctypes.byref(p), ctypes.c_void_p(d_ptr), n,
                                       ctypes.c_void_p(d_out), cap, ctypes.byref(n_out)))
        return n_out.value

    @_locked
    def chunk_batch_device_to_device(self, p: McdcParams, d_arena: int, offsets, lens, d_out: int, cap: int):
        """Many device-resident files -> device-resident boundary list; returns
        (total chunks, per-file counts)."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        ls = np.ascontiguousarray(lens, dtype=np.uint64)
        n = offs.size
        counts = np.empty(max(n, 1), dtype=np.uint64)  # (every entry written by the call)
        n_out = ctypes.c_size_t()
        check(load().mcdc_chunk_batch_device(self._h, ctypes.byref(p), ctypes.c_void_p(d_arena),
                                             offs.ctypes.data, ls.ctypes.data, n, ctypes.c_void_p(d_out), cap,
                                             counts.ctypes.data, ctypes.byref(n_out)))
        return n_out.value, counts[:n].view(np.int64)  # (counts < 2^63: a view, no copy)

    @_locked
    def chunk_ids(self, d_data: int, n: int, chunks, ids=None) -> np.ndarray:
        """BLAKE3 chunk IDs (ID::from_content) of a boundary list over the device
        buffer d_data[0, n).  `chunks`: a CHUNK_DTYPE array (host) or an int
        device pointer with `count` given as (ptr, count).  Returns (count, 32) uint8
        unless `ids` (an int device pointer) is given, then returns None."""
        if isinstance(chunks, tuple):
            cptr, count = chunks
        else:
            arr = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
            cptr, count = arr.ctypes.data, arr.size
            keep = arr  # noqa: F841  (alive across the call)
        if ids is not None:
            check(load().mcdc_chunk_ids_device(self._h, ctypes.c_void_p(d_data), n, ctypes.c_void_p(cptr), count,
                                               ctypes.c_void_p(ids)))
            return None
        out = np.zeros((max(count, 1), 32), dtype=np.uint8)
        check(load().mcdc_chunk_ids_device(self._h, ctypes.c_void_p(d_data), n, ctypes.c_void_p(cptr), count,
                                           out.ctypes.data))
        return out[:count]

    # ------------------------------------------- SecureStorage encode/decode --
    @_locked
    def encode_blobs(self, key, data, offsets, lengths, nonces):
        """SecureStorage::encode of every blob data[offsets[i], +lengths[i]) (host
        bytes): zstd on host threads, AES-256-GCM-SIV on the GPU
        (mcdc_encode_blobs).  key=None: SecureStorage::build() (compress only,
        nonces unused).  Returns (packed bytes, nblobs + 1 offsets)."""
        a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        ext = self._extents(offsets, lengths)
        nz = np.ascontiguousarray(np.zeros(0, np.uint8) if nonces is None else nonces, dtype=np.uint8).reshape(-1)
        if key is not None and nz.size != NONCE_BYTES * len(ext):
            raise ValueError("need 12 nonce bytes per blob")
        oo = np.zeros(len(ext) + 1, dtype=np.uint64)
        cap = int(a.size + (a.size >> 7) + 64 * len(ext) + 64)  # zstd's bound + 28 per blob
        out = np.empty(max(cap, 1), dtype=np.uint8)
        rc = load().mcdc_encode_blobs(self._h, self._key(key), a.ctypes.data, a.size, ext.ctypes.data, len(ext),
                                      nz.ctypes.data, out.ctypes.data, cap, oo.ctypes.data)
        if rc == MCDC_E_CAPACITY:
            out = np.empty(int(oo[-1]), dtype=np.uint8)
            rc = load().mcdc_encode_blobs(self._h, self._key(key), a.ctypes.data, a.size, ext.ctypes.data,
                                          len(ext), nz.ctypes.data, out.ctypes.data, out.size, oo.ctypes.data)
        check(rc)
        return out[:int(oo[-1])], oo

    @_locked
    def decode_blobs(self, key, data, offsets, lengths, cap: int):
        """SecureStorage::decode of every sealed extent (mcdc_decode_blobs).
        Returns (packed plaintexts, nblobs + 1 offsets, status); status -1 / -2
        marks blobs that failed (no exception for those)."""
        a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        ext = self._extents(offsets, lengths)
        oo = np.zeros(len(ext) + 1, dtype=np.uint64)
        st = np.zeros(max(len(ext), 1), dtype=np.int32)
        out = np.empty(max(cap, 1), dtype=np.uint8)
        rc = load().mcdc_decode_blobs(self._h, self._key(key), a.ctypes.data, a.size, ext.ctypes.data, len(ext),
                                      out.ctypes.data, cap, oo.ctypes.data, st.ctypes.data)
        if rc != MCDC_E_AUTH:
            check(rc)
        return out[:int(oo[-1])], oo, st[:len(ext)]

    @_locked
    def zstd_frames(self, d_data: int, n: int, chunks, d_out: int, out_cap: int, frames_out=None):
        """zstd raw-block frames of every chunk (mcdc_zstd_frames_device).  chunks:
        CHUNK_DTYPE array or (device pointer, count).  Returns (frames as an
        (count, 2) uint64 array of (offset, length), output span), or writes the
        extents to the device pointer frames_out and returns (None, span)."""
        if isinstance(chunks, tuple):
            cptr, count = chunks
        else:
            arr = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
            cptr, count = arr.ctypes.data, arr.size
            keep = arr  # noqa: F841
        span = ctypes.c_size_t()
        fr = None if frames_out is not None else np.zeros((max(count, 1), 2), dtype=np.uint64)
        fptr = frames_out if frames_out is not None else fr.ctypes.data
        check(load().mcdc_zstd_frames_device(self._h, ctypes.c_void_p(d_data), n, ctypes.c_void_p(cptr), count,
                                             ctypes.c_void_p(d_out), out_cap, ctypes.byref(span),
                                             ctypes.c_void_p(fptr)))
        return (None if fr is None else fr[:count]), span.value

    @_locked
    def zstd_compress(self, d_data: int, n: int, chunks, d_out: int, out_cap: int, frames_out=None):
        """SecureStorage::compress of every chunk on the GPU
        (mcdc_zstd_compress_device).  chunks: CHUNK_DTYPE array or (device
        pointer, count).  Returns (frames as (count, 2) uint64 (offset, length)
        or None with frames_out, bytes written).  out_cap too small raises
        McdcError(MCDC_E_CAPACITY); zstd_compress_bound gives the capacity."""
        if isinstance(chunks, tuple):
            cptr, count = chunks
        else:
            arr = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
            cptr, count = arr.ctypes.data, arr.size
            keep = arr  # noqa: F841
        span = ctypes.c_size_t()
        fr = None if frames_out is not None else np.zeros((max(count, 1), 2), dtype=np.uint64)
        fptr = frames_out if frames_out is not None else fr.ctypes.data
        check(load().mcdc_zstd_compress_device(self._h, ctypes.c_void_p(d_data), n, ctypes.c_void_p(cptr), count,
                                               ctypes.c_void_p(d_out), out_cap, ctypes.byref(span),
                                               ctypes.c_void_p(fptr)))
        return (None if fr is None else fr[:count]), span.value

    @staticmethod
    def zstd_compress_bound(lengths) -> int:
        """Output capacity that always suffices for zstd_compress: the raw frames
        of 32 KiB blocks (length + 6 + 3 per block)."""
        ln = np.asarray(lengths, dtype=np.uint64)
        nb = np.maximum((ln + np.uint64(32767)) // np.uint64(32768), np.uint64(1))
        return int((ln + np.uint64(6) + np.uint64(3) * nb).sum())

    @_locked
    def pack_blobs(self, key, data, offsets, lengths, ids, types, max_pack_size: int, header_nonces, padding):
        """Packer::add_blob + flush over encoded host blobs (mcdc_pack_blobs).
        Returns (packed bytes, PACK_DTYPE records)."""
        a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        ext = self._extents(offsets, lengths)
        iv = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1)
        ty = np.ascontiguousarray(types, dtype=np.uint8).reshape(-1)
        hn = np.ascontiguousarray(np.zeros(0, np.uint8) if header_nonces is None else header_nonces,
                                  dtype=np.uint8).reshape(-1)
        pd = np.ascontiguousarray(padding, dtype=np.uint8).reshape(-1)
        nb, np_, cap = ctypes.c_size_t(), ctypes.c_size_t(), 0
        packs = np.zeros(1, dtype=PACK_DTYPE)
        out = np.empty(1, dtype=np.uint8)
        for _ in range(2):  # size query, then the call
            rc = load().mcdc_pack_blobs(self._h, self._key(key), a.ctypes.data, a.size, ext.ctypes.data,
                                        iv.ctypes.data, ty.ctypes.data, len(ext), max_pack_size, hn.ctypes.data,
                                        hn.size // NONCE_BYTES, pd.ctypes.data, pd.size // 36, out.ctypes.data, cap,
                                        ctypes.byref(nb), packs.ctypes.data, packs.size, ctypes.byref(np_))
            if rc != MCDC_E_CAPACITY:
                break
            cap = nb.value
            out = np.empty(max(cap, 1), dtype=np.uint8)
            packs = np.zeros(max(np_.value, 1), dtype=PACK_DTYPE)
        check(rc)
        return out[:nb.value], packs[:np_.value]

    # --------------------------------------------------------- save path --
    @_locked
    def save_files(self, p: "McdcParams", index: "Index", data, offsets, lengths, key=None, nonces=None,
                   header_nonces=None, padding=None, max_pack_size: int = 16 << 20, n: int | None = None,
                   gpu_compress: bool = False, gate_bytes: int = 0, out_buf: np.ndarray | None = None,
                   split: bool = True):
        """The Archiver's save path for a run of files (mcdc_save_files): data is
        a host array (or a device pointer with n bytes); file f = data[offsets[f],
        + lengths[f]); gpu_compress: compress with the GPU zstd kernels in HBM
        (decode-equal blobs) instead of level 3 on host threads; gate_bytes:
        save_file's size gate (0 = MIN_CHUNK_SIZE, 512 KiB); out_buf: a uint8
        host array (e.g. pinned_bytes) the packs are written into when it is
        large enough (the returned packed bytes are then a view of it).  Returns
        (ids_per_file: list of (k, 32) uint8 arrays,
        is_new per blob, packed bytes, PACK_DTYPE records); split=False returns
        the IDs as one (blobs, 32) array and file_blobs (file f's IDs are rows
        file_blobs[f] .. file_blobs[f + 1]) instead of the per-file list
        (80 000 files: ~40 ms of Python slicing, more than the call itself):
        (ids, file_blobs, is_new, packed bytes, PACK_DTYPE records)."""
        if isinstance(data, int):
            dptr, nbytes, keep = data, int(n), None
        else:
            keep = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
            dptr, nbytes = keep.ctypes.data, keep.size
        ext = self._extents(offsets, lengths)
        nf = len(ext)
        k = self._key(key)
        arrs = [np.ascontiguousarray(np.zeros(0, np.uint8) if x is None else x, dtype=np.uint8).reshape(-1)
                for x in (nonces, header_nonces, padding)]
        kbuf = ctypes.create_string_buffer(k, len(k)) if k else None
        st = McdcStore(ctypes.addressof(kbuf) if k else None, max_pack_size,
                       arrs[0].ctypes.data, arrs[0].size // NONCE_BYTES, arrs[1].ctypes.data,
                       arrs[1].size // NONCE_BYTES, arrs[2].ctypes.data, arrs[2].size // 36, int(bool(gpu_compress)),
                       int(gate_bytes))
        fb = np.zeros(nf + 1, np.uint64)
        bcap = int((ext[:, 1] // np.uint64(max(p.min_size - 1, 1)) + np.uint64(2)).sum()) if nf else 1
        ids = np.zeros((max(bcap, 1), 32), np.uint8)
        nw = np.zeros(max(bcap, 1), np.uint8)
        ocap = int(ext[:, 1].sum() * 1.01) + 4096 * nf + (1 << 16) if nf else 1
        out = out_buf if out_buf is not None else np.empty(max(ocap, 1), np.uint8)
        packs = np.zeros(max(1, ocap // max(max_pack_size, 1) + 2), PACK_DTYPE)
        nb, pb, np_ = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        for _ in range(3):
            rc = load().mcdc_save_files(self._h, ctypes.byref(p), ctypes.c_void_p(index._h), ctypes.byref(st),
                                        ctypes.c_void_p(dptr), nbytes, ext.ctypes.data, nf, fb.ctypes.data,
                                        ids.ctypes.data, nw.ctypes.data, len(ids), ctypes.byref(nb),
                                        out.ctypes.data, out.size, ctypes.byref(pb), packs.ctypes.data, packs.size,
                                        ctypes.byref(np_))
            if rc != MCDC_E_CAPACITY:
                break
            if nb.value > len(ids):
                ids = np.zeros((nb.value, 32), np.uint8)
                nw = np.zeros(nb.value, np.uint8)
            if pb.value > out.size:
                out = np.empty(pb.value, np.uint8)
            if np_.value > packs.size:
                packs = np.zeros(np_.value, PACK_DTYPE)
        check(rc)
        del keep, kbuf
        if not split:
            return ids[:nb.value], fb, nw[:nb.value].astype(bool), out[:pb.value], packs[:np_.value]
        per_file = [ids[int(fb[f]):int(fb[f + 1])].copy() for f in range(nf)]
        return per_file, nw[:nb.value].astype(bool), out[:pb.value], packs[:np_.value]

    # ------------------------------------------------------- dedup index --
    @_locked
    def index_create(self) -> "Index":
        """A device-resident dedup index on this context's device (mcdc_index_create)."""
        h = ctypes.c_void_p()
        check(load().mcdc_index_create(self._h, ctypes.byref(h)))
        return Index(self, h.value)

    # ----------------------------------------------------------- sealing --
    @staticmethod
    def _extents(offsets, lengths) -> np.ndarray:
        ext = np.empty((len(offsets), 2), dtype=np.uint64)
        ext[:, 0] = np.asarray(offsets, dtype=np.uint64)
        ext[:, 1] = np.asarray(lengths, dtype=np.uint64)
        return ext

    @staticmethod
    def _key(key):
        """32 key bytes, or None (SecureStorage::build(): no encryption)."""
        if key is None:
            return None
        key = bytes(key)
        if len(key) != 32:
            raise ValueError("AES-256-GCM-SIV key must be 32 bytes")
        return key

    @_locked
    def seal_device_ext(self, key, d_in: int, n_in: int, d_ext: int, count: int, d_nonces: int, d_out: int,
                        out_cap: int, d_offsets: int) -> None:
        """mcdc_seal_device with every array in HBM: (offset, length) extents,
        nonces and the nblobs + 1 output offsets."""
        check(load().mcdc_seal_device(self._h, self._key(key), ctypes.c_void_p(d_in), n_in, ctypes.c_void_p(d_ext),
                                      count, ctypes.c_void_p(d_nonces), ctypes.c_void_p(d_out), out_cap,
                                      ctypes.c_void_p(d_offsets)))

    @_locked
    def seal(self, key, d_in: int, n_in: int, offsets, lengths, nonces, d_out: int, out_cap: int) -> np.ndarray:
        """SecureStorage::encrypt_with_key for every blob d_in[offsets[i], +lengths[i])
        (mcdc_seal_device): results nonce || ct || tag packed from d_out.  Returns the
        nblobs + 1 output offsets (last = total bytes)."""
        ext = self._extents(offsets, lengths)
        nz = np.ascontiguousarray(nonces, dtype=np.uint8).reshape(-1)
        if nz.size != NONCE_BYTES * len(ext):
            raise ValueError("need 12 nonce bytes per blob")
        oo = np.zeros(len(ext) + 1, dtype=np.uint64)
        check(load().mcdc_seal_device(self._h, self._key(key), ctypes.c_void_p(d_in), n_in, ext.ctypes.data,
                                      len(ext), nz.ctypes.data, ctypes.c_void_p(d_out), out_cap, oo.ctypes.data))
        return oo

    @_locked
    def seal_chunks(self, key, d_in: int, n_in: int, chunks, nonces, d_out: int, out_cap: int, offsets_out=None):
        """mcdc_seal_chunks_device: the blobs are the records of a boundary list --
        a CHUNK_DTYPE array (host) or (device pointer, count).  Returns the nblobs + 1
        output offsets, or writes them to the device pointer `offsets_out`."""
        if isinstance(chunks, tuple):
            cptr, count = chunks
        else:
            arr = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
            cptr, count = arr.ctypes.data, arr.size
            keep = arr  # noqa: F841  (alive across the call)
        nz = np.ascontiguousarray(nonces, dtype=np.uint8).reshape(-1) if not isinstance(nonces, int) else None
        nptr = nonces if nz is None else nz.ctypes.data
        oo = None if offsets_out is not None else np.zeros(count + 1, dtype=np.uint64)
        check(load().mcdc_seal_chunks_device(self._h, self._key(key), ctypes.c_void_p(d_in), n_in,
                                             ctypes.c_void_p(cptr), count, ctypes.c_void_p(nptr),
                                             ctypes.c_void_p(d_out), out_cap,
                                             ctypes.c_void_p(offsets_out if oo is None else oo.ctypes.data)))
        return oo

    @_locked
    def open(self, key, d_in: int, n_in: int, offsets, lengths, d_out: int, out_cap: int, raise_on_auth=True):
        """SecureStorage::decrypt_with_key for every sealed extent (mcdc_open_device):
        plaintexts packed from d_out.  Returns (out offsets, status per blob: 0 ok, -1 not);
        raises McdcError(MCDC_E_AUTH) when a blob fails and raise_on_auth."""
        ext = self._extents(offsets, lengths)
        oo = np.zeros(len(ext) + 1, dtype=np.uint64)
        stat = np.zeros(max(len(ext), 1), dtype=np.int32)
        rc = load().mcdc_open_device(self._h, self._key(key), ctypes.c_void_p(d_in), n_in, ext.ctypes.data, len(ext),
                                     ctypes.c_void_p(d_out), out_cap, oo.ctypes.data, stat.ctypes.data)
        if rc != MCDC_E_AUTH or raise_on_auth:
            check(rc)
        return oo, stat[: len(ext)]

    @_locked
    def d2h_bytes(self, d_src: int, nbytes: int) -> np.ndarray:
        out = np.empty(max(nbytes, 1), dtype=np.uint8)
        if nbytes:
            check(load().mcdc_memcpy_d2h(self._h, out.ctypes.data, ctypes.c_void_p(d_src), nbytes))
        return out[:nbytes]

    @_locked
    def d2h_chunks(self, d_out: int, count: int) -> np.ndarray:
        out = np.empty(max(count, 1), dtype=CHUNK_DTYPE)
        if count:
            check(load().mcdc_memcpy_d2h(self._h, out.ctypes.data, ctypes.c_void_p(d_out),
                                         count * CHUNK_DTYPE.itemsize))
        return out[:count]

    @_locked
    def synchronize(self) -> None:
        """Wait for all work of this context (mcdc_ctx_synchronize: its streams
        and the null stream, not other contexts')."""
        check(load().mcdc_ctx_synchronize(self._h))

    @_locked
    def zstd_compress_scratch(self, chunks) -> int:
        """Device scratch (bytes) mcdc_zstd_compress_device allocates for this
        chunk list (mcdc_zstd_compress_scratch)."""
        arr = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
        b = ctypes.c_size_t()
        check(load().mcdc_zstd_compress_scratch(self._h, arr.ctypes.data if arr.size else None, arr.size,
                                                ctypes.byref(b)))
        return b.value

    @_locked
    def set_option(self, name: str, value: int) -> None:
        """mcdc_ctx_set_option: "zc_batch_blocks", "zc_two", "zc_small",
        "test_fail_after_index" (test and tuning settings of this context)."""
        check(load().mcdc_ctx_set_option(self._h, name.encode(), int(value)))

    @_locked
    def timing(self) -> dict:
        t = McdcTiming()
        check(load().mcdc_ctx_timing(self._h, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in McdcTiming._fields_}

    # ---------------------------------------------------------- plumbing --
    @_locked
    def device_alloc(self, n: int) -> int:
        p = ctypes.c_void_p()
        check(load().mcdc_device_alloc(self._h, n, ctypes.byref(p)))
        return p.value

    @_locked
    def device_free(self, ptr: int) -> None:
        check(load().mcdc_device_free(self._h, ctypes.c_void_p(ptr)))

    @_locked
    def host_alloc(self, n: int) -> int:
        p = ctypes.c_void_p()
        check(load().mcdc_host_alloc(self._h, n, ctypes.byref(p)))
        return p.value

    @_locked
    def host_free(self, ptr: int) -> None:
        check(load().mcdc_host_free(self._h, ctypes.c_void_p(ptr)))

    @_locked
    def h2d(self, d_dst: int, data) -> None:
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                                 else data.view(np.uint8).reshape(-1))
        check(load().mcdc_memcpy_h2d(self._h, ctypes.c_void_p(d_dst), ctypes.c_void_p(a.ctypes.data), a.size))

    @_locked
    def fill_random(self, d_dst: int, n: int, seed: int, pos: int = 0) -> None:
        check(load().mcdc_fill_random_device(self._h, ctypes.c_void_p(d_dst), pos, n, seed))


class Batcher:
    """mcdc_batcher: worker threads call chunk() concurrently; files submitted
    together are chunked by one batched call (include/mcdc.h, "batching")."""

    def __init__(self, p: McdcParams, device: int = 0, max_batch_bytes: int = 1 << 30,
                 max_batch_files: int = 4096, gather_us: int = 200):
        L = load()
        self.params = p
        self._h = None
        h = ctypes.c_void_p()
        check(L.mcdc_batcher_create(device, ctypes.byref(p), max_batch_bytes, max_batch_files, gather_us,
                                    ctypes.byref(h)))
        self._h = h

    def chunk(self, data) -> np.ndarray:
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                                 else data.view(np.uint8).reshape(-1))
        cap = a.size // max(self.params.min_size - 1, 1) + 2
        out = np.empty(cap, dtype=CHUNK_DTYPE)
        n_out = ctypes.c_size_t()
        check(load().mcdc_batcher_chunk(self._h, ctypes.c_void_p(a.ctypes.data), a.size, out.ctypes.data, cap,
                                        ctypes.byref(n_out)))
        return out[: n_out.value].copy()

    def stats(self) -> dict:
        st = McdcBatcherStats()
        check(load().mcdc_batcher_stats(self._h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in McdcBatcherStats._fields_}

    def close(self):
        if self._h:
            load().mcdc_batcher_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def digest(chunks: np.ndarray) -> int:
    a = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
    return int(load().mcdc_digest(ctypes.c_void_p(a.ctypes.data), a.size))


class Index:
    """mcdc_index: the IDs stored or pending so far (Repository::save_blob's
    index.contains / add_pending_blob check, repository_v1.rs:169-180)."""

    def __init__(self, ctx: "Context", h: int):
        self._ctx, self._h = ctx, h

    def close(self):
        if self._h:
            load().mcdc_index_destroy(ctypes.c_void_p(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return int(load().mcdc_index_size(ctypes.c_void_p(self._h)))

    def add_device(self, d_ids: int, n: int, d_chunks: int, d_new: int) -> int:
        """Device-resident form: IDs and chunk records in HBM, the new chunks
        compacted into d_new (HBM); returns their number (no flags copied back)."""
        nn = ctypes.c_size_t()
        with self._ctx._lock:
            check(load().mcdc_index_add(self._ctx._h, ctypes.c_void_p(self._h), ctypes.c_void_p(d_ids), n, None,
                                        ctypes.c_void_p(d_chunks), ctypes.c_void_p(d_new), ctypes.byref(nn)))
        return nn.value

    def add(self, ids, chunks=None, d_ids: int = None, n: int = None):
        """Mark which IDs of a batch are new (mcdc_index_add) and add them.
        ids: (n, 32) uint8 host array, or d_ids (device pointer) with n.
        Returns is_new (n bools); with `chunks` (CHUNK_DTYPE, n records) also
        the new chunks in order."""
        if d_ids is None:
            a = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 32)
            iptr, n = a.ctypes.data, a.shape[0]
        else:
            a, iptr = None, d_ids
        flags = np.zeros(max(n, 1), dtype=np.uint8)
        nn = ctypes.c_size_t()
        if chunks is not None:
            c = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
            if c.size != n:
                raise ValueError("one chunk record per ID")
            out = np.zeros(max(n, 1), dtype=CHUNK_DTYPE)
            cptr, optr = c.ctypes.data, out.ctypes.data
        else:
            c = out = None
            cptr = optr = None
        with self._ctx._lock:
            check(load().mcdc_index_add(self._ctx._h, ctypes.c_void_p(self._h), ctypes.c_void_p(iptr), n,
                                        flags.ctypes.data, ctypes.c_void_p(cptr), ctypes.c_void_p(optr),
                                        ctypes.byref(nn)))
        is_new = flags[:n].astype(bool)
        if chunks is None:
            return is_new
        return is_new, out[:nn.value]
