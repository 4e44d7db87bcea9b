"""Python mirror of the chunker API mapache calls, backed by the MI355X kernels.

The reference calls the Rust crate ``fastcdc`` 3.2.1, module ``v2020``
(``/root/reference/Cargo.toml:23``) at
``/root/reference/src/archiver/processor.rs:173-202``::

    let chunker = StreamCDC::with_level(reader, MIN_CHUNK_SIZE as u32,
                                        AVG_CHUNK_SIZE as u32, MAX_CHUNK_SIZE as u32,
                                        Normalization::Level1);
    for result in chunker { let chunk = result?; ... chunk.data ... }

This module keeps those names and argument meanings:

* ``Normalization`` — ``Level0`` .. ``Level3``.
* ``FastCDC(source, min_size, avg_size, max_size, level=Level1)`` /
  ``FastCDC.with_level`` — iterate ``Chunk(hash, offset, length)`` over an
  in-memory buffer.
* ``StreamCDC(source, ...)`` / ``StreamCDC.with_level`` — iterate
  ``ChunkData(hash, offset, length, data)`` over a ``read()``-able source.
* Invalid sizes fail the crate's ``assert!``s; here they raise
  ``AssertionError`` with the crate's condition (a Rust panic has no
  recoverable counterpart).  Read failures raise ``IoError`` (the crate's
  ``Error::IoError``); end of stream simply ends iteration (``Error::Empty``).

Every boundary comes from ``libmcdc.so`` (HIP, gfx950) through the C ABI in
``include/mcdc.h``; nothing here computes a cut.
"""
from __future__ import annotations

import enum
import io
import threading
from dataclasses import dataclass
from typing import Iterator, Optional

import numpy as np

from . import _lib

# crate v2020 bounds (asserted by FastCDC/StreamCDC::with_level)
MINIMUM_MIN, MINIMUM_MAX = 64, 1_048_576
AVERAGE_MIN, AVERAGE_MAX = 256, 4_194_304
MAXIMUM_MIN, MAXIMUM_MAX = 1024, 16_777_216

# mapache's own parameters (src/global/defaults.rs:35-40)
MAPACHE_MIN_CHUNK_SIZE = 512 * 1024
MAPACHE_AVG_CHUNK_SIZE = 1024 * 1024
MAPACHE_MAX_CHUNK_SIZE = 8 * 1024 * 1024


class Normalization(enum.IntEnum):
    Level0 = 0
    Level1 = 1
    Level2 = 2
    Level3 = 3


@dataclass(frozen=True)
class Chunk:
    """fastcdc::v2020::Chunk — a cut point in a slice."""
    hash: int
    offset: int
    length: int


@dataclass(frozen=True)
class ChunkData:
    """fastcdc::v2020::ChunkData — a chunk read from a stream, with its bytes."""
    hash: int
    offset: int
    length: int
    data: bytes


class Error(Exception):
    """fastcdc::v2020::Error."""


class IoError(Error):
    """Error::IoError — the source's read() failed."""


class Other(Error):
    """Error::Other."""


def _check_sizes(min_size: int, avg_size: int, max_size: int, level) -> None:
    # the crate's asserts, in the crate's order
    assert min_size >= MINIMUM_MIN, "assertion failed: min_size >= MINIMUM_MIN"
    assert min_size <= MINIMUM_MAX, "assertion failed: min_size <= MINIMUM_MAX"
    assert avg_size >= AVERAGE_MIN, "assertion failed: avg_size >= AVERAGE_MIN"
    assert avg_size <= AVERAGE_MAX, "assertion failed: avg_size <= AVERAGE_MAX"
    assert max_size >= MAXIMUM_MIN, "assertion failed: max_size >= MAXIMUM_MIN"
    assert max_size <= MAXIMUM_MAX, "assertion failed: max_size <= MAXIMUM_MAX"
    Normalization(int(level))


# ------------------------------------------------------------- contexts --
# One default context per thread: mapache chunks files on several rayon
# workers at once (/root/reference/src/archiver/mod.rs:162-215), a context
# serves one thread at a time (mcdc.h), and replacing a too-small context must
# never close one that another thread is using.
_tls = threading.local()
DEFAULT_MAX_BYTES = 1 << 30


def default_context(max_bytes: int = DEFAULT_MAX_BYTES, device: int = 0) -> _lib.Context:
    """This thread's context on `device` (created on first use, grown on demand)."""
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    c = ctxs.get(device)
    if c is None or c.max_bytes < max_bytes:
        if c is not None:
            c.close()  # only this thread ever used it
        c = ctxs[device] = _lib.Context(device, max(max_bytes, DEFAULT_MAX_BYTES))
    return c


class Chunker:
    """Reusable handle: one mcdc context (device, stream, workspace) + params."""

    def __init__(self, min_size: int, avg_size: int, max_size: int,
                 level: Normalization = Normalization.Level1, *, device: int = 0,
                 max_bytes: int = DEFAULT_MAX_BYTES, ctx: Optional[_lib.Context] = None):
        _check_sizes(min_size, avg_size, max_size, level)
        self.params = _lib.params(min_size, avg_size, max_size, int(level))
        self.min_size, self.avg_size, self.max_size = min_size, avg_size, max_size
        self.level = Normalization(int(level))
        self.ctx = ctx if ctx is not None else _lib.Context(device, max_bytes)

    def chunk(self, data) -> np.ndarray:
        """Structured array (offset, length, hash) for one host buffer."""
        return self.ctx.chunk_host(self.params, data)

    def chunk_device(self, d_ptr: int, n: int) -> np.ndarray:
        return self.ctx.chunk_device(self.params, d_ptr, n)

    def chunk_many(self, buffers):
        """(chunks, per-buffer counts) for many independent buffers (files)."""
        return self.ctx.chunk_batch(self.params, buffers)

    def timing(self) -> dict:
        return self.ctx.timing()


# --------------------------------------------------------------- FastCDC --
class FastCDC:
    """fastcdc::v2020::FastCDC over an in-memory buffer."""

    def __init__(self, source, min_size: int, avg_size: int, max_size: int,
                 level: Normalization = Normalization.Level1, *, ctx: Optional[_lib.Context] = None):
        _check_sizes(min_size, avg_size, max_size, level)
        self._buf = memoryview(source).cast("B") if not isinstance(source, np.ndarray) else source
        self._params = _lib.params(min_size, avg_size, max_size, int(level))
        self._ctx = ctx
        self._chunks: Optional[np.ndarray] = None
        self._i = 0

    @classmethod
    def new(cls, source, min_size: int, avg_size: int, max_size: int) -> "FastCDC":
        return cls(source, min_size, avg_size, max_size, Normalization.Level1)

    @classmethod
    def with_level(cls, source, min_size: int, avg_size: int, max_size: int,
                   level: Normalization) -> "FastCDC":
        return cls(source, min_size, avg_size, max_size, level)

    def _run(self) -> np.ndarray:
        if self._chunks is None:
            n = len(self._buf)
            ctx = self._ctx or default_context(max(n, 1))
            self._chunks = ctx.chunk_host(self._params, np.frombuffer(self._buf, dtype=np.uint8)
                                          if not isinstance(self._buf, np.ndarray) else self._buf)
        return self._chunks

    def __iter__(self) -> Iterator[Chunk]:
        return self

    def __next__(self) -> Chunk:
        c = self._run()
        if self._i >= len(c):
            raise StopIteration
        r = c[self._i]
        self._i += 1
        return Chunk(int(r["hash"]), int(r["offset"]), int(r["length"]))


# ------------------------------------------------------------- StreamCDC --
class StreamCDC:
    """fastcdc::v2020::StreamCDC over a read()-able source.

    The source is consumed in windows of ``window`` bytes (>= 2 * max_size).
    A chunk starting at c is final once c + max_size lies inside the bytes
    read so far (cut_gear never looks further); the unfinished tail is carried
    into the next window, so the output equals chunking the whole stream.
    """

    def __init__(self, source, min_size: int, avg_size: int, max_size: int,
                 level: Normalization = Normalization.Level1, *, window: int = 256 << 20,
                 ctx: Optional[_lib.Context] = None):
        _check_sizes(min_size, avg_size, max_size, level)
        self._src = source
        self._params = _lib.params(min_size, avg_size, max_size, int(level))
        self._max = max_size
        self._window = max(int(window), 2 * max_size)
        self._ctx = ctx
        self._pending: list = []
        self._carry = b""
        self._processed = 0
        self._eof = False

    @classmethod
    def new(cls, source, min_size: int, avg_size: int, max_size: int) -> "StreamCDC":
        return cls(source, min_size, avg_size, max_size, Normalization.Level1)

    @classmethod
    def with_level(cls, source, min_size: int, avg_size: int, max_size: int,
                   level: Normalization) -> "StreamCDC":
        return cls(source, min_size, avg_size, max_size, level)

    def _read(self, n: int) -> bytes:
        out = []
        got = 0
        while got < n:
            try:
                b = self._src.read(n - got)
            except (OSError, io.UnsupportedOperation) as e:  # Error::IoError
                raise IoError(str(e)) from e
            if not b:
                self._eof = True
                break
            out.append(bytes(b))
            got += len(b)
        return b"".join(out)

    def _fill(self) -> None:
        buf = self._carry + self._read(self._window - len(self._carry))
        if not buf:
            return
        ctx = self._ctx or default_context(max(len(buf), 1))
        chunks = ctx.chunk_host(self._params, np.frombuffer(buf, dtype=np.uint8))
        if self._eof:
            final, keep_from = chunks, len(buf)
        else:
            ok = chunks["offset"] + self._max <= len(buf)
            final = chunks[ok]
            keep_from = int(chunks["offset"][~ok][0]) if (~ok).any() else len(buf)
        mv = memoryview(buf)
        for r in final:
            o, ln = int(r["offset"]), int(r["length"])
            self._pending.append(ChunkData(int(r["hash"]), self._processed + o, ln, bytes(mv[o:o + ln])))
        self._processed += keep_from
        self._carry = buf[keep_from:]

    def __iter__(self) -> Iterator[ChunkData]:
        return self

    def __next__(self) -> ChunkData:
        while not self._pending:
            if self._eof:
                raise StopIteration  # Error::Empty ends the iterator
            self._fill()
        return self._pending.pop(0)
