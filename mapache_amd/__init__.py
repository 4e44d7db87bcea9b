"""mapache_amd — MI355X-native FastCDC v2020 chunker (the mapache Archiver hot path).

Host-side Python mirror of the chunker interface mapache uses
(``fastcdc::v2020::{StreamCDC, FastCDC, ChunkData, Normalization}``, called at
``/root/reference/src/archiver/processor.rs:173-202``) over the C ABI in
``include/mcdc.h`` (``libmcdc.so``: HIP kernels for gfx950).  There is no CPU
fallback: without the built library or a HIP device every call raises.
"""
from . import _lib, shard  # noqa: F401
from .fastcdc import (  # noqa: F401
    AVERAGE_MAX, AVERAGE_MIN, MAXIMUM_MAX, MAXIMUM_MIN, MINIMUM_MAX, MINIMUM_MIN,
    Chunk, ChunkData, Chunker, Error, FastCDC, Normalization, StreamCDC,
)

__all__ = ["Chunk", "ChunkData", "Chunker", "Error", "FastCDC", "Normalization", "StreamCDC"]
