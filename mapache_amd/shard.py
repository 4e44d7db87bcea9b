"""Multi-GPU sharding of the chunking path: one process per GPU, files as the unit.

mapache's Archiver builds a fresh chunker per file
(/root/reference/src/archiver/processor.rs:160-179) and its rayon workers
process files independently (/root/reference/src/archiver/mod.rs:162-167), so
the path partitions by file with no data exchange: each rank chunks the files
assigned to it on its own GPU.  The only communication is control-plane — the
per-file boundary lists gathered to the caller (a few dozen bytes per chunk),
done with ``torch.distributed`` object collectives, never on the byte stream.

  assign_files(sizes, world)          longest-processing-time greedy by bytes
  chunk_files_sharded(files, chunk)   this rank's share -> gathered per-file lists
"""
from __future__ import annotations

import heapq
from typing import Callable, Sequence

import numpy as np

from ._lib import CHUNK_DTYPE


def assign_files(sizes: Sequence[int], world: int) -> list[list[int]]:
    """Partition file indices over `world` ranks, balancing total bytes.

    LPT greedy: files in decreasing size go to the least-loaded rank (ties by
    rank id), which bounds the busiest rank at 4/3 of optimal.  Every rank's
    list is returned in increasing file index, so each rank's batch keeps the
    caller's order.  Deterministic: every rank computes the same assignment
    from the same sizes without communicating.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0, r) for r in range(world)]
    out: list[list[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-int(sizes[i]), i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    for lst in out:
        lst.sort()
    return out


def rank_bytes(sizes: Sequence[int], assignment: list[list[int]]) -> list[int]:
    return [sum(int(sizes[i]) for i in lst) for lst in assignment]


ChunkFn = Callable[[list], "tuple[np.ndarray, np.ndarray]"]


def chunk_files_sharded(files: Sequence, chunk: ChunkFn, group=None, dst: int | None = None) -> list[np.ndarray] | None:
    """Chunk `files` (sequence of byte buffers, identical on every rank) across
    the ranks of `group`; return the per-file chunk arrays in file order.

    `chunk(list_of_buffers) -> (chunks, counts)` is this rank's batch chunker,
    normally ``Context.chunk_batch`` bound to ``params`` on this rank's GPU.
    With ``dst=None`` every rank receives the full result; otherwise only rank
    `dst` does (others get None).  Without an initialised process group this
    is a single-rank call.
    """
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    else:
        world, rank = 1, 0
    sizes = [len(f) for f in files]
    mine = assign_files(sizes, world)[rank]
    if mine:
        ch, counts = chunk([files[i] for i in mine])
    else:
        ch, counts = np.empty(0, CHUNK_DTYPE), np.empty(0, np.uint64)
    part = (mine, np.asarray(ch, dtype=CHUNK_DTYPE), np.asarray(counts, dtype=np.uint64))
    if world == 1:
        parts = [part]
    elif dst is None:
        parts = [None] * world
        dist.all_gather_object(parts, part, group=group)
    else:
        parts = [None] * world if rank == dst else None
        dist.gather_object(part, parts, dst=dst, group=group)
        if rank != dst:
            return None
    result: list[np.ndarray | None] = [None] * len(files)
    for idx, ch, counts in parts:
        pos = 0
        for i, k in zip(idx, counts.tolist()):
            result[i] = ch[pos:pos + k]
            pos += k
    return result
