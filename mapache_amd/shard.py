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


def _world(group):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def chunk_sharded(sizes: Sequence[int], chunk_indices: Callable[[list], "tuple[np.ndarray, np.ndarray]"],
                  group=None, dst: int | None = None) -> list[np.ndarray] | None:
    """Chunk a corpus of files (only their sizes are needed here) across the
    ranks of `group`; return the per-file chunk arrays in file order.

    `chunk_indices(indices) -> (chunks, counts)` chunks this rank's files (in
    the given, increasing order) — e.g. one ``mcdc_chunk_batch_device`` call
    over the rank's device arena.  With ``dst=None`` every rank receives the
    full result; otherwise only rank `dst` does (others get None).  Without an
    initialised process group this is a single-rank call."""
    import torch.distributed as dist

    world, rank = _world(group)
    mine = assign_files(sizes, world)[rank]
    if mine:
        ch, counts = chunk_indices(mine)
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
    result: list[np.ndarray | None] = [None] * len(sizes)
    for idx, ch, counts in parts:
        pos = 0
        for i, k in zip(idx, counts.tolist()):
            result[i] = ch[pos:pos + k]
            pos += k
    return result


def corpus_digest(counts: Sequence[int], digests: Sequence[int]) -> int:
    """Order-sensitive digest of a whole corpus's boundary lists, in file order:
    a fold of each file's chunk count and boundary-list digest (mcdc_digest of
    its file-relative records).  The bench gathers it across ranks; the oracle
    side folds oracle.random_files_digest the same way."""
    d = 0
    for c, x in zip(counts, digests):
        d = (d * 0x100000001b3 ^ int(x) ^ int(c)) & ((1 << 64) - 1)
    return d


def chunk_files_sharded(files: Sequence, chunk: ChunkFn, group=None, dst: int | None = None) -> list[np.ndarray] | None:
    """Chunk `files` (byte buffers, identical on every rank) across the ranks of
    `group`: ``chunk(list_of_buffers) -> (chunks, counts)`` is this rank's batch
    chunker, normally ``Context.chunk_batch`` bound to params on this rank's
    GPU.  See chunk_sharded."""
    return chunk_sharded([len(f) for f in files], lambda idx: chunk([files[i] for i in idx]), group, dst)


# ------------------------------------------------- one stream across ranks --
# A single long stream (one file) split across ranks ("fixed-
# size resyncing segments shard across the GPUs").  Chunk boundaries form a
# serial chain (a chunk starts where the previous one was cut), but chains
# started at different positions meet after a chunk or two and coincide from
# there on, so:
#
#   1. rank r holds its slice [s_r, e_r) plus a right halo of `max` bytes
#      (cut_gear never reads more than max bytes past a chunk start) and chunks
#      [s_r, min(e_r + max, n)) as if a file started at s_r: a speculative
#      chain, exact for every chunk starting before e_r *given* where it started;
#   2. each rank's exit (the end of its last chunk that starts before e_r) is
#      exchanged: one integer per rank, the only communication — no bytes move
#      between GPUs;
#   3. rank r continues the previous rank's exit x with short calls over
#      [x, x + W) until that chain meets its speculative chain (merge point):
#      its exact chunks are the continuation's up to the merge and the
#      speculative chain's from there.  A merge inside the slice leaves its
#      exit unchanged; a continuation that runs past e_r (a candidate-free
#      stretch across the seam) changes it, and the exchange repeats until no
#      exit changes (at most `world` rounds; two exchanges in the common case).
#
# `chunk(a, b)`: the rank's chunker over stream range [a, b) taken as one file
# (a CHUNK_DTYPE array, offsets relative to a; [a, b) within the rank's bytes).
# `allgather(v)`: every rank's integer v, in rank order.

def _absolute(ch, a):
    out = np.array(ch, dtype=CHUNK_DTYPE, copy=True)
    out["offset"] += np.uint64(a)
    return out


class ArrayChunks:
    """A chunk list in host memory (stream offsets)."""

    def __init__(self, recs: np.ndarray):
        self.recs = recs

    def __len__(self):
        return len(self.recs)

    def get(self, i0: int, i1: int) -> np.ndarray:
        return self.recs[i0:i1]

    def index(self, x: int) -> int:
        """first index whose offset >= x"""
        return int(np.searchsorted(self.recs["offset"], np.uint64(x)))

    def near_head(self, x: int) -> bool:
        return True


class DeviceChunks:
    """A chunk list left in HBM by mcdc_chunk_device (offsets relative to
    `base`): only its first and last `window` records are copied to the host
    (the seam exchange needs no more); anything else is fetched on demand."""

    def __init__(self, ctx, d_out: int, count: int, base: int, window: int = 256):
        self.ctx, self.d_out, self.count, self.base = ctx, d_out, count, base
        self.head = self._fetch(0, min(window, count))
        self.tail0 = max(count - window, len(self.head))
        self.tail = self._fetch(self.tail0, count)
        self.fetched_all = False

    def _fetch(self, i0, i1):
        if i1 <= i0:
            return np.empty(0, CHUNK_DTYPE)
        r = self.ctx.d2h_bytes(self.d_out + 24 * i0, 24 * (i1 - i0)).view(CHUNK_DTYPE).copy()
        r["offset"] += np.uint64(self.base)
        return r

    def __len__(self):
        return self.count

    def get(self, i0: int, i1: int) -> np.ndarray:
        i1 = min(i1, self.count)
        if i1 <= len(self.head):
            return self.head[i0:i1]
        if i0 >= self.tail0:
            return self.tail[i0 - self.tail0:i1 - self.tail0]
        return self._fetch(i0, i1)

    def index(self, x: int) -> int:
        x = np.uint64(x)
        if len(self.head) and (len(self.head) == self.count or x <= self.head["offset"][-1]):
            return int(np.searchsorted(self.head["offset"], x))
        if len(self.tail) and x > self.tail["offset"][0]:
            return self.tail0 + int(np.searchsorted(self.tail["offset"], x))
        self.fetched_all = True  # rare (an entry deep inside the slice): binary search over HBM
        lo, hi = len(self.head), self.tail0
        while lo < hi:
            mid = (lo + hi) // 2
            if self._fetch(mid, mid + 1)["offset"][0] < x:
                lo = mid + 1
            else:
                hi = mid
        return lo

    def near_head(self, x: int) -> bool:
        return len(self.head) == self.count or (len(self.head) and x <= int(self.head["offset"][-1]))


class SplitResult:
    """A rank's exact chunks: continuation records, then spec[k0:k1]."""

    def __init__(self, fix: np.ndarray, spec, k0: int, k1: int):
        self.fix, self.spec, self.k0, self.k1 = fix, spec, k0, k1

    def __len__(self):
        return len(self.fix) + max(self.k1 - self.k0, 0)

    def last(self):
        if self.k1 > self.k0:
            return self.spec.get(self.k1 - 1, self.k1)[0]
        return self.fix[-1] if len(self.fix) else None

    def materialize(self) -> np.ndarray:
        parts = [self.fix] + ([self.spec.get(self.k0, self.k1)] if self.k1 > self.k0 else [])
        return np.concatenate(parts) if len(parts) > 1 else parts[0].copy()


def split_stream(chunk, allgather, s: int, e: int, n: int, max_size: int, rank: int, world: int,
                 fix_window: int | None = None, spec=None, materialize: bool = True):
    """This rank's exact chunks of the stream [0, n) that start in [s, e) (stream
    offsets, in order) and a dict of counters: continuation calls, exchange
    rounds, whether the entry merged into the speculative chain.

    `spec`: this rank's speculative list if already computed (an ArrayChunks /
    DeviceChunks over [s, min(e + max, n))); with materialize=False the result
    is a SplitResult (count and records on demand)."""
    hi = min(e + max_size, n)
    if spec is None:
        spec = ArrayChunks(_absolute(chunk(s, hi), s))
    empty = np.empty(0, CHUNK_DTYPE)
    stats = {"fixup_calls": 0, "rounds": 0, "merged": True}
    k_end = spec.index(e)  # spec records starting before e

    def on_spec(x):
        k = spec.index(x)
        return k if k < len(spec) and int(spec.get(k, k + 1)["offset"][0]) == x else -1

    def resolve(x: int) -> SplitResult:
        recs, w = [], int(fix_window or 16 * max_size)
        while x < e:
            k = on_spec(x)
            if k >= 0:  # on the speculative chain from here on
                return SplitResult(np.concatenate(recs) if recs else empty, spec, k, k_end)
            stats["merged"] = False
            b = min(x + w, hi)
            f = _absolute(chunk(x, b), x)
            stats["fixup_calls"] += 1
            if b < n:  # exact cuts only: >= max bytes ahead of their start
                f = f[f["offset"] + np.uint64(max_size) <= np.uint64(b)]
            if len(f) == 0:
                w *= 2
                continue
            k0, k1 = spec.index(int(f["offset"][0])), spec.index(int(f["offset"][-1]) + 1)
            near = spec.get(k0, k1)["offset"]
            hit = np.nonzero(np.isin(f["offset"], near))[0]
            if hit.size:  # merge: the continuation's chunks before it, then the speculative chain
                g = f[: hit[0]]
                recs.append(g[g["offset"] < e])
                x = int(f["offset"][hit[0]])
                stats["merged"] = True
                continue
            recs.append(f[f["offset"] < e])
            x = int(f["offset"][-1] + f["length"][-1])  # a true node past the exact cuts
            w *= 2
        return SplitResult(np.concatenate(recs) if recs else empty, spec, 0, 0)

    def exit_of(res: SplitResult, entry: int) -> int:
        r = res.last()
        return int(r["offset"] + r["length"]) if r is not None else entry

    mine = resolve(s)  # round 0: assume the chain enters at s
    my_exit = exit_of(mine, s)
    entry_prev, seen = s, None
    while True:
        stats["rounds"] += 1
        exits = [int(v) for v in allgather(my_exit if rank < world - 1 else n)]
        if exits == seen:
            break
        seen = exits
        entry = 0 if rank == 0 else exits[rank - 1]
        if entry != entry_prev:
            entry_prev = entry
            mine = resolve(entry)
            my_exit = exit_of(mine, entry)
        if stats["rounds"] > world + 1:
            raise RuntimeError("seam exchange did not settle")
    return (mine.materialize() if materialize else mine), stats


def torch_allgather(group=None):
    """allgather(v) over torch.distributed's gloo backend: one int64 per rank,
    host tensors only.  The exchange is 8 bytes per rank (no
    data-path collective), so it never needs RCCL, and the libmcdc process
    never initialises torch's own HIP runtime beside libmcdc's."""
    import torch
    import torch.distributed as dist

    def ag(v):
        world = dist.get_world_size(group)
        t = torch.tensor([int(v)], dtype=torch.int64)
        out = torch.zeros(world, dtype=torch.int64)
        dist.all_gather_into_tensor(out, t, group=group)
        return out.tolist()
    return ag


def stream_slices(n: int, world: int, align: int = 4096):
    """[s_r, e_r) of a stream of n bytes split into `world` near-equal slices
    (boundaries rounded to `align`)."""
    cuts = [min(n, (n * r // world) // align * align) for r in range(world)] + [n]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]
