"""Multi-rank sharding (mapache_amd.shard): files partition across ranks with
no data exchange; gathered per-file boundary lists equal single-process
chunking.  CPU: world_size 2 over gloo with the oracle as each rank's chunker
(the GPU chunker is the same callable on a GPU box: Context.chunk_batch)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mapache_amd import shard
from oracle import oracle as O

P = (4096, 16384, 65536, 1)


def _files():
    rng = np.random.default_rng(5)
    sizes = [0, 1, 4095, 70_000, 3 << 20, 100] + rng.integers(0, 1 << 20, 37).tolist()
    return [O.random_bytes(int(s), 500 + i) for i, s in enumerate(sizes)]


def test_assign_files_balances_and_covers():
    rng = np.random.default_rng(1)
    sizes = rng.integers(0, 1 << 30, 1000).tolist()
    for world in (1, 2, 3, 8):
        a = shard.assign_files(sizes, world)
        flat = sorted(i for lst in a for i in lst)
        assert flat == list(range(len(sizes)))
        assert all(lst == sorted(lst) for lst in a)
        loads = shard.rank_bytes(sizes, a)
        # LPT: busiest rank <= mean + largest file
        assert max(loads) <= sum(sizes) / world + max(sizes)
    assert shard.assign_files([], 4) == [[], [], [], []]
    with pytest.raises(ValueError):
        shard.assign_files([1], 0)


def test_assign_files_deterministic_ties():
    assert shard.assign_files([5, 5, 5, 5], 2) == [[0, 2], [1, 3]]


def test_single_rank_without_process_group():
    files = _files()
    got = shard.chunk_files_sharded(files, lambda fs: O.chunk_files(O.Params(*P), fs))
    for f, g in zip(files, got):
        r = O.chunk(O.Params(*P), f)
        assert (g == r).all() and len(g) == len(r)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = _files()
        seen = []

        def chunk(fs):
            seen.append(sum(len(f) for f in fs))
            return O.chunk_files(O.Params(*P), fs)

        full = shard.chunk_files_sharded(files, chunk)
        only0 = shard.chunk_files_sharded(files, chunk, dst=0)
        ok = all(len(g) == len(O.chunk(O.Params(*P), f)) and (g == O.chunk(O.Params(*P), f)).all()
                 for f, g in zip(files, full))
        if rank == 0:
            ok &= all((a == b).all() for a, b in zip(full, only0))
        else:
            ok &= only0 is None
        q.put((rank, ok, seen[0]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_world2_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [r[1] for r in res] == [True, True]
    total = sum(len(f) for f in _files())
    assert res[0][2] + res[1][2] == total          # every byte chunked exactly once
    assert min(res[0][2], res[1][2]) > total // 4  # and the work is split


@pytest.mark.gpu
def test_gpu_rank_chunker_through_shard(ctx):
    from mapache_amd import _lib
    files = _files()
    got = shard.chunk_files_sharded(files, lambda fs: ctx.chunk_batch(_lib.params(*P), fs))
    for f, g in zip(files, got):
        r = O.chunk(O.Params(*P), f)
        assert len(g) == len(r) and (g == r).all()


# ------------------------------------------------------ one stream, split --
def _split_threads(data, p, world, fix_window=None):
    """split_stream on `world` threads (a barrier-synchronised allgather), the
    oracle as every rank's chunker; returns the concatenated list and stats."""
    import threading
    n = len(data)
    slices = shard.stream_slices(n, world)
    bar = threading.Barrier(world)
    box = [None] * world
    res, errs = [None] * world, []

    def ag_for(r):
        def ag(v):
            box[r] = v
            bar.wait()
            out = list(box)
            bar.wait()
            return out
        return ag

    def run(r):
        try:
            s, e = slices[r]
            res[r] = shard.split_stream(lambda a, b: O.chunk(O.Params(*p), data[a:b]), ag_for(r), s, e, n, p[2], r,
                                        world, fix_window)
        except BaseException as ex:
            errs.append(repr(ex))
            bar.abort()
    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    return np.concatenate([x[0] for x in res]), [x[1] for x in res]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("p", [(16384, 65536, 262144, 1), (64, 256, 1024, 1), (524288, 1048576, 8388608, 1)],
                         ids=lambda p: "/".join(map(str, p)))
def test_split_stream_random(p, world):
    d = O.random_bytes((24 << 20) + 12345, 61)
    got, st = _split_threads(d, p, world)
    ref = O.chunk(O.Params(*p), d)
    assert len(got) == len(ref) and (got == ref).all()
    assert all(s["rounds"] <= 2 for s in st)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_split_stream_seams_in_forced_stretches(world):
    """Zero stretches out of phase with every slice start, some spanning several
    seams: continuations run past slice ends, exits change, the exchange repeats."""
    p = (4096, 16384, 65536, 1)
    parts = [O.random_bytes(100_003, 71)]
    for k in range(6):
        parts += [np.zeros((3 << 20) + 777 * k, np.uint8), O.random_bytes(200_000 + 33 * k, 72 + k)]
    parts += [np.zeros(9 << 20, np.uint8), O.random_bytes(1 << 20, 90)]
    d = np.concatenate(parts)
    got, st = _split_threads(d, p, world, fix_window=4 * p[2])
    ref = O.chunk(O.Params(*p), d)
    assert len(got) == len(ref) and (got == ref).all()
    assert max(s["rounds"] for s in st) >= 2


def _split_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = (16384, 65536, 262144, 1)
        n = (20 << 20) + 99
        s, e = shard.stream_slices(n, world)[rank]
        hi = min(e + p[2], n)
        mine = O.random_bytes(hi - s, 63, pos=s)  # this rank's bytes only: slice + right halo
        got, st = shard.split_stream(lambda a, b: O.chunk(O.Params(*p), mine[a - s:b - s]),
                                     shard.torch_allgather(), s, e, n, p[2], rank, world)
        parts = [None] * world
        dist.all_gather_object(parts, got)
        if rank == 0:
            ref = O.chunk(O.Params(*p), O.random_bytes(n, 63))
            allc = np.concatenate(parts)
            q.put((rank, bool(len(allc) == len(ref) and (allc == ref).all()), st["rounds"]))
        else:
            q.put((rank, True, st["rounds"]))
    finally:
        dist.destroy_process_group()


def test_split_stream_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [r[1] for r in res] == [True, True], res
