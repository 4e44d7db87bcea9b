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
