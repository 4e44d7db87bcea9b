"""Multi-rank rehearsal on one GPU: world_size 2 (and 3), every rank a fresh
spawned process with its own mcdc context on device 0, gloo for the exchange
(the 8-GPU node runs the same code with one device per rank).  The HIP chunker
runs on every rank; the gathered result is compared with the oracle.

* file-sharded corpus (BASELINE configs[4]'s shape): files assigned by
  mapache_amd.shard.assign_files, each rank chunks its files in ONE
  mcdc_chunk_batch_device call over its own device arena; per-file lists
  gathered (mapache's per-file chunker, /root/reference/src/archiver/
  processor.rs:173; files processed independently, mod.rs:162-215);
* one stream split across ranks (shard.split_stream): each rank holds its slice
  plus a max-byte right halo in HBM, chunks it speculatively on the GPU, the
  exits are exchanged (integers only) and each rank continues the previous
  rank's exit on its GPU until the chains merge.  Random data and zero
  stretches spanning the seams (several exchange rounds).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SEED = 0x6d61706163686521
P16 = (16384, 65536, 262144, 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpus_sizes():
    rng = np.random.default_rng(91)
    sizes = rng.integers(0, 3 << 20, 300)
    sizes[::17] = 0
    sizes[5] = 40 << 20
    return [int(x) for x in sizes]


def _stream_parts():
    """(kind, length) pieces of the split-stream input: random, and zero runs
    that straddle slice boundaries out of phase."""
    return [("r", 5_000_003), ("z", 70 << 20), ("r", 30 << 20), ("z", 3 << 20), ("r", 60 << 20), ("z", 9_999_991),
            ("r", 40 << 20)]


def _stream_fill(ctx, dp, pos, length):
    """Write stream bytes [pos, pos + length) to device pointer dp."""
    at = 0
    zero = np.zeros(1 << 20, np.uint8)
    for kind, ln in _stream_parts():
        a, b = max(at, pos), min(at + ln, pos + length)
        if a < b:
            if kind == "r":
                ctx.fill_random(dp + (a - pos), b - a, SEED + 5, pos=a)
            else:
                for q in range(a, b, len(zero)):
                    ctx.h2d(dp + (q - pos), zero[: min(len(zero), b - q)])
        at += ln


def _stream_host():
    from oracle import oracle as O
    out, at = [], 0
    for kind, ln in _stream_parts():
        out.append(O.random_bytes(ln, SEED + 5, pos=at) if kind == "r" else np.zeros(ln, np.uint8))
        at += ln
    return np.concatenate(out)


def _worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mapache_amd import _lib, shard
        p = _lib.params(*P16)
        with _lib.Context(0, 1 << 30) as ctx:
            if mode == "files":
                sizes = _corpus_sizes()
                mine = shard.assign_files(sizes, world)[rank]
                offs = np.cumsum([0] + [sizes[i] for i in mine]).astype(np.uint64)
                arena = ctx.device_alloc(int(offs[-1]) + 16)
                try:
                    for i, o in zip(mine, offs[:-1]):
                        if sizes[i]:
                            ctx.fill_random(arena + int(o), sizes[i], SEED ^ (i + 1))

                    def chunk_indices(idx):
                        assert idx == mine
                        return ctx.chunk_batch_device(p, arena, offs[:-1], [sizes[i] for i in idx])
                    res = shard.chunk_sharded(sizes, chunk_indices, dst=0)
                finally:
                    ctx.device_free(arena)
                if rank == 0:
                    from oracle import oracle as O
                    ok = all(len(res[i]) == len(r) and (res[i] == r).all() for i, r in enumerate(
                        O.chunk(O.Params(*P16), O.random_bytes(sizes[i], SEED ^ (i + 1))) for i in range(len(sizes))))
                    q.put((rank, bool(ok), len(mine)))
                else:
                    q.put((rank, res is None, len(mine)))
            else:
                n = sum(ln for _, ln in _stream_parts())
                s, e = shard.stream_slices(n, world)[rank]
                hi = min(e + P16[2], n)
                dp = ctx.device_alloc(hi - s + 16)
                try:
                    _stream_fill(ctx, dp, s, hi - s)
                    got, st = shard.split_stream(lambda a, b: ctx.chunk_device(p, dp + (a - s), b - a),
                                                 shard.torch_allgather(), s, e, n, P16[2], rank, world)
                finally:
                    ctx.device_free(dp)
                parts = [None] * world
                dist.all_gather_object(parts, got)
                if rank == 0:
                    from oracle import oracle as O
                    ref = O.chunk(O.Params(*P16), _stream_host())
                    allc = np.concatenate(parts)
                    q.put((rank, bool(len(allc) == len(ref) and (allc == ref).all()), st["rounds"]))
                else:
                    q.put((rank, True, st["rounds"]))
    except BaseException as ex:
        q.put((rank, False, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


def _launch(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_rehearsal_file_sharded_corpus(world):
    res = _launch(world, "files")
    assert all(r[1] for r in res), res
    assert sum(r[2] for r in res) == len(_corpus_sizes())


@pytest.mark.parametrize("world", [2, 3])
def test_rehearsal_split_stream(world):
    res = _launch(world, "split")
    assert all(r[1] for r in res), res


def test_bench_two_ranks_rehearsal():
    """bench.py's own N > 1 path (the split stream with its exit exchange and the
    file-sharded corpus), launched as the driver launches it (torch.distributed.run,
    one fresh process per rank) in rehearsal mode (MCDC_BENCH_ONE_DEVICE=1: both
    ranks on device 0, the exchange and barriers over gloo), at a small size: the
    gathered split-stream boundary list (--parity) and every file of the sharded
    corpus must equal the oracle's."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MCDC_BENCH_ONE_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--gib", "0.75", "--corpus-files-per-gpu", "24", "--parity", "--no-cpu", "--cpu-threads",
           "8"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["bytes_per_gpu"] == int(0.75 * (1 << 30))
    sp = d["stream_parity"]
    assert sp["ok"], sp
    assert d["config"]["chunks_per_step"] == sp["oracle_chunks"]
    cs = d["corpus_sharded"]
    assert cs["parity_ok"] and cs["files"] == 48 and cs["corpus_digest"] == cs["oracle_corpus_digest"], cs
