#!/usr/bin/env python3
"""bench.py — device-resident GiB/s chunked, FastCDC 16/64/256 KiB L1, MI355X.

Workload (BASELINE.json configs[1]): per GPU one 64 GiB uniform-random byte
buffer resident in HBM (counter-based PRNG generated on the device, seed per
rank), FastCDC v2020 at min/avg/max = 16/64/256 KiB, Normalization::Level1.
A step = one full chunking pass over that buffer through the C ABI
(mcdc_chunk_device: scan + chain resolution + boundary emission), with the
boundary list written to a device-resident output array (device-resident in,
device-resident out: the next pipeline stage consumes it in HBM).  The same
call with the list written to pinned host memory is reported beside it
("host_out").  N GPUs = N independent streams (weak scaling, no collectives on
the data path; torch.distributed is used only for the barrier and the
max-over-ranks timing).

Prints ONE JSON line (rank 0).  Extra objects:
  roofline      - the scan kernel (dominant) vs HBM peak: algorithmic bytes per
                  launch (1 byte read per input byte) / average launch time from
                  HIP events recorded on the library's stream.
  cpu_baseline  - oracle/ C restatement of the crate, 1 thread, bounded sample
                  of the same stream (rank 0, N=1 only).
  host_out      - same step, boundary list to pinned host memory (PCIe-inclusive)
  e2e_host      - pinned host input -> H2D -> kernels -> boundaries to host
  batch_files   - BASELINE configs[2]: 10 000 independent 8 MiB files, one call
  small_files   - BASELINE configs[3] stand-in: synthetic kernel-tree-like mix
  chunk_ids     - SURVEY.md §8(f) next stage: BLAKE3 chunk IDs of the same 64 GiB
                  boundary list in HBM (ID::from_content, processor.rs:184), and
                  the chunk + ID pipeline
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident GiB/s chunked, FastCDC 16/64/256 KiB, 1 & 8 MI355X"
SEED = 0x6d61706163686521
PARAMS = (16384, 65536, 262144, 1)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GIB = 1 << 30


def _dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def _pmc_traffic():
    """Calibrated PMC read traffic of the scan (profiles/r01/pmc_traffic.json, written from a
    separate rocprofv3 --pmc FETCH_SIZE pass by tools/pmc_calib.sh): HBM bytes per input byte."""
    path = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return float(d["traffic_per_input_byte"]), os.path.relpath(path, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def _bind_near_gpu(device: int):
    """Run this process on the CPUs of the GPU's NUMA node (intersected with the
    CPUs it may use), so pinned host buffers are first-touched next to the GPU's
    PCIe root.  Returns the node or None; never fails the bench."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return None
        bus = buf.value.decode().lower()
        node = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
        if node < 0:
            return None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        mine = cpus & os.sched_getaffinity(0)
        if not mine:
            return None
        os.sched_setaffinity(0, mine)
        return node
    except (OSError, ValueError, AttributeError):
        return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def _same(a: np.ndarray, b: np.ndarray) -> bool:
    return bool(len(a) == len(b) and (a["offset"] == b["offset"]).all() and (a["length"] == b["length"]).all()
                and (a["hash"] == b["hash"]).all())


def cpu_baseline(sample_gib: float, gpu_chunks: np.ndarray) -> dict:
    """Oracle (C restatement of fastcdc v2020), single thread, on the first
    `sample_gib` GiB of rank 0's stream.  Also cross-checks the GPU boundaries
    that lie wholly inside the sample (a size-independent parity probe)."""
    from oracle import oracle as O
    n = int(sample_gib * GIB)
    d = O.random_bytes(n, SEED)  # generation is not timed
    t0 = time.perf_counter()
    c = O.chunk(O.Params(*PARAMS), d)
    dt = time.perf_counter() - t0
    # GPU chunks that end before the sample's last max-window are final in both
    lim = n - PARAMS[2]
    g = gpu_chunks[gpu_chunks["offset"] + PARAMS[2] <= lim]
    ok = len(g) > 0 and _same(g, c[: len(g)])
    return {"value": round(n / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {sample_gib:g} GiB of the rank-0 stream (seed 0x{SEED:x}), 16/64/256 KiB L1, "
                      f"oracle/fastcdc_oracle.c cut_gear loop, 1 thread, input pre-generated in RAM",
            "cpu": _cpu_model(), "seconds": round(dt, 3), "parity_probe_chunks": int(len(g)),
            "parity_probe_ok": bool(ok)}


def e2e_host(ctx, p, gib: float) -> dict:
    """End-to-end host path: pinned host buffer -> H2D -> kernels -> boundaries to host."""
    import ctypes
    from mapache_amd import _lib
    n = int(gib * GIB)
    hp = ctx.host_alloc(n)
    dp = ctx.device_alloc(n)
    try:
        ctx.fill_random(dp, n, SEED ^ 0x55)
        lib = _lib.load()
        _lib.check(lib.mcdc_memcpy_d2h(ctx._h, ctypes.c_void_p(hp), ctypes.c_void_p(dp), n))
        out = np.zeros(n // (p.min_size - 1) + 2, dtype=_lib.CHUNK_DTYPE)
        n_out = ctypes.c_size_t()
        best, bt = None, None
        for _ in range(3):
            t0 = time.perf_counter()
            _lib.check(lib.mcdc_chunk_host(ctx._h, ctypes.byref(p), ctypes.c_void_p(hp), n,
                                           out.ctypes.data, out.size, ctypes.byref(n_out)))
            dt = time.perf_counter() - t0
            if best is None or dt < best:
                best, bt = dt, ctx.timing()
        return {"bytes": n, "gib_s": round(n / best / GIB, 2), "h2d_ms": round(bt["h2d_ms"], 3),
                "device_ms": round(bt["device_ms"], 3), "d2h_ms": round(bt["d2h_ms"], 3),
                "total_ms": round(bt["total_ms"], 3), "source": "pinned host buffer (hipHostMalloc)"}
    finally:
        ctx.host_free(hp)
        ctx.device_free(dp)


def _timed(fn, steps: int, warmup: int):
    for _ in range(warmup):
        fn()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = fn()
    return (time.perf_counter() - t0) / steps, r


def batch_files(ctx, p, nfiles: int, size: int, steps: int, cpu_files: int = 0, cpu_threads: int = 16) -> dict:
    """BASELINE configs[2]: `nfiles` independent files of `size` bytes back to back
    in one device arena (each file's chain restarts at 0), one batched call."""
    from mapache_amd import _lib
    n = nfiles * size
    arena = ctx.device_alloc(n)
    cap = nfiles * (size // (p.min_size - 1) + 2)
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(arena, n, SEED ^ 0xB0)
        offs = np.arange(nfiles, dtype=np.uint64) * size
        lens = np.full(nfiles, size, dtype=np.uint64)
        dt, (total, counts) = _timed(lambda: ctx.chunk_batch_device_to_device(p, arena, offs, lens, d_out, cap),
                                     steps, 1)
        t = ctx.timing()
        # parity probe: three files against the oracle
        from oracle import oracle as O
        chunks = ctx.d2h_chunks(d_out, total)
        starts = np.concatenate([[0], np.cumsum(counts)])
        ok = int(counts.sum()) == total
        for i in (nfiles // 2, nfiles - 1):
            host = O.random_bytes(size, SEED ^ 0xB0, pos=i * size)
            ok &= _same(chunks[starts[i]:starts[i + 1]], O.chunk(O.Params(*PARAMS), host))
        r = {"files": nfiles, "file_bytes": size, "bytes": n, "steps": steps,
             "ms_per_step": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2),
             "files_per_s": round(nfiles / dt, 1), "chunks": int(total),
             "scan_ms": round(t["scan_ms"], 3), "device_ms": round(t["device_ms"], 3),
             "data": "synthetic uniform-random (device PRNG), per-file counts returned"}
        if cpu_files > 0:
            # files in parallel on the host cores (the nproc-thread
            # baseline), the first `cpu_files` files of the same arena; their
            # boundary lists double as the parity probe
            k = min(cpu_files, nfiles)
            host = O.random_bytes(k * size, SEED ^ 0xB0)  # generation is not timed
            files = [host[i * size:(i + 1) * size] for i in range(k)]
            O.chunk_files(O.Params(*PARAMS), files[:cpu_threads], threads=cpu_threads)  # page-in, warm
            t0 = time.perf_counter()
            ref, rc = O.chunk_files(O.Params(*PARAMS), files, threads=cpu_threads)
            cdt = time.perf_counter() - t0
            ok &= bool((rc == counts[:k]).all()) and _same(chunks[:int(starts[k])], ref)
            r["cpu_baseline"] = {"value": round(k * size / cdt / GIB, 3), "unit": "GiB/s", "cores": cpu_threads,
                                 "kind": "port", "seconds": round(cdt, 3),
                                 "sample": f"first {k} of the {nfiles} files ({k * size / GIB:g} GiB), "
                                           f"oracle/fastcdc_oracle.c, one file per thread at a time, "
                                           f"{cpu_threads} threads, input pre-generated in RAM",
                                 "cpu": _cpu_model()}
        r["parity_probe_files"] = 2 + (min(cpu_files, nfiles) if cpu_files > 0 else 0)
        r["parity_probe_ok"] = bool(ok)
        return r
    finally:
        ctx.device_free(d_out)
        ctx.device_free(arena)


def small_files(ctx, p, nfiles: int, steps: int) -> dict:
    """Stand-in for BASELINE configs[3] (no kernel tree here or on the box):
    `nfiles` files with a log-normal size mix (median 8 KiB, sigma 1.2, capped at
    64 MiB), random bytes, packed back to back in one device arena."""
    from mapache_amd import _lib
    rng = np.random.default_rng(20251016)
    sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, nfiles)).astype(np.uint64) + 1, 64 << 20)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    n = int(sizes.sum())
    arena = ctx.device_alloc(n + 16)
    cap = int(sum(int(s) // (p.min_size - 1) + 2 for s in sizes))
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(arena, n, SEED ^ 0x5F)
        dt, (total, counts) = _timed(lambda: ctx.chunk_batch_device_to_device(p, arena, offs, sizes, d_out, cap),
                                     steps, 1)
        from oracle import oracle as O
        chunks = ctx.d2h_chunks(d_out, total)
        host = O.random_bytes(n, SEED ^ 0x5F)
        ref, rc = O.chunk_files(O.Params(*PARAMS), [host[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)],
                                threads=8)
        ok = _same(chunks, ref) and bool((counts == rc).all())
        return {"files": nfiles, "bytes": n, "median_file_bytes": int(np.median(sizes)),
                "ms_per_step": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2),
                "files_per_s": round(nfiles / dt, 1), "chunks": int(total), "parity_ok": bool(ok),
                "data": "synthetic log-normal size mix (median 8 KiB), uniform-random bytes"}
    finally:
        ctx.device_free(d_out)
        ctx.device_free(arena)


def chunk_ids(ctx, p, dp: int, n: int, d_out: int, count: int, steps: int, cpu_sample_gib: float,
              no_cpu: bool) -> dict:
    """BLAKE3 of every chunk of the headline boundary list (device in, device out),
    timed per step; then chunk + IDs back to back.  Parity probe: the IDs of the
    chunks inside the first GiB against the oracle."""
    d_ids = ctx.device_alloc(32 * count)
    try:
        dt, _ = _timed(lambda: ctx.chunk_ids(dp, n, (d_out, count), ids=d_ids), steps, 1)
        ids_ms = ctx.timing()["ids_ms"]
        cap = n // (p.min_size - 1) + 2

        def both():
            k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
            ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)
        dt2, _ = _timed(both, steps, 1)
        from oracle import oracle as O
        probe_bytes = 1 << 30
        chunks = ctx.d2h_chunks(d_out, count)
        sel = chunks[chunks["offset"] + chunks["length"] <= probe_bytes]
        host = O.random_bytes(probe_bytes, SEED)
        got = ctx.d2h_bytes(d_ids, 32 * len(sel)).reshape(len(sel), 32)
        ok = bool(len(sel) > 0 and (got == O.chunk_ids(host, sel, threads=16)).all())
        # VALU roofline: 672 lane-ops per 64-byte block (7 rounds x 8 G x 12 ops)
        # are the algorithmic work; peak = this mix's own issue rate on the whole
        # chip, wall clock (tools/ubench3.hip: the product's compression in
        # registers, 4 waves per SIMD on every CU: 1.68 ns per wave64
        # instruction per SIMD -- 2.4 cycles at the ~1.45 GHz the chip holds
        # under this load) x 256 CUs x 4 SIMDs x 64 lanes.
        alg_ops = n / 64 * 672
        peak_tops = 256 * 4 * 64 / 1.68e-9 / 1e12
        r = {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2), "device_ms": round(ids_ms, 3),
             "bound": "valu (32-bit add/xor/rotate of the BLAKE3 compression, ~11 ops per byte)",
             "roofline": {"bound": "valu", "achieved": round(alg_ops / (ids_ms * 1e-3) / 1e12, 2),
                          "peak": round(peak_tops, 2), "unit": "T int32 lane-ops/s",
                          "frac": round(alg_ops / (ids_ms * 1e-3) / 1e12 / peak_tops, 4),
                          "ops_per_block": 672,
                          "note": "algorithmic compression ops only (leaves; parents add ~1/16); peak: "
                                  "tools/ubench3.hip, the compression alone at full occupancy, wall clock"},
             "chunk_plus_ids_ms": round(dt2 * 1e3, 3), "chunk_plus_ids_gib_s": round(n / dt2 / GIB, 2),
             "parity_probe_chunks": int(len(sel)), "parity_probe_ok": ok}
        if not no_cpu:
            m = int(cpu_sample_gib * GIB)
            sample = chunks[chunks["offset"] + chunks["length"] <= m]
            hs = host if m == probe_bytes else O.random_bytes(m, SEED)
            t0 = time.perf_counter()
            O.chunk_ids(hs, sample, threads=1)
            cdt = time.perf_counter() - t0
            r["cpu_baseline"] = {"value": round(int(sample["length"].sum()) / cdt / GIB, 3), "unit": "GiB/s",
                                 "cores": 1, "kind": "port",
                                 "sample": f"chunks of the first {cpu_sample_gib:g} GiB, oracle/blake3_oracle.c "
                                           f"(portable scalar C, no SIMD), 1 thread"}
        return r
    finally:
        ctx.device_free(d_ids)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=64.0, help="bytes per GPU (GiB)")
    ap.add_argument("--cpu-sample-gib", type=float, default=16.0)
    ap.add_argument("--e2e-gib", type=float, default=8.0)
    ap.add_argument("--batch-files", type=int, default=10000, help="configs[2] file count (0: skip)")
    ap.add_argument("--small-files", type=int, default=80000, help="configs[3] file count (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="threads of the files-in-parallel CPU baseline "
                    "(16: this pool's CPU share per GPU)")
    ap.add_argument("--cpu-batch-files", type=int, default=4096, help="files in the multi-thread CPU sample")
    ap.add_argument("--no-ids", action="store_true", help="skip the chunk-ID (BLAKE3) stage")
    a = ap.parse_args()

    world, rank, local = _dist()
    if world != a.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {a.gpus}", file=sys.stderr)
    # Rehearsal only (a 1-GPU box standing in for a node): every rank on
    # device 0, barriers and the max-over-ranks reduction over gloo.
    rehearse = os.environ.get("MCDC_BENCH_ONE_DEVICE") == "1"
    if rehearse:
        local = 0
    numa_node = _bind_near_gpu(local)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if rehearse else "nccl", init_method="env://")

    from mapache_amd import _lib
    p = _lib.params(*PARAMS)
    n = int(a.gib * GIB)
    extras = rank == 0 and world == 1
    max_bytes = max(n, a.batch_files * (8 << 20) if extras else 0)
    ctx = _lib.Context(local, max_bytes)
    # Allocation order matters on this device heap: memory that a freed
    # multi-GiB buffer occupied is slower afterwards (tools/e2e_probe.py: a DMA
    # into it runs at 33 instead of 57.6 GB/s).  So the headline runs first on
    # a fresh heap, and the e2e host leg takes fresh memory of its own before
    # the 64 GiB buffers are freed.
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, SEED ^ rank)  # rank 0 uses SEED itself
    cap = n // (p.min_size - 1) + 2
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(a.warmup):
        ctx.chunk_device_to_device(p, dp, n, d_out, cap)
    scan_ms, dev_ms, total_ms = [], [], []
    barrier()
    t0 = time.perf_counter()
    count = 0
    for _ in range(a.steps):
        count = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
        t = ctx.timing()
        scan_ms.append(t["scan_ms"])
        dev_ms.append(t["device_ms"])
        total_ms.append(t["total_ms"])
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    n_gpus = world if world > 1 else 1
    total_bytes = n_gpus * n * a.steps
    value = total_bytes / elapsed / GIB
    scan_avg = float(np.mean(scan_ms))
    achieved = n / (scan_avg * 1e-3) / 1e9
    tpb, tsrc = _pmc_traffic()
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": n_gpus, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"one {a.gib:g} GiB uniform-random buffer per GPU, device-resident in and out "
                               f"(BASELINE configs[1])", "params": "FastCDC v2020 16/64/256 KiB Level1",
                   "bytes_per_gpu": n, "chunks_per_step": int(count),
                   "parallelism": f"{n_gpus} independent streams, no collectives",
                   "host_numa_node": numa_node},
        "roofline": {"bound": "hbm", "kernel": "k_scan_q", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": int(round(tpb * n)) if tpb else None, "traffic_unit": "bytes per launch",
                     "traffic_source": tsrc, "bytes_per_launch": n, "avg_launch_ms": round(scan_avg, 3)},
        "device_only": {"scan_ms": round(scan_avg, 3), "device_ms": round(float(np.mean(dev_ms)), 3),
                        "gib_s": round(n / (float(np.mean(dev_ms)) * 1e-3) / GIB, 2),
                        "call_ms": round(float(np.mean(total_ms)), 3)},
    }
    chunks = ctx.d2h_chunks(d_out, count)
    if extras:
        # same step, boundary list to pinned host memory (crosses PCIe inside the call)
        out = ctx.pinned_out(cap)
        dt, hc = _timed(lambda: ctx.chunk_device(p, dp, n, out=out), max(3, a.steps // 2), 1)
        result["host_out"] = {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2),
                              "identical_to_device_out": _same(hc, chunks),
                              "output": "pinned host array (hipHostMalloc), written by k_emit over PCIe"}
        if not a.no_ids:
            try:
                result["chunk_ids"] = chunk_ids(ctx, p, dp, n, d_out, int(count), 3, 1.0, a.no_cpu)
            except Exception as e:  # reported, never silently dropped
                result["chunk_ids"] = {"error": f"{type(e).__name__}: {e}"}
        if a.e2e_gib > 0:
            try:
                result["e2e_host"] = e2e_host(ctx, p, a.e2e_gib)
            except Exception as e:  # reported, never silently dropped
                result["e2e_host"] = {"error": f"{type(e).__name__}: {e}"}
    if extras:
        # (after the chunk-ID stage, which reads the headline's list in d_out)
        # mapache's own defaults (src/global/defaults.rs:35-40), same buffer
        p512 = _lib.params(512 << 10, 1 << 20, 8 << 20, 1)
        cap512 = n // ((512 << 10) - 1) + 2
        dt5, c5 = _timed(lambda: ctx.chunk_device_to_device(p512, dp, n, d_out, cap512), max(3, a.steps // 2), 1)
        t5 = ctx.timing()
        from oracle import oracle as O
        probe = 1 << 30  # parity probe: chunks that end before the first GiB's last max-window
        g5 = ctx.d2h_chunks(d_out, c5)
        g5 = g5[g5["offset"] + (8 << 20) <= probe - (8 << 20)]
        r5 = O.chunk(O.Params(512 << 10, 1 << 20, 8 << 20, 1), O.random_bytes(probe, SEED))
        result["params_512k_1m_8m"] = {"ms_per_step": round(dt5 * 1e3, 3), "gib_s": round(n / dt5 / GIB, 2),
                                       "chunks": int(c5), "scan_ms": round(t5["scan_ms"], 3),
                                       "device_ms": round(t5["device_ms"], 3),
                                       "parity_probe_chunks": int(len(g5)),
                                       "parity_probe_ok": bool(len(g5) > 0 and _same(g5, r5[:len(g5)])),
                                       "note": "same 64 GiB buffer, device-resident in and out, mapache defaults"}
    ctx.device_free(d_out)
    ctx.device_free(dp)
    if extras:
        cpu_files = 0 if a.no_cpu else a.cpu_batch_files
        threads = max(1, min(a.cpu_threads, os.cpu_count() or 1))
        for key, fn in (("batch_files", lambda: batch_files(ctx, p, a.batch_files, 8 << 20, 3, cpu_files, threads)
                         if a.batch_files > 0 else None),
                        ("small_files", lambda: small_files(ctx, p, a.small_files, 5) if a.small_files > 0 else None)):
            try:
                result[key] = fn()
            except Exception as e:  # reported, never silently dropped
                result[key] = {"error": f"{type(e).__name__}: {e}"}
        if not a.no_cpu:
            result["cpu_baseline"] = cpu_baseline(a.cpu_sample_gib, chunks)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
