#!/usr/bin/env python3
"""bench.py — device-resident GiB/s chunked, FastCDC 16/64/256 KiB L1, MI355X.

Workload (BASELINE.json configs[1]): per GPU one 64 GiB uniform-random byte
buffer resident in HBM (counter-based PRNG generated on the device, seed per
rank), FastCDC v2020 at min/avg/max = 16/64/256 KiB, Normalization::Level1.
A step = one full chunking pass over that buffer through the C ABI
(mcdc_chunk_device: scan + chain resolution + boundary emission + boundary
list copied to host).  N GPUs = N independent streams (weak scaling, no
collectives on the data path; torch.distributed is used only for the barrier
and the max-over-ranks timing).

Prints ONE JSON line (rank 0).  Extra objects:
  roofline     - the scan kernel (dominant) vs HBM peak: algorithmic bytes per
                 launch (1 byte read per input byte) / average launch time from
                 HIP events recorded on the library's stream.
  cpu_baseline - oracle/ C restatement of the crate, 1 thread, bounded sample
                 of the same stream (rank 0, N=1 only).
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


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(sample_gib: float, gpu_chunks: np.ndarray) -> dict:
    """Oracle (C restatement of fastcdc v2020), single thread, on the first
    `sample_gib` GiB of rank 0's stream.  Also cross-checks the GPU boundaries
    that lie wholly inside the sample (a size-independent parity probe)."""
    from oracle import oracle as O
    n = int(sample_gib * (1 << 30))
    d = O.random_bytes(n, SEED)  # generation is not timed
    t0 = time.perf_counter()
    c = O.chunk(O.Params(*PARAMS), d)
    dt = time.perf_counter() - t0
    # GPU chunks that end before the sample's last max-window are final in both
    lim = n - PARAMS[2]
    g = gpu_chunks[gpu_chunks["offset"] + PARAMS[2] <= lim]
    r = c[: len(g)]
    ok = bool(len(g) > 0 and (g["offset"] == r["offset"]).all() and (g["length"] == r["length"]).all()
              and (g["hash"] == r["hash"]).all())
    return {"value": round(n / dt / (1 << 30), 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {sample_gib:g} GiB of the rank-0 stream (seed 0x{SEED:x}), 16/64/256 KiB L1, "
                      f"oracle/fastcdc_oracle.c cut_gear loop, 1 thread, input pre-generated in RAM",
            "cpu": _cpu_model(), "seconds": round(dt, 3), "parity_probe_chunks": int(len(g)),
            "parity_probe_ok": ok}


def e2e_host(ctx, p, gib: float) -> dict:
    """End-to-end host path: pinned host buffer -> H2D -> kernels -> boundaries to host."""
    import ctypes
    from mapache_amd import _lib
    n = int(gib * (1 << 30))
    hp = ctx.host_alloc(n)
    dp = ctx.device_alloc(n)
    try:
        ctx.fill_random(dp, n, SEED ^ 0x55)
        _copy_d2h(dp, hp, n)  # synthetic bytes into pinned host memory (untimed)
        lib = _lib.load()
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
        return {"bytes": n, "gib_s": round(n / best / (1 << 30), 2), "h2d_ms": round(bt["h2d_ms"], 3),
                "device_ms": round(bt["device_ms"], 3), "d2h_ms": round(bt["d2h_ms"], 3),
                "total_ms": round(bt["total_ms"], 3), "source": "pinned host buffer (hipHostMalloc)"}
    finally:
        ctx.host_free(hp)
        ctx.device_free(dp)


def _copy_d2h(dp: int, hp: int, n: int) -> None:
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rc = hip.hipMemcpy(ctypes.c_void_p(hp), ctypes.c_void_p(dp), n, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError(f"hipMemcpy D2H failed: {rc}")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=64.0, help="bytes per GPU (GiB)")
    ap.add_argument("--cpu-sample-gib", type=float, default=16.0)
    ap.add_argument("--e2e-gib", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()

    world, rank, local = _dist()
    if world != a.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {a.gpus}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")

    from mapache_amd import _lib
    p = _lib.params(*PARAMS)
    n = int(a.gib * (1 << 30))
    ctx = _lib.Context(local, n)
    dp = ctx.device_alloc(n)
    ctx.fill_random(dp, n, SEED ^ rank)  # rank 0 uses SEED itself

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    out = ctx.pinned_out(n // (p.min_size - 1) + 2)  # reused pinned boundary list
    for _ in range(a.warmup):
        ctx.chunk_device(p, dp, n, out=out)
    scan_ms, dev_ms, total_ms = [], [], []
    barrier()
    t0 = time.perf_counter()
    chunks = None
    for _ in range(a.steps):
        chunks = ctx.chunk_device(p, dp, n, out=out)
        t = ctx.timing()
        scan_ms.append(t["scan_ms"])
        dev_ms.append(t["device_ms"])
        total_ms.append(t["total_ms"])
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    n_gpus = world if world > 1 else 1
    total_bytes = n_gpus * n * a.steps
    value = total_bytes / elapsed / (1 << 30)
    scan_avg = float(np.mean(scan_ms))
    achieved = n / (scan_avg * 1e-3) / 1e9
    tpb, tsrc = _pmc_traffic()
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": n_gpus, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"one {a.gib:g} GiB uniform-random buffer per GPU, device-resident "
                               f"(BASELINE configs[1])", "params": "FastCDC v2020 16/64/256 KiB Level1",
                   "bytes_per_gpu": n, "chunks_per_step": int(len(chunks)),
                   "parallelism": f"{n_gpus} independent streams, no collectives"},
        "roofline": {"bound": "hbm", "kernel": "k_scan_q", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": int(round(tpb * n)) if tpb else None, "traffic_unit": "bytes per launch",
                     "traffic_source": tsrc, "bytes_per_launch": n, "avg_launch_ms": round(scan_avg, 3)},
        "device_only": {"scan_ms": round(scan_avg, 3), "device_ms": round(float(np.mean(dev_ms)), 3),
                        "gib_s": round(n / (float(np.mean(dev_ms)) * 1e-3) / (1 << 30), 2),
                        "call_ms": round(float(np.mean(total_ms)), 3)},
    }
    chunks = chunks.copy()
    if rank == 0 and n_gpus == 1:
        try:
            result["e2e_host"] = e2e_host(ctx, p, a.e2e_gib) if a.e2e_gib > 0 else None
        except Exception as e:  # reported, never silently dropped
            result["e2e_host"] = {"error": str(e)}
        if not a.no_cpu:
            result["cpu_baseline"] = cpu_baseline(a.cpu_sample_gib, chunks)
    ctx.device_free(dp)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
