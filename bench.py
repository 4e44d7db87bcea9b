#!/usr/bin/env python3
"""bench.py — device-resident GiB/s chunked, FastCDC 16/64/256 KiB L1, MI355X.

Workload (BASELINE.json configs[1]): per GPU 64 GiB of one uniform-random
byte stream resident in HBM (counter-based PRNG generated on the device),
FastCDC v2020 at min/avg/max = 16/64/256 KiB, Normalization::Level1.  A step =
one full chunking pass over the stream through the C ABI (mcdc_chunk_device:
scan + chain resolution + boundary emission), boundary list written to a
device-resident array (the next pipeline stage consumes it in HBM).

N GPUs (one process per GPU, torchrun): ONE stream of N x 64 GiB split across
the GPUs (weak scaling: 64 GiB per GPU) — mapache_amd.shard.split_stream: each
rank chunks its slice plus a max-byte right halo, the ranks exchange their exit
positions (one int64 each, gloo all_gather) and each continues the previous
rank's exit until it meets its own chain.  At N = 1 that is exactly configs[1].

Prints ONE JSON line (rank 0).  Extra objects:
  roofline        - the scan kernel (dominant) vs HBM peak: algorithmic bytes per
                    launch (1 byte read per input byte) / average launch time from
                    HIP events recorded on the library's stream.
  cpu_baseline    - oracle/ C restatement of the crate, 1 thread, median of 5
                    runs on a bounded sample of the same stream (rank 0, N=1).
  corpus_sharded  - BASELINE configs[4]: a corpus of N x 8192 files of 8 MiB
                    sharded by file across the GPUs (shard.assign_files), one
                    batched device call per rank per step; every N.
  host_out        - same step, boundary list to pinned host memory (PCIe-inclusive)
  e2e_host        - pinned host input -> H2D -> kernels -> boundaries to host
  e2e_pageable    - pageable host input (the Archiver's Vec<u8>), staged
  batch_files     - BASELINE configs[2]: 10 000 independent 8 MiB files, one call
  small_files     - BASELINE configs[3] size mix (80 000 log-normal files) of random bytes, chunker only
  kernel_tree     - BASELINE configs[3] stand-in through the composed save path (mcdc_save_files at
                    512K/1M/8M, gate, IDs, dedup, encode, packs): C-like text, ~10 % duplicate files
  chunk_ids       - SURVEY.md §8(f) next stage: BLAKE3 chunk IDs of the same 64 GiB
                    boundary list in HBM (ID::from_content, processor.rs:184), and
                    the chunk + ID pipeline
  encode          - SecureStorage::encode / decode of host blobs: zstd on host threads +
                    sealing on the GPU (1 GiB of synthetic text)
  seal            - SURVEY.md §8(f) rank 3: SecureStorage encryption (AES-256-GCM-SIV,
                    storage.rs:97-118) of every chunk of the same stream as a blob
                    (mcdc_seal_device), its inverse (mcdc_open_device), parity probe
                    vs the oracle, CPU references
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


def _newest_profile(name: str):
    """(parsed JSON, relative path) of profiles/rNN[/part]/<name> of the newest round, or (None, None)."""
    import glob
    import re
    cands = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", name)) + \
            glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "*", name)):
        rel = os.path.relpath(path, ROOT)
        m = re.match(r"profiles/r(\d+)/", rel)
        if m:
            cands.append((int(m.group(1)), rel.count("/") == 2, rel))
    for _, _, rel in sorted(cands, reverse=True):
        try:
            with open(os.path.join(ROOT, rel)) as f:
                return json.load(f), rel
        except (OSError, ValueError):
            continue
    return None, None


def _pmc_traffic():
    """Calibrated PMC read traffic of the scan (profiles/rNN/pmc_traffic.json, written from
    separate rocprofv3 --pmc FETCH_SIZE passes by tools/profile_round.sh): HBM bytes per input byte.
    The newest round's file wins (a round's top level before its part directories)."""
    import glob
    import re
    cands = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "pmc_traffic.json")) + \
            glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "*", "pmc_traffic.json")):
        rel = os.path.relpath(path, ROOT)
        m = re.match(r"profiles/r(\d+)/", rel)
        if m:
            cands.append((int(m.group(1)), rel.count("/") == 2, rel))
    for _, _, rel in sorted(cands, reverse=True):
        try:
            with open(os.path.join(ROOT, rel)) as f:
                d = json.load(f)
            return float(d["traffic_per_input_byte"]), rel
        except (OSError, KeyError, ValueError):
            continue
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


class ClockSampler:
    """The engine clock the GPU holds during a timed region: a thread reads
    the amdgpu driver's current SCLK (the starred level of
    /sys/class/drm/cardN/device/pp_dpm_sclk; the card whose PCI address is
    this process's HIP device) every `period_s` while the region runs.  Read
    only, no GPU context: a box whose clock sags under load is told apart from
    a slow kernel by this number beside the roofline fraction."""

    def __init__(self, device: int, period_s: float = 0.002):
        import threading
        self.period, self.samples, self.path, self.why = period_s, [], None, None
        self._stop = threading.Event()
        self._t = None
        try:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            buf = ctypes.create_string_buffer(64)
            if hip.hipDeviceGetPCIBusId(buf, 64, int(device)) != 0:
                raise OSError("hipDeviceGetPCIBusId failed")
            bus = buf.value.decode().lower()
            for card in sorted(os.listdir("/sys/class/drm")):
                dev = os.path.join("/sys/class/drm", card, "device")
                f = os.path.join(dev, "pp_dpm_sclk")
                if card.startswith("card") and os.path.exists(f) and \
                        os.path.basename(os.path.realpath(dev)).lower().endswith(bus[-7:]):
                    self.path = f
                    break
            if self.path is None:
                self.why = f"no pp_dpm_sclk for PCI {bus}"
        except Exception as ex:  # reported, never fatal
            self.why = f"{type(ex).__name__}: {ex}"

    def _read(self):
        with open(self.path) as f:
            for line in f:
                if line.rstrip().endswith("*"):
                    return int(line.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz"))
        return None

    def _run(self):
        while not self._stop.is_set():
            try:
                v = self._read()
                if v:
                    self.samples.append(v)
            except Exception:
                pass
            self._stop.wait(self.period)

    def __enter__(self):
        import threading
        if self.path:
            self._t = threading.Thread(target=self._run, daemon=True)
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t:
            self._t.join()

    def summary(self) -> dict:
        if not self.samples:
            return {"sclk_mhz": None, "why": self.why or "no samples"}
        v = np.array(self.samples, np.float64)
        return {"sclk_mhz_mean": round(float(v.mean()), 1), "sclk_mhz_min": int(v.min()), "sclk_mhz_max": int(v.max()),
                "samples": int(v.size), "source": f"{self.path}, the starred level every "
                                                  f"{self.period * 1e3:g} ms over the timed region"}


def _cpus():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(sample_gib: float, gpu_chunks: np.ndarray, runs: int = 5) -> dict:
    """Oracle (C restatement of fastcdc v2020), single thread, median of `runs`
    timed runs on the first `sample_gib` GiB of rank 0's stream (pre-generated,
    pre-faulted).  Also cross-checks the GPU boundaries that lie wholly inside
    the sample (a size-independent parity probe)."""
    from oracle import oracle as O
    n = int(sample_gib * GIB)
    d = O.random_bytes(n, SEED)  # generation is not timed
    times, c = [], None
    for _ in range(runs):
        t0 = time.perf_counter()
        c = O.chunk(O.Params(*PARAMS), d)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    # GPU chunks that end before the sample's last max-window are final in both
    lim = n - PARAMS[2]
    g = gpu_chunks[gpu_chunks["offset"] + PARAMS[2] <= lim]
    ok = len(g) > 0 and _same(g, c[: len(g)])
    return {"value": round(n / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {sample_gib:g} GiB of the rank-0 stream (seed 0x{SEED:x}), 16/64/256 KiB L1, "
                      f"oracle/fastcdc_oracle.c cut_gear loop, 1 thread, input pre-generated in RAM, "
                      f"median of {runs} runs",
            "runs_s": [round(t, 3) for t in times], "cpu": _cpu_model(), "nproc": os.cpu_count(),
            "cpus_usable": _cpus(), "seconds": round(dt, 3), "parity_probe_chunks": int(len(g)),
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


def e2e_pageable(ctx, p, gib: float) -> dict:
    """End-to-end from PAGEABLE host memory, the Archiver adapter's real input:
    tests/cpp/test_host_api bench_stream (C++, its own process and contexts):
    one mcdc_chunk_host over the whole buffer (pinned staging slabs filled by
    the copy pool while the previous slab's DMA runs), and the windowed
    StreamCDC mirror (256 MiB windows, each chunk's bytes copied out as the
    crate's ChunkData.data)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "test_host_api")
    r = subprocess.run([exe, "bench_stream", str(gib)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": (r.stdout + r.stderr)[-500:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d["source"] = "pageable std::vector (C++ host mirror), 16/64/256 KiB"
    return d


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
    arena = ctx.device_alloc(n + 64)
    cap = int(sum(int(s) // (p.min_size - 1) + 2 for s in sizes))
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        ctx.fill_random(arena, n, SEED ^ 0x5F)
        # every call a new layout (offsets alternately +0 / +16 bytes): the
        # segment plan and the scan's run list rebuilt per call (timed first;
        # the repeated layout below is the line's number)
        fresh = []
        for c in range(steps + 2):
            t0 = time.perf_counter()
            ctx.chunk_batch_device_to_device(p, arena, offs + np.uint64(16 * (c % 2)), sizes, d_out, cap)
            fresh.append(time.perf_counter() - t0)
        fresh_ms = float(np.median(fresh[2:])) * 1e3
        # (two warm-up calls: the first plans the layout, the second builds its run list)
        dt, (total, counts) = _timed(lambda: ctx.chunk_batch_device_to_device(p, arena, offs, sizes, d_out, cap),
                                     steps, 2)
        from oracle import oracle as O
        chunks = ctx.d2h_chunks(d_out, total)
        host = O.random_bytes(n, SEED ^ 0x5F)
        ref, rc = O.chunk_files(O.Params(*PARAMS), [host[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)],
                                threads=8)
        ok = _same(chunks, ref) and bool((counts == rc).all())
        return {"files": nfiles, "bytes": n, "median_file_bytes": int(np.median(sizes)),
                "ms_per_step": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2),
                "files_per_s": round(nfiles / dt, 1), "chunks": int(total), "parity_ok": bool(ok),
                "fresh_layout_ms": round(fresh_ms, 3), "fresh_layout_gib_s": round(n / (fresh_ms * 1e-3) / GIB, 2),
                "note": "ms_per_step: the same layout every call (the segment plan and the list-mode scan's run "
                        "list kept from the previous call, DESIGN.md §5 'List-mode scan'); fresh_layout_ms: a new "
                        "layout every call (median)",
                "data": "synthetic log-normal size mix (median 8 KiB), uniform-random bytes"}
    finally:
        ctx.device_free(d_out)
        ctx.device_free(arena)


def kernel_tree(ctx, nfiles: int, steps: int) -> dict:
    """BASELINE configs[3] ("extracted Linux kernel source tree, ~80 k small
    files, dedup-heavy realistic mix") through the composed save path
    (mcdc_save_files) at mapache's own 512K/1M/8M with the 512 KiB size gate:
    most files take processor::save_file's whole-file branch
    (/root/reference/src/archiver/processor.rs:144-153), the rest are chunked
    (:160-205); IDs, the dedup index (repository_v1.rs:169-180), SecureStorage
    encode with a key, packs.  Stand-in corpus (tests/corpora.kernel_tree: no
    tree here or on the box): log-normal sizes, median 8 KiB, C-like text, ~10 %
    duplicate files.  Device input, fresh index per call, packs D2H into a
    reused pinned buffer; host_zstd (level 3 on host threads) vs gpu_compress.
    Also the chunker alone over the same files (BASELINE's 16/64/256 KiB, no
    gate: configs[3]'s chunking metric on text-like files)."""
    from mapache_amd import _lib
    from tests import corpora
    from oracle import oracle as O
    data, offs, lens, dup = corpora.kernel_tree(nfiles)
    n = int(data.size)
    p512 = _lib.params(512 << 10, 1 << 20, 8 << 20, 1)
    key = bytes(range(32))
    rng = np.random.default_rng(9)
    nonces = rng.integers(0, 256, (nfiles + n // (512 << 10) + 64, 12), dtype=np.uint8)
    hn, pad = rng.integers(0, 256, (4096, 12), dtype=np.uint8), rng.integers(0, 256, (4096 * 63, 36), dtype=np.uint8)
    dp = ctx.device_alloc(n + 16)
    ob = ctx.pinned_bytes(int(n * 1.01) + 4096 * nfiles + (1 << 16))
    out = {"files": nfiles, "bytes": n, "median_file_bytes": int(np.median(lens)), "duplicate_files": int((dup >= 0).sum()),
           "files_at_or_above_gate": int((lens >= (512 << 10)).sum())}
    try:
        ctx.h2d(dp, data)
        p16 = _lib.params(*PARAMS)
        cap = int(sum(int(s) // (p16.min_size - 1) + 2 for s in lens))
        d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
        try:
            dt, (total, counts) = _timed(lambda: ctx.chunk_batch_device_to_device(p16, dp, offs, lens, d_out, cap),
                                         steps, 2)  # (as small_files: plan, then run list)
            g = ctx.d2h_chunks(d_out, total)
            pick = np.arange(0, nfiles, 997)
            ends = np.cumsum(counts)
            ok = True
            for f in pick:  # sampled files against the oracle
                r = O.chunk(O.Params(*PARAMS), data[int(offs[f]):int(offs[f] + lens[f])])
                gf = g[int(ends[f] - counts[f]):int(ends[f])]
                ok &= _same(gf, r)
            out["chunk_only_p16"] = {"ms": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2),
                                     "files_per_s": round(nfiles / dt, 1), "chunks": int(total),
                                     "parity_probe_files": int(len(pick)), "parity_probe_ok": bool(ok)}
        finally:
            ctx.device_free(d_out)
        for mode in ("host_zstd", "gpu_compress"):
            def call():  # (the IDs as one array: the per-file split is Python work, not the call's)
                with ctx.index_create() as ix:
                    return ctx.save_files(p512, ix, dp, offs, lens, key, nonces, hn, pad, n=n,
                                          gpu_compress=mode == "gpu_compress", out_buf=ob, split=False)
            calls = []

            def timed_call():
                t0 = time.perf_counter()
                r = call()
                calls.append(time.perf_counter() - t0)
                return r
            dt, (ids, fb, new, packed, packs) = _timed(timed_call, steps, 1)
            calls = calls[1:]  # (the warm-up call out)
            t = ctx.timing()
            distinct = len({x.tobytes() for x in ids})
            body = packed[int(packs[0]["offset"]):int(packs[0]["offset"] + packs[0]["length"])].tobytes()
            hdr = O.parse_header(body, key)
            okd = all(O.blake3(np.frombuffer(O.storage_decode(body[o:o + ln], key, 16 << 20), np.uint8)) == b
                      for b, _, o, ln in hdr[:64])
            out[mode] = {"ms": round(dt * 1e3, 1), "gib_s": round(n / dt / GIB, 2), "files_per_s": round(nfiles / dt, 1),
                         "ms_calls": [round(x * 1e3, 1) for x in calls],
                         "ms_median": round(float(np.median(calls)) * 1e3, 1),
                         "blobs": int(new.size), "stored": int(new.sum()), "distinct_ids": distinct,
                         "packs": int(len(packs)), "packed_bytes": int(packed.size), "ratio": round(n / packed.size, 3),
                         "device_ms": round(t.get("device_ms", 0.0), 2), "decode_probe_ok": bool(okd and
                                                                                               int(new.sum()) == distinct)}
    finally:
        ctx.device_free(dp)
    out["note"] = ("mcdc_save_files from device memory at 512K/1M/8M (gate 512 KiB), key, fresh index per call, "
                   "packs D2H into a reused pinned buffer; ms: the mean of the timed calls (ms_calls: each; in this "
                   "process an occasional call waits 12-30 ms with its first kernels queued and the GPU idle, "
                   "DESIGN.md 0e item 2); decode probe: the first pack's first 64 blobs decoded "
                   "and BLAKE3-checked, stored == distinct IDs; full parity: tests/test_gpu_configs3.py")
    out["data"] = "synthetic kernel-tree stand-in (tests/corpora.kernel_tree)"
    return out


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
                          # nominal: 256 CUs x 128 int32 lanes per clock x 2.4 GHz
                          "peak_nominal": 78.64,
                          "frac_nominal": round(alg_ops / (ids_ms * 1e-3) / 1e12 / 78.64, 4),
                          "note": "algorithmic compression ops only (leaves; parents add ~1/16); peak: "
                                  "tools/ubench3.hip, the compression alone at full occupancy, wall clock "
                                  "(the clock the chip holds under this load); peak_nominal at the 2.4 GHz "
                                  "peak engine clock"},
             "chunk_plus_ids_ms": round(dt2 * 1e3, 3), "chunk_plus_ids_gib_s": round(n / dt2 / GIB, 2),
             "parity_probe_chunks": int(len(sel)), "parity_probe_ok": ok}
        pmc, src = _newest_profile("b3_pmc.json")  # counters of the same kernel (separate --pmc passes)
        if pmc and pmc.get("held_clock_ghz"):
            # VALU-issue floor at the clock the chip holds under this kernel: the
            # measured instructions per block at 100 % VALUBusy
            busy = pmc.get("valu_busy_pct") or None
            r["roofline"]["pmc"] = {"valu_busy_pct": busy, "held_clock_ghz": pmc["held_clock_ghz"],
                                    "valu_per_wave_block": pmc.get("valu_per_wave_block"),
                                    "floor_ms_at_held_clock": round(ids_ms * busy / 100, 3) if busy else None,
                                    "source": src}
        # dedup index (save_blob's index check, repository_v1.rs:169-180) over these IDs in HBM:
        # into an empty index (all new) and again into the populated one (all duplicates)
        try:
            k = ctx.chunk_device_to_device(p, dp, n, d_out, cap)
            ctx.chunk_ids(dp, n, (d_out, k), ids=d_ids)

            def fresh():
                with ctx.index_create() as ix:
                    f = ix.add(None, d_ids=d_ids, n=k)
                    return f, len(ix)
            dtf, (ff, size) = _timed(fresh, steps, 1)
            with ctx.index_create() as ix:
                ix.add(None, d_ids=d_ids, n=k)
                dtd, fd = _timed(lambda: ix.add(None, d_ids=d_ids, n=k), steps, 1)
            idh = ctx.d2h_bytes(d_ids, 32 * k).reshape(k, 32)
            t0 = time.perf_counter()
            ref = O.DedupIndex().add(idh)
            cdt = time.perf_counter() - t0
            r["dedup"] = {"ids": int(k), "new_ms_per_step": round(dtf * 1e3, 3),
                          "dup_ms_per_step": round(dtd * 1e3, 3), "new_ids_per_s": round(k / dtf),
                          "parity_ok": bool(ff.all() and size == k and not fd.any() and (ff == ref).all()),
                          "note": "mcdc_index_add of the headline's chunk IDs (device-resident): a fresh index "
                                  "per step (all new), then the same IDs into the populated index (all seen)",
                          "cpu_baseline": {"value": round(k / cdt), "unit": "IDs/s", "cores": 1, "kind": "port",
                                           "sample": "oracle.DedupIndex (Python set) over the same IDs"}}
        except Exception as ex:  # reported, never silently dropped
            r["dedup"] = {"error": f"{type(ex).__name__}: {ex}"}
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


def _openssl_gcm_gib_s(sample_bytes: int, runs: int = 3):
    """AES-256-GCM of one buffer with the system OpenSSL (AES-NI + carry-less
    multiply), 1 thread: a CPU proxy for the crate's AES-256-GCM-SIV, which costs
    the same two primitives (one AES-256 CTR pass, one GF(2^128) hash pass).
    None when libcrypto is absent."""
    import ctypes
    import ctypes.util
    name = ctypes.util.find_library("crypto")
    if not name:
        return None
    L = ctypes.CDLL(name)
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    L.EVP_CIPHER_CTX_new.restype = vp
    L.EVP_CIPHER_CTX_free.argtypes = [vp]
    L.EVP_aes_256_gcm.restype = vp
    L.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, vp, vp]
    L.EVP_EncryptUpdate.argtypes = [vp, vp, ip, vp, ctypes.c_int]
    L.EVP_EncryptFinal_ex.argtypes = [vp, vp, ip]
    src = np.frombuffer(np.random.default_rng(1).bytes(sample_bytes), np.uint8)
    dst = np.empty(sample_bytes + 64, np.uint8)
    key, iv = bytes(range(32)), bytes(12)
    best = []
    for _ in range(runs):
        c = L.EVP_CIPHER_CTX_new()
        n = ctypes.c_int()
        L.EVP_EncryptInit_ex(c, L.EVP_aes_256_gcm(), None, key, iv)
        t0 = time.perf_counter()
        for o in range(0, sample_bytes, 1 << 30):  # int-sized updates
            m = min(1 << 30, sample_bytes - o)
            L.EVP_EncryptUpdate(c, dst.ctypes.data + o, ctypes.byref(n), src.ctypes.data + o, m)
        L.EVP_EncryptFinal_ex(c, dst.ctypes.data + sample_bytes, ctypes.byref(n))
        best.append(time.perf_counter() - t0)
        L.EVP_CIPHER_CTX_free(c)
    return sample_bytes / float(np.median(best)) / GIB


def incremental(ctx, p, dp: int, n: int, d_ch: int, cap_c: int, d_ids: int, key: bytes, d_nonce: int,
                d_offs: int) -> dict:
    """A second snapshot of the stream with 1024 bytes changed, all in HBM: chunk
    -> IDs -> dedup against the index of the first snapshot (save_blob's check,
    repository_v1.rs:169-180) -> seal only the new chunks.  One timed pass (the
    index then holds the new IDs); the changed bytes are restored afterwards.
    Check: every chunk holding a changed byte is new, and few others are."""
    rng = np.random.default_rng(11)
    pos = np.unique(rng.integers(0, n, 1024))
    old = [ctx.d2h_bytes(dp + int(q), 1) for q in pos]
    with ctx.index_create() as ix:
        k0 = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
        ctx.chunk_ids(dp, n, (d_ch, k0), ids=d_ids)
        ix.add_device(d_ids, k0, d_ch, d_ch)  # (compacted in place: every chunk is new here)
        for q, b in zip(pos, old):
            ctx.h2d(dp + int(q), (b ^ 0x5A).astype(np.uint8))
        d_new = ctx.device_alloc(cap_c * 24)
        try:
            t0 = time.perf_counter()
            k1 = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
            t1 = time.perf_counter()
            ctx.chunk_ids(dp, n, (d_ch, k1), ids=d_ids)
            t2 = time.perf_counter()
            m = ix.add_device(d_ids, k1, d_ch, d_new)
            t3 = time.perf_counter()
            if m:  # (into a buffer of its own: d_seal still holds the full seal for the parity probe)
                cap_m = m * (p.max_size + 28)
                d_sm = ctx.device_alloc(cap_m)
                try:
                    t3 = time.perf_counter()
                    ctx.seal_chunks(key, dp, n, (d_new, m), d_nonce, d_sm, cap_m, offsets_out=d_offs)
                    t4 = time.perf_counter()
                finally:
                    ctx.device_free(d_sm)
            else:
                t4 = time.perf_counter()
            allc = ctx.d2h_chunks(d_ch, k1)
            newc = ctx.d2h_chunks(d_new, m)
        finally:
            ctx.device_free(d_new)
            for q, b in zip(pos, old):
                ctx.h2d(dp + int(q), b)
    holder = np.searchsorted(allc["offset"], pos, side="right") - 1
    must = np.unique(allc["offset"][holder])
    ok = bool(np.isin(must, newc["offset"]).all() and m <= 4 * len(pos))
    return {"changed_bytes": int(len(pos)), "chunks": int(k1), "new_chunks": int(m),
            "ms": round((t4 - t0) * 1e3, 3), "gib_s": round(n / (t4 - t0) / GIB, 2),
            "chunk_ms": round((t1 - t0) * 1e3, 3), "ids_ms": round((t2 - t1) * 1e3, 3),
            "dedup_ms": round((t3 - t2) * 1e3, 3), "seal_new_ms": round((t4 - t3) * 1e3, 3),
            "check_ok": ok,
            "note": "one pass, wall clock per stage (each call synchronises); index seeded with the first "
                    "snapshot's IDs"}


def encode(ctx, gib: float, steps: int) -> dict:
    """SecureStorage::encode / decode (storage.rs:61-94) of the chunks of a
    compressible host buffer: zstd on host threads + AES-256-GCM-SIV on the GPU
    (mcdc_encode_blobs / mcdc_decode_blobs), PCIe both ways included.  Data:
    synthetic text (a 2 000-word vocabulary), chunked at 16/64/256 KiB."""
    from mapache_amd import _lib
    from oracle import oracle as O
    rng = np.random.default_rng(21)
    vocab = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 11, 2000)]
    base = b" ".join(vocab[i] for i in rng.integers(0, 2000, 12_000_000))[:64 << 20]
    n = int(gib * GIB) // len(base) * len(base)
    data = np.frombuffer(base * (n // len(base)), np.uint8)
    ch = ctx.chunk_host(_lib.params(*PARAMS), data)
    nz = np.zeros((len(ch), 12), np.uint8)
    nz[:, :4] = np.arange(len(ch), dtype=np.uint32).view(np.uint8).reshape(-1, 4)
    dte, (enc, oo) = _timed(lambda: ctx.encode_blobs(bytes(range(32)), data, ch["offset"], ch["length"], nz),
                            steps, 1)
    dtd, (dec, do, st) = _timed(lambda: ctx.decode_blobs(bytes(range(32)), enc, oo[:-1], np.diff(oo), n + 64),
                                steps, 1)
    ok = bool((st == 0).all() and dec.size == n and (dec == data).all())
    pick = rng.integers(0, len(ch), 8)  # sealed bytes open with the oracle
    ok_o = all(O.decrypt_with_key(bytes(range(32)), enc[int(oo[i]):int(oo[i + 1])].tobytes()) is not None
               for i in pick)
    gpu = gpu_encode_text(ctx, data, ch, nz, steps, rng)
    save = save_path_text(ctx, base, n, steps)
    return {"gpu_compress": gpu, "save_path": save,
            "bytes": n, "blobs": int(len(ch)), "sealed_bytes": int(oo[-1]), "ratio": round(n / int(oo[-1]), 3),
            "encode_ms": round(dte * 1e3, 2), "encode_gib_s": round(n / dte / GIB, 3),
            "decode_ms": round(dtd * 1e3, 2), "decode_gib_s": round(n / dtd / GIB, 3),
            "round_trip_ok": ok, "oracle_open_ok": ok_o,
            "note": "host bytes in and out: zstd level 3 / window 20 on up to 16 host threads (system libzstd), "
                    "sealing on the GPU, H2D and D2H included",
            "data": "synthetic text, 2 000-word vocabulary, 64 MiB pattern repeated (repeats lie beyond the "
                    "1 MiB window)"}


def save_path_text(ctx, base: bytes, n: int, steps: int) -> dict:
    """mcdc_save_files (the composed save path: size gate, chunk, IDs, dedup,
    encode, packs) over n bytes of text in 4 MiB files from device memory,
    with a key and a fresh index per call (every blob new), encode by host
    zstd level 3 vs the GPU compressor (store.gpu_compress).  Each 64 MiB
    copy of the text pattern is XOR-ed with its index so no copy dedups
    against another.  Wall clock of the call: packs come back to host memory."""
    from mapache_amd import _lib
    b = np.frombuffer(base, np.uint8)
    data = np.concatenate([b ^ np.uint8(k % 31 + 1) for k in range(n // b.size)])
    fsz = 4 << 20
    offs = np.arange(0, n, fsz, dtype=np.uint64)
    lens = np.minimum(fsz, n - offs).astype(np.uint64)
    p = _lib.params(*PARAMS)
    key = bytes(range(32))
    rng = np.random.default_rng(5)
    nonces = rng.integers(0, 256, (n // (PARAMS[0] - 1) + len(offs) + 2, 12), dtype=np.uint8)
    hn, pad = rng.integers(0, 256, (4096, 12), dtype=np.uint8), rng.integers(0, 256, (4096 * 63, 36), dtype=np.uint8)
    dp = ctx.device_alloc(n)
    ob = ctx.pinned_bytes(int(n * 1.01) + 4096 * len(offs) + (1 << 16))  # the packs' host buffer, reused
    out = {}
    try:
        ctx.h2d(dp, data)
        for mode in ("host_zstd", "gpu_compress"):
            def call():
                with ctx.index_create() as ix:
                    return ctx.save_files(p, ix, dp, offs, lens, key, nonces, hn, pad, n=n,
                                          gpu_compress=mode == "gpu_compress", out_buf=ob)
            dt, (ids, new, packed, packs) = _timed(call, steps, 1)
            out[mode] = {"ms": round(dt * 1e3, 1), "gib_s": round(n / dt / GIB, 2), "blobs": int(new.size),
                         "stored": int(new.sum()), "packs": int(len(packs)), "packed_bytes": int(packed.size),
                         "ratio": round(n / packed.size, 3)}
    finally:
        ctx.device_free(dp)
    out["note"] = ("mcdc_save_files from device memory, 4 MiB files of synthetic text, with a key; wall clock "
                   "incl. the packs' D2H into a reused pinned buffer; host_zstd: level 3 on host threads, packs "
                   "on the host; gpu_compress: compress, seal, pack assembly and pack IDs in HBM, one D2H "
                   "(decode-equal frames, tests/test_gpu_save.py)")
    return out


def gpu_encode_text(ctx, data: np.ndarray, ch: np.ndarray, nz: np.ndarray, steps: int, rng) -> dict:
    """SecureStorage::encode of the same text blobs with the compression on the
    GPU too (mcdc_zstd_compress_device, then mcdc_seal_device over the frames),
    device-resident in and out; the ratio beside the host level-3 one.  Parity:
    sampled sealed blobs opened by the oracle and decoded by libzstd."""
    from mapache_amd import _lib
    from oracle import oracle as O
    n = data.size
    key = bytes(range(32))
    cap = _lib.Context.zstd_compress_bound(ch["length"])
    dp, d_z = ctx.device_alloc(n), ctx.device_alloc(cap)
    d_ch, d_fr = ctx.device_alloc(24 * len(ch)), ctx.device_alloc(16 * len(ch))
    d_nz, d_seal = ctx.device_alloc(12 * len(ch)), ctx.device_alloc(cap + 28 * len(ch))
    d_off = ctx.device_alloc(8 * (len(ch) + 1))
    try:
        ctx.h2d(dp, data)
        ctx.h2d(d_ch, ch.view(np.uint8))
        ctx.h2d(d_nz, nz.reshape(-1))
        dtc, (_, zb) = _timed(lambda: ctx.zstd_compress(dp, n, (d_ch, len(ch)), d_z, cap, frames_out=d_fr), steps, 1)
        zdev = ctx.timing()["device_ms"]

        def enc():
            _, b = ctx.zstd_compress(dp, n, (d_ch, len(ch)), d_z, cap, frames_out=d_fr)
            ctx.seal_device_ext(key, d_z, b, d_fr, len(ch), d_nz, d_seal, cap + 28 * len(ch), d_off)
            return b
        dte, _ = _timed(enc, steps, 1)
        fr = ctx.d2h_bytes(d_fr, 16 * len(ch)).view(np.uint64).reshape(-1, 2)
        oo = ctx.d2h_bytes(d_off, 8 * (len(ch) + 1)).view(np.uint64)
        z = O.Zstd()
        ok = True
        for i in rng.integers(0, len(ch), 16):
            blob = ctx.d2h_bytes(d_seal + int(oo[i]), int(oo[i + 1] - oo[i])).tobytes()
            frame = O.decrypt_with_key(key, blob)
            src = data[int(ch["offset"][i]):int(ch["offset"][i] + ch["length"][i])].tobytes()
            ok &= frame is not None and z.decompress(frame, len(src) + 64) == src
        return {"compress_ms": round(dtc * 1e3, 3), "compress_gib_s": round(n / dtc / GIB, 2),
                "compress_device_ms": round(zdev, 3), "compressed_bytes": int(zb), "ratio": round(n / zb, 3),
                "encode_ms": round(dte * 1e3, 3), "encode_gib_s": round(n / dte / GIB, 2),
                "sealed_bytes": int(oo[-1]), "encode_ratio": round(n / int(oo[-1]), 3), "parity_probe_ok": bool(ok),
                "note": "mcdc_zstd_compress_device (greedy LZ, Huffman literals, FSE sequences with per-block or predefined tables, 32 KiB blocks) "
                        "+ mcdc_seal_device, all in HBM; ratio vs the host level-3 ratio of the same blobs above"}
    finally:
        for x in (d_off, d_seal, d_nz, d_fr, d_ch, d_z, dp):
            ctx.device_free(x)


def seal(ctx, dp: int, n: int, chunks: np.ndarray, steps: int, no_cpu: bool) -> dict:
    """Every chunk of the headline stream sealed as one blob (random data: zstd
    would store it raw, so the blobs stand in for the compressed chunks), device
    in, device out; then opened again.  Parity probe: 96 sealed blobs against
    the oracle; the round trip: every tag verifies and sampled windows of the
    opened stream equal the input."""
    from oracle import oracle as O
    from mapache_amd import _lib
    k = len(chunks)
    offs, lens = chunks["offset"], chunks["length"]
    key = bytes(range(0x40, 0x60))
    nonces = np.zeros((k, 3), np.uint32)  # nonce i = le32(i) || "mapache!"
    nonces[:, 0] = np.arange(k, dtype=np.uint32)
    nonces[:, 1:] = np.frombuffer(b"mapache!", np.uint32)
    nonces = nonces.view(np.uint8).reshape(k, 12)
    cap = n + 28 * k
    d_seal = ctx.device_alloc(cap + (64 << 20))  # (+ room for the store-mode frames' headers, below)
    d_open = ctx.device_alloc(n + (64 << 20))
    try:
        dt, oo = _timed(lambda: ctx.seal(key, dp, n, offs, lens, nonces, d_seal, cap), steps, 1)
        ts = ctx.timing()
        dto, (po, st) = _timed(lambda: ctx.open(key, d_seal, int(oo[-1]), oo[:-1], np.diff(oo), d_open, n), steps, 1)
        to = ctx.timing()
        # parity probe and round trip now (the store-mode path below reuses d_seal / d_open)
        rng = np.random.default_rng(3)
        pick = np.unique(np.concatenate([np.arange(32), rng.integers(0, k, 64)]))
        got = [ctx.d2h_bytes(d_seal + int(oo[i]), int(lens[i]) + 28).tobytes() for i in pick]
        ref = [O.encrypt_with_key(key, nonces[i], O.random_bytes(int(lens[i]), SEED, pos=int(offs[i]))) for i in pick]
        windows = [int(x) for x in rng.integers(0, n - (1 << 20), 16)]
        rt_ok = bool((st == 0).all()) and all(
            (ctx.d2h_bytes(d_open + w, 1 << 20) == O.random_bytes(1 << 20, SEED, pos=w)).all() for w in windows)
        # the save path's GPU stages back to back, all in HBM: chunk -> IDs -> seal
        p = _lib.params(*PARAMS)
        cap_c = n // (p.min_size - 1) + 2
        d_ch = ctx.device_alloc(cap_c * _lib.CHUNK_DTYPE.itemsize)
        d_ids = ctx.device_alloc(32 * cap_c)
        d_nonce = ctx.device_alloc(12 * k)
        d_offs = ctx.device_alloc(8 * (k + 1))
        try:
            ctx.h2d(d_nonce, nonces.reshape(-1))

            def save_path():
                kk = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
                ctx.chunk_ids(dp, n, (d_ch, kk), ids=d_ids)
                ctx.seal_chunks(key, dp, n, (d_ch, kk), d_nonce, d_seal, cap, offsets_out=d_offs)
            dtp, _ = _timed(save_path, steps, 1)  # (rewrites d_seal with the same bytes: same list, nonces, key)
            incr = incremental(ctx, p, dp, n, d_ch, cap_c, d_ids, key, d_nonce, d_offs)
            # the whole GPU encode in store mode: chunk -> IDs -> zstd raw frames -> seal,
            # every array in HBM (blobs mapache's decoder reads; no compression)
            d_fr = ctx.device_alloc(16 * cap_c)
            try:
                def store_path():
                    kk = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
                    ctx.chunk_ids(dp, n, (d_ch, kk), ids=d_ids)
                    _, span = ctx.zstd_frames(dp, n, (d_ch, kk), d_open, n + (64 << 20), frames_out=d_fr)
                    t_fr = ctx.timing()["device_ms"]
                    ctx.seal_device_ext(key, d_open, span, d_fr, kk, d_nonce, d_seal, cap + (64 << 20), d_offs)
                    return span, t_fr
                dts, (span_s, t_fr) = _timed(store_path, steps, 1)
                fr_probe = ctx.d2h_bytes(d_fr, 16 * 4).view(np.uint64).reshape(4, 2)
                probe_ok = all(ctx.d2h_bytes(d_open + int(fr_probe[i, 0]), int(fr_probe[i, 1])).tobytes()
                               == O.zstd_raw_frame(O.random_bytes(int(lens[i]), SEED, pos=int(offs[i])))
                               for i in range(4))
                store = {"ms_per_step": round(dts * 1e3, 3), "gib_s": round(n / dts / GIB, 2),
                         "frames_ms": round(t_fr, 3), "frame_bytes": int(span_s), "frames_probe_ok": probe_ok,
                         "note": "mcdc_chunk_device + mcdc_chunk_ids_device + mcdc_zstd_frames_device + "
                                 "mcdc_seal_device per step, all in HBM: zstd frames in raw-block mode"}

                # the same with real compression on the GPU (mcdc_zstd_compress_device)
                def comp_path():
                    kk = ctx.chunk_device_to_device(p, dp, n, d_ch, cap_c)
                    ctx.chunk_ids(dp, n, (d_ch, kk), ids=d_ids)
                    _, zb = ctx.zstd_compress(dp, n, (d_ch, kk), d_open, n + (64 << 20), frames_out=d_fr)
                    t_z = ctx.timing()["device_ms"]
                    ctx.seal_device_ext(key, d_open, zb, d_fr, kk, d_nonce, d_seal, cap + (64 << 20), d_offs)
                    return zb, t_z
                dtz, (zb, t_z) = _timed(comp_path, steps, 1)
                zf = ctx.d2h_bytes(d_fr, 16 * 4).view(np.uint64).reshape(4, 2)
                zok = all(O.Zstd().decompress(ctx.d2h_bytes(d_open + int(zf[i, 0]), int(zf[i, 1])).tobytes(),
                                              int(lens[i]) + 64)
                          == O.random_bytes(int(lens[i]), SEED, pos=int(offs[i])).tobytes() for i in range(4))
                store["compressed_encode_path"] = {
                    "ms_per_step": round(dtz * 1e3, 3), "gib_s": round(n / dtz / GIB, 2),
                    "compress_device_ms": round(t_z, 3), "compress_gib_s": round(n / (t_z * 1e-3) / GIB, 2),
                    "compressed_bytes": int(zb), "ratio": round(n / zb, 4), "decode_probe_ok": bool(zok),
                    "note": "chunk -> IDs -> mcdc_zstd_compress_device -> seal, all in HBM (random data: every "
                            "block falls back to raw, as zstd stores incompressible data)"}
            finally:
                ctx.device_free(d_fr)
        finally:
            for ptr in (d_offs, d_nonce, d_ids, d_ch):
                ctx.device_free(ptr)
        r = {"blobs": k, "bytes": n, "steps": steps,
             "seal_ms_per_step": round(dt * 1e3, 3), "seal_gib_s": round(n / dt / GIB, 2),
             "seal_device_ms": round(ts["device_ms"], 3), "seal_kernels_ms": round(ts["aead_ms"], 3),
             "open_ms_per_step": round(dto * 1e3, 3), "open_gib_s": round(n / dto / GIB, 2),
             "open_device_ms": round(to["device_ms"], 3),
             "chunk_ids_seal_ms_per_step": round(dtp * 1e3, 3), "chunk_ids_seal_gib_s": round(n / dtp / GIB, 2),
             "chunk_ids_seal": "mcdc_chunk_device + mcdc_chunk_ids_device + mcdc_seal_chunks_device per step, "
                               "boundary list, IDs, nonces and output offsets in HBM",
             "parity_probe_blobs": int(len(pick)), "parity_probe_ok": got == ref,
             "round_trip_ok": rt_ok, "incremental_save_path": incr, "store_mode_encode_path": store,
             "output": "nonce || ciphertext || tag per blob, packed in blob order (the pack body)",
             "data": "synthetic: the chunks of the 64 GiB headline stream as blobs, nonce i = le32(i) || 'mapache!'"}
        if not no_cpu:
            sample = chunks[:max(1, int(np.searchsorted(np.cumsum(lens), 32 << 20)))]
            host = O.random_bytes(int(sample["offset"][-1] + sample["length"][-1]), SEED)
            t0 = time.perf_counter()
            O.seal_blobs(key, host, sample["offset"], sample["length"], nonces[:len(sample)], threads=1)
            cdt = time.perf_counter() - t0
            r["cpu_baseline"] = {"value": round(int(sample["length"].sum()) / cdt / GIB, 4), "unit": "GiB/s",
                                 "cores": 1, "kind": "port",
                                 "sample": f"the first {len(sample)} blobs (~32 MiB), oracle/aead_oracle.c "
                                           f"(byte-oriented AES, bitwise POLYVAL: a restatement, not a fast CPU "
                                           f"implementation), 1 thread"}
            g = _openssl_gcm_gib_s(1 << 30)
            if g is not None:
                r["cpu_proxy_openssl_aes256gcm"] = {"value": round(g, 3), "unit": "GiB/s", "cores": 1,
                                                    "sample": "1 GiB, one AES-256-GCM message, system OpenSSL "
                                                              "(AES-NI/PCLMUL): the crate's per-core cost class"}
        return r
    finally:
        ctx.device_free(d_open)
        ctx.device_free(d_seal)


def corpus_sharded(ctx, p, files_per_gpu: int, file_bytes: int, steps: int, warmup: int, world: int, rank: int,
                   barrier, allreduce_max, gather, oracle_threads: int = 16) -> dict:
    """BASELINE configs[4]: a corpus of world x files_per_gpu files of file_bytes
    (file i = the counter-based stream of seed SEED ^ (i + 1)), assigned to
    ranks by shard.assign_files (no data exchange); each rank chunks its files
    with one mcdc_chunk_batch_device call per step over its own arena."""
    from mapache_amd import _lib, shard
    nfiles = world * files_per_gpu
    sizes = [file_bytes] * nfiles
    mine = shard.assign_files(sizes, world)[rank]
    offs = np.arange(len(mine), dtype=np.uint64) * np.uint64(file_bytes)
    lens = np.full(len(mine), file_bytes, dtype=np.uint64)
    nbytes = len(mine) * file_bytes
    arena = ctx.device_alloc(nbytes)
    cap = len(mine) * (file_bytes // (p.min_size - 1) + 2)
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    try:
        for k, i in enumerate(mine):
            ctx.fill_random(arena + k * file_bytes, file_bytes, SEED ^ (i + 1))
        run = lambda: ctx.chunk_batch_device_to_device(p, arena, offs, lens, d_out, cap)  # noqa: E731
        for _ in range(warmup):
            run()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            total, counts = run()
        barrier()
        mine_s = time.perf_counter() - t0
        elapsed = allreduce_max(mine_s)
        # gathered result: per-file counts and an order-sensitive digest of the
        # whole corpus's boundary lists (file order).  Parity (after timing):
        # every file of this rank against the oracle regenerating it on
        # `oracle_threads` host threads (oracle.random_files_digest), and the
        # gathered corpus digest against the fold of the oracle's digests.
        chunks = ctx.d2h_chunks(d_out, total)
        starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        per_file = [(i, int(counts[k]), _lib.digest(chunks[starts[k]:starts[k + 1]])) for k, i in enumerate(mine)]
        from oracle import oracle as O
        t0 = time.perf_counter()
        rc, rd, _ = O.random_files_digest(O.Params(*PARAMS), [SEED ^ (i + 1) for i in mine], 0,
                                          [file_bytes] * len(mine), threads=oracle_threads)
        oracle_s = time.perf_counter() - t0
        ref_file = [(i, int(rc[k]), int(rd[k])) for k, i in enumerate(mine)]
        parts = gather((per_file, ref_file, mine_s, oracle_s))
    finally:
        ctx.device_free(d_out)
        ctx.device_free(arena)
    if parts is None:
        return {}
    allf = sorted(x for part in parts for x in part[0])
    allr = sorted(x for part in parts for x in part[1])
    dig = shard.corpus_digest([c for _, c, _ in allf], [d for _, _, d in allf])
    rdig = shard.corpus_digest([c for _, c, _ in allr], [d for _, _, d in allr])
    bad = [i for (i, c, d), (_, rc_, rd_) in zip(allf, allr) if (c, d) != (rc_, rd_)]
    total_bytes = nfiles * file_bytes
    return {"files": nfiles, "file_bytes": file_bytes, "bytes": total_bytes, "steps": steps,
            "ms_per_step": round(elapsed / steps * 1e3, 3), "gib_s": round(total_bytes * steps / elapsed / GIB, 2),
            "per_rank_gib_s": [round(nbytes * steps / part[2] / GIB, 2) for part in parts],
            "chunks": int(sum(c for _, c, _ in allf)), "corpus_digest": f"{dig:016x}",
            "oracle_corpus_digest": f"{rdig:016x}",
            "parity_ok": bool(len(allf) == nfiles and [x[0] for x in allf] == list(range(nfiles))
                              and not bad and dig == rdig),
            "parity_files_checked": len(allr), "parity_bad_files": bad[:8],
            "oracle_seconds_per_rank": [round(part[3], 2) for part in parts],
            "parity": f"every file against oracle.random_files_digest ({oracle_threads} host threads per rank, "
                      f"after the timed steps); corpus digest = shard.corpus_digest",
            "assignment": "shard.assign_files (LPT by bytes; equal sizes -> round robin), no data exchange",
            "data": "synthetic uniform-random files (device PRNG, per-file seeds)"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=64.0, help="bytes per GPU (GiB)")
    ap.add_argument("--cpu-sample-gib", type=float, default=4.0)
    ap.add_argument("--cpu-runs", type=int, default=5)
    ap.add_argument("--e2e-gib", type=float, default=8.0)
    ap.add_argument("--batch-files", type=int, default=10000, help="configs[2] file count (0: skip)")
    ap.add_argument("--small-files", type=int, default=80000, help="configs[3] file count (0: skip)")
    ap.add_argument("--kernel-tree", type=int, default=80000,
                    help="configs[3] kernel-tree stand-in through the save path: file count (0: skip)")
    ap.add_argument("--corpus-files-per-gpu", type=int, default=8192, help="configs[4]: 8 MiB files per GPU (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="threads of the files-in-parallel CPU baseline "
                    "(16: this pool's CPU share per GPU)")
    ap.add_argument("--cpu-batch-files", type=int, default=4096, help="files in the multi-thread CPU sample")
    ap.add_argument("--no-ids", action="store_true", help="skip the chunk-ID (BLAKE3) stage")
    ap.add_argument("--no-seal", action="store_true", help="skip the SecureStorage sealing stage")
    ap.add_argument("--encode-gib", type=float, default=1.0, help="host encode/decode sample (GiB, 0: skip)")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the timed headline steps (warmup + steps calls of the 64 GiB stream): the command "
                         "whose rocprofv3 kernel trace is the roofline's evidence (profiles/rNN/headline_*)")
    ap.add_argument("--parity", action="store_true",
                    help="after timing, gather every rank's exact chunks of the split stream and compare the "
                         "whole list with the oracle's (small --gib; tests/test_gpu_multirank.py)")
    a = ap.parse_args()

    world, rank, local = _dist()
    if world != a.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {a.gpus}", file=sys.stderr)
    # One backend for every N: gloo carries the exit exchange (one int64 per
    # rank), the barriers and the gathers (no data-path
    # collective).  The process never touches torch.cuda: torch ships its own
    # HIP runtime, and libmcdc's is the only one initialised here.  The timed
    # region's device-side bracket is mcdc_ctx_synchronize.
    # Rehearsal (a 1-GPU box standing in for a node): every rank on device 0;
    # the code path is otherwise the one an 8-GPU node runs.
    rehearse = os.environ.get("MCDC_BENCH_ONE_DEVICE") == "1"
    if rehearse:
        local = 0
    numa_node = _bind_near_gpu(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")

    from mapache_amd import _lib, shard
    p = _lib.params(*PARAMS)
    n = int(a.gib * GIB)
    extras = rank == 0 and world == 1 and not a.headline_only
    if a.headline_only:
        a.corpus_files_per_gpu = 0
    corpus_bytes = a.corpus_files_per_gpu * (8 << 20)
    max_bytes = max(n + PARAMS[2], corpus_bytes, a.batch_files * (8 << 20) if extras else 0,
                    (2 << 30) if extras and a.kernel_tree else 0)  # (the kernel-tree arena: ~1.3 GB)
    ctx = _lib.Context(local, max_bytes)

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    def allreduce_max(x: float) -> float:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def gather(obj):
        if dist is None:
            return [obj]
        parts = [None] * world if rank == 0 else None
        dist.gather_object(obj, parts, dst=0)
        return parts

    # The stream: N x n bytes, rank r holds slice r plus a max-byte right halo.
    # Allocation order matters on this device heap: memory that a freed
    # multi-GiB buffer occupied is slower afterwards (tools/e2e_probe.py: a DMA
    # into it runs at 33 instead of 57.6 GB/s).  So the headline runs first on
    # a fresh heap, and the e2e host leg takes fresh memory of its own before
    # the 64 GiB buffers are freed.
    total = world * n
    s, e = shard.stream_slices(total, world)[rank] if world > 1 else (0, n)
    hi = min(e + PARAMS[2], total)
    dp = ctx.device_alloc(hi - s)
    ctx.fill_random(dp, hi - s, SEED, pos=s)  # the one stream (rank 0 at N = 1: configs[1])
    cap = (hi - s) // (p.min_size - 1) + 2
    d_out = ctx.device_alloc(cap * _lib.CHUNK_DTYPE.itemsize)
    allgather = shard.torch_allgather() if dist is not None else None
    split_stats = {}

    def step():
        k = ctx.chunk_device_to_device(p, dp, hi - s, d_out, cap)
        if world == 1:
            return k
        spec = shard.DeviceChunks(ctx, d_out, k, base=s, window=64)
        res, st = shard.split_stream(lambda x, y: ctx.chunk_device(p, dp + (x - s), y - x), allgather, s, e, total,
                                     PARAMS[2], rank, world, spec=spec, materialize=False)
        split_stats.update(st)
        split_stats["fixup_calls_total"] = split_stats.get("fixup_calls_total", 0) + st["fixup_calls"]
        return len(res)

    for _ in range(a.warmup):
        step()
    split_stats.clear()
    scan_ms, dev_ms, total_ms = [], [], []
    clock = ClockSampler(local)
    barrier()
    with clock:
        t0 = time.perf_counter()
        count = 0
        for _ in range(a.steps):
            count = step()
            t = ctx.timing() if world == 1 else None
            if t:
                scan_ms.append(t["scan_ms"])
                dev_ms.append(t["device_ms"])
                total_ms.append(t["total_ms"])
        barrier()
        elapsed = allreduce_max(time.perf_counter() - t0)
    if world > 1:  # the main call's device timings (outside the timed loop)
        ctx.chunk_device_to_device(p, dp, hi - s, d_out, cap)
        t = ctx.timing()
        scan_ms, dev_ms, total_ms = [t["scan_ms"]], [t["device_ms"]], [t["total_ms"]]

    n_gpus = world if world > 1 else 1
    total_bytes = n_gpus * n * a.steps
    value = total_bytes / elapsed / GIB
    scan_avg = float(np.mean(scan_ms))
    achieved = (hi - s) / (scan_avg * 1e-3) / 1e9
    tpb, tsrc = _pmc_traffic()
    counts = gather(int(count))
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": n_gpus, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": (f"one {a.gib:g} GiB uniform-random stream, device-resident in and out "
                                f"(BASELINE configs[1])" if world == 1 else
                                f"one {n_gpus * a.gib:g} GiB uniform-random stream split across {n_gpus} GPUs "
                                f"({a.gib:g} GiB per GPU + 256 KiB halo), device-resident in and out"),
                   "params": "FastCDC v2020 16/64/256 KiB Level1",
                   "bytes_per_gpu": n, "chunks_per_step": int(sum(counts)) if counts else int(count),
                   "parallelism": ("1 GPU" if world == 1 else
                                   f"{n_gpus} slices of one stream; exits exchanged (gloo all_gather, int64 per "
                                   f"rank, no data-path collective), seam continuations on the receiving GPU"),
                   "host_numa_node": numa_node},
        "roofline": {"bound": "hbm", "kernel": "k_scan_q", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": int(round(tpb * (hi - s))) if tpb else None, "traffic_unit": "bytes per launch",
                     "traffic_source": tsrc, "bytes_per_launch": hi - s, "avg_launch_ms": round(scan_avg, 3),
                     "clock": clock.summary()},
        "device_only": {"scan_ms": round(scan_avg, 3), "device_ms": round(float(np.mean(dev_ms)), 3),
                        "gib_s": round((hi - s) / (float(np.mean(dev_ms)) * 1e-3) / GIB, 2),
                        "call_ms": round(float(np.mean(total_ms)), 3)},
    }
    if a.parity:  # the whole stream's boundary list against the oracle (after timing)
        if world == 1:
            mine = ctx.d2h_chunks(d_out, ctx.chunk_device_to_device(p, dp, n, d_out, cap))
        else:
            spec = shard.DeviceChunks(ctx, d_out, ctx.chunk_device_to_device(p, dp, hi - s, d_out, cap), base=s)
            mine, _ = shard.split_stream(lambda x, y: ctx.chunk_device(p, dp + (x - s), y - x), allgather, s, e,
                                         total, PARAMS[2], rank, world, spec=spec)
        parts = gather(mine)
        if parts is not None:
            from oracle import oracle as O
            allc = np.concatenate(parts)
            rk, rdig, rsum = O.random_stream_digest(O.Params(*PARAMS), SEED, total)
            result["stream_parity"] = {"chunks": int(len(allc)), "oracle_chunks": int(rk),
                                       "digest": f"{_lib.digest(allc):016x}", "oracle_digest": f"{rdig:016x}",
                                       "ok": bool(len(allc) == rk and _lib.digest(allc) == rdig and rsum == total)}
    if world > 1:
        st = gather(dict(split_stats))
        if st:
            result["split_stream"] = {"rounds_max": max(x.get("rounds", 0) for x in st),
                                      "fixup_calls_per_step": round(sum(x.get("fixup_calls_total", 0) for x in st)
                                                                    / a.steps, 2),
                                      "merged_in_slice": all(x.get("merged", True) for x in st)}
    chunks = ctx.d2h_chunks(d_out, ctx.chunk_device_to_device(p, dp, hi - s, d_out, cap)) if extras else None
    if extras:
        # same step, boundary list to pinned host memory (crosses PCIe inside the call)
        out = ctx.pinned_out(cap)
        dt, hc = _timed(lambda: ctx.chunk_device(p, dp, n, out=out), max(3, a.steps // 2), 1)
        result["host_out"] = {"ms_per_step": round(dt * 1e3, 3), "gib_s": round(n / dt / GIB, 2),
                              "identical_to_device_out": _same(hc, chunks),
                              "output": "pinned host array (hipHostMalloc), written by k_emit over PCIe"}
        if not a.no_ids:
            try:
                result["chunk_ids"] = chunk_ids(ctx, p, dp, n, d_out, len(chunks), 3, 1.0, a.no_cpu)
            except Exception as ex:  # reported, never silently dropped
                result["chunk_ids"] = {"error": f"{type(ex).__name__}: {ex}"}
        if a.e2e_gib > 0:
            for key, fn in (("e2e_host", e2e_host), ("e2e_pageable", e2e_pageable)):
                try:
                    result[key] = fn(ctx, p, a.e2e_gib)
                except Exception as ex:  # reported, never silently dropped
                    result[key] = {"error": f"{type(ex).__name__}: {ex}"}
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
        if not a.no_seal and a.encode_gib > 0:
            try:
                result["encode"] = encode(ctx, a.encode_gib, 2)
            except Exception as ex:  # reported, never silently dropped
                result["encode"] = {"error": f"{type(ex).__name__}: {ex}"}
        if not a.no_seal:  # (last: its 128 GiB of buffers are freed before nothing else is allocated)
            try:
                result["seal"] = seal(ctx, dp, n, chunks, max(3, a.steps // 2), a.no_cpu)
            except Exception as ex:  # reported, never silently dropped
                result["seal"] = {"error": f"{type(ex).__name__}: {ex}"}
    ctx.device_free(d_out)
    ctx.device_free(dp)
    if a.corpus_files_per_gpu > 0:
        try:
            r = corpus_sharded(ctx, p, a.corpus_files_per_gpu, 8 << 20, max(3, a.steps // 2), 1, world, rank,
                               barrier, allreduce_max, gather, max(1, min(a.cpu_threads, _cpus())))
            if r:
                result["corpus_sharded"] = r
        except Exception as ex:  # reported, never silently dropped
            result["corpus_sharded"] = {"error": f"{type(ex).__name__}: {ex}"}
    if extras:
        cpu_files = 0 if a.no_cpu else a.cpu_batch_files
        threads = max(1, min(a.cpu_threads, _cpus()))
        for key, fn in (("batch_files", lambda: batch_files(ctx, p, a.batch_files, 8 << 20, 3, cpu_files, threads)
                         if a.batch_files > 0 else None),
                        ("small_files", lambda: small_files(ctx, p, a.small_files, 5) if a.small_files > 0 else None),
                        ("kernel_tree", lambda: kernel_tree(ctx, a.kernel_tree, 5) if a.kernel_tree > 0 else None)):
            try:
                result[key] = fn()
            except Exception as ex:  # reported, never silently dropped
                result[key] = {"error": f"{type(ex).__name__}: {ex}"}
        if not a.no_cpu:
            result["cpu_baseline"] = cpu_baseline(a.cpu_sample_gib, chunks, a.cpu_runs)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
