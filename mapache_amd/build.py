"""Build libmcdc.so in-tree (hipcc, gfx950) — no JIT cache, so the shared
object travels with the repository snapshot to the GPU box.

    python -m mapache_amd.build          # library
    python -m mapache_amd.build --all    # + oracle, C++ host tests, tools
    python -m mapache_amd.build --ab     # + libmcdc_ab.so: A/B build honouring the
                                         #   experiment-only MCDC_* switches (tools/)
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MCDC_ARCH", "gfx950")
CXXFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result"]

LIB_SRCS = ["csrc/mcdc_kernels.hip", "csrc/mcdc_blake3.hip", "csrc/mcdc_aead.hip", "csrc/mcdc_index.hip",
            "csrc/mcdc_zframe.hip", "csrc/mcdc_zcomp.hip", "csrc/mcdc_api.hip"]
LIB_DEPS = LIB_SRCS + ["csrc/mcdc_internal.h", "csrc/mcdc_blake3.h", "csrc/mcdc_aead.h", "csrc/mcdc_index.h", "csrc/mcdc_zframe.h", "csrc/mcdc_zcomp.h", "csrc/mcdc_zstd.h", "csrc/gear_table.h", "../include/mcdc.h",
                       "host/batcher.hpp", "host/zstd_stage.hpp"]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, cwd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


# Kernels allowed to fill their VGPR allocation exactly: none
# of ours.  (The headline scan k_scan_q<4096,2,true> was the last exemption,
# at 128/128; since round 4 lane 0's warm-up hash waits in LDS instead of two
# VGPRs across the tile and it uses 127 of 128.)
# * rocPRIM/hipCUB library kernels (transform, onesweep histogram, block
#   merge) whose source cannot carry MCDC_VGPR_PAD: build_lib raises their
#   descriptors' allocation by one granule in the linked library instead
#   (devaudit.pad_descriptors: code unchanged, the cure §3a measured), after
#   checking that the larger allocation still fits their workgroup size, and
#   re-reads the library's descriptors to confirm it.
EXACT_FILL_OK = ()
LIB_EXACT_FILL_OK = ("_ZN7rocprim",)


def vgpr_report(asm_dir: str):
    """(kernel, next_free_vgpr) of every mcdc kernel in the device assembly hipcc
    left in asm_dir (-save-temps)."""
    out = []
    for f in sorted(os.listdir(asm_dir)):
        if not (f.endswith(".s") and "amdgcn" in f):
            continue
        txt = open(os.path.join(asm_dir, f)).read()
        for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", txt, re.S):
            if m.group(1).startswith("_ZN4mcdc"):
                out.append((m.group(1), int(re.search(r"\.amdhsa_next_free_vgpr\s+(\d+)", m.group(2)).group(1))))
    return out


def exact_fills(report):
    """Kernels whose registers fill their 8-VGPR-granular allocation exactly
    (MCDC_VGPR_PAD in csrc/mcdc_internal.h), outside EXACT_FILL_OK."""
    return [(k, v) for k, v in report if v % 8 == 0 and not (EXACT_FILL_OK and k.startswith(EXACT_FILL_OK))]


def device_guard(asm_dir: str):
    """Every kernel and device function in the library (rocPRIM/hipCUB
    instantiations included), DESIGN.md §3a:
      * the kernel descriptor's VGPR allocation (decoded from the code object)
        equals next_free_vgpr rounded up to the 8-register granule;
      * no register named while a load into it may be outstanding
        (devaudit's waitcnt data-flow pass; in-order write-after-write excluded);
      * every non-kernel device function starts with a full s_waitcnt;
      * no exact fill outside EXACT_FILL_OK / LIB_EXACT_FILL_OK.
    Returns (problems, rows)."""
    from mapache_amd import devaudit
    rows, hazards = devaudit.audit(asm_dir, quiet=True)
    problems = []
    kernels = [r for r in rows if r["kernel"]]
    if not kernels:
        problems.append("no kernels found in the device assembly")
    for r in kernels:
        nfv = r["next_free_vgpr"]
        if r["alloc"] is None:
            problems.append(f"{r['name']}: no kernel descriptor found in the code object")
        elif r["alloc"] != (nfv + 7) // 8 * 8:
            problems.append(f"{r['name']}: descriptor allocates {r['alloc']} VGPRs, code uses {nfv}")
        if nfv % 8 == 0 and not r["name"].startswith(EXACT_FILL_OK + LIB_EXACT_FILL_OK):
            problems.append(f"{r['name']}: fills its VGPR allocation exactly ({nfv}); pad it (MCDC_VGPR_PAD)")
    for r in rows:
        if not r["entry_wait"]:
            problems.append(f"{r['name']}: device function without a full s_waitcnt at entry")
    for h in hazards:
        if h[5] == "raw":
            problems.append(f"{h[0]}: insn {h[1]} '{h[2]}' names v{h[3][0]} while a load into it is outstanding")
    return problems, rows


def pad_library_fills(lib: str, asm_dir: str, rows) -> int:
    """Library kernels (LIB_EXACT_FILL_OK) that fill their allocation exactly get
    one more granule in `lib`'s descriptors; verified from the library bytes."""
    from mapache_amd import devaudit
    names = {r["name"] for r in rows if r["kernel"] and r["next_free_vgpr"] % 8 == 0
             and r["name"].startswith(LIB_EXACT_FILL_OK)}
    if not names:
        return 0
    for r in rows:  # one more granule must still fit the kernel's workgroup (else the launch fails)
        if r["name"] in names:
            if r.get("wg_size") is None:
                raise RuntimeError(f"{r['name']}: no max_flat_workgroup_size in the metadata; cannot pad safely")
            ceil = devaudit.vgpr_ceiling(r["wg_size"])
            if r["next_free_vgpr"] + 8 > ceil:
                raise RuntimeError(f"{r['name']}: padding to {r['next_free_vgpr'] + 8} VGPRs exceeds the "
                                   f"{ceil} a {r['wg_size']}-thread workgroup may allocate")
    done = devaudit.pad_descriptors(lib, asm_dir, names)
    got = devaudit.library_allocations(lib, asm_dir, names)
    nfv = {r["name"]: r["next_free_vgpr"] for r in rows if r["name"] in names}
    bad = [k for k in names if got.get(k) != nfv[k] + 8]
    if bad:
        raise RuntimeError(f"descriptor padding not confirmed for {len(bad)} kernels, e.g. {bad[0]}")
    return len(done)


def build_lib(force: bool = False, ab: bool = False, defines=(), out: str | None = None) -> str:
    """libmcdc.so (ab: libmcdc_ab.so; defines/out: a variant for on-box A/B
    runs, tools/build_variants.py), through the same device-code guard and
    descriptor padding as the product: an unpadded variant once left a
    library kernel at an exact VGPR fill."""
    out = out or os.path.join(HERE, "libmcdc_ab.so" if ab else "libmcdc.so")
    deps = [os.path.join(HERE, d) for d in LIB_DEPS]
    if force or _stale(out, deps):
        tmp = out + ".tmp"
        with tempfile.TemporaryDirectory() as td:  # -save-temps: device assembly + code objects for the guard
            flags = [HIPCC, *CXXFLAGS, *(["-DMCDC_AB_KNOBS"] if ab else []), *[f"-D{d}" for d in defines],
                     "-save-temps", "-fPIC", f"-I{os.path.join(ROOT, 'include')}"]
            procs, objs = [], []
            for src in LIB_SRCS:  # one translation unit per process, in parallel
                o = os.path.join(td, os.path.basename(src).replace(".hip", ".o"))
                objs.append(o)
                cmd = [*flags, "-c", "-o", o, os.path.join(HERE, src)]
                print("+", " ".join(cmd), flush=True)
                procs.append(subprocess.Popen(cmd, cwd=td))
            if any(p.wait() != 0 for p in procs):
                raise RuntimeError("hipcc failed")
            _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], td)
            problems, rows = device_guard(td)
            padded = pad_library_fills(tmp, td, rows)
            if padded:
                print(f"device-code guard: {padded} library kernel descriptors padded by one granule", flush=True)
        if problems and not ab:
            os.remove(tmp)
            raise RuntimeError("device-code guard (DESIGN.md §3a) failed:\n  " + "\n  ".join(problems))
        print(f"device-code guard: {sum(r['kernel'] for r in rows)} kernels, {len(rows)} units checked", flush=True)
        os.replace(tmp, out)
    return out


def build_host_tests(force: bool = False) -> str:
    """C++ test driver for the crate-shaped host API (mapache_amd/host)."""
    out = os.path.join(ROOT, "tests", "cpp", "test_host_api")
    src = os.path.join(ROOT, "tests", "cpp", "test_host_api.cpp")
    deps = [src, os.path.join(HERE, "host", "fastcdc_v2020.hpp"), os.path.join(ROOT, "include", "mcdc.h"),
            os.path.join(HERE, "libmcdc.so")]
    if os.path.exists(src) and (force or _stale(out, deps)):
        build_oracle()
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-Iinclude", "-Imapache_amd/host", "-o", out, src,
              "-Lmapache_amd", "-lmcdc", "-Loracle/_build", "-loracle",
              "-Wl,-rpath,$ORIGIN/../../mapache_amd", "-Wl,-rpath,$ORIGIN/../../oracle/_build", "-lpthread"],
             ROOT)
    return out


# CPU-side C/C++ (the oracle restatement, the crate-shaped host mirror, the
# batching front-end) built plainly and under sanitizers:
# test_batcher{,_asan,_tsan} (oracle as the batch function) and
# test_host_api_asan (host mirror + oracle, `cpu` mode needs no GPU).
SANITIZERS = {"": ["-O2"], "_asan": ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                                      "-fno-sanitize-recover=undefined"],
              "_tsan": ["-O1", "-g", "-fsanitize=thread"]}


def build_cpu_tests(force: bool = False) -> None:
    cpp = os.path.join(ROOT, "tests", "cpp")
    osrc = [os.path.join(ROOT, "oracle", f) for f in ("fastcdc_oracle.c", "blake3_oracle.c")]
    deps = osrc + [os.path.join(ROOT, "oracle", "fastcdc_oracle.h"), os.path.join(HERE, "host", "batcher.hpp"),
                   os.path.join(HERE, "host", "fastcdc_v2020.hpp"), os.path.join(ROOT, "include", "mcdc.h")]
    for suffix, flags in SANITIZERS.items():
        out = os.path.join(cpp, "test_batcher" + suffix)
        src = os.path.join(cpp, "test_batcher.cpp")
        if force or _stale(out, deps + [src]):
            objs = []
            for c in osrc:
                o = os.path.join(cpp, os.path.basename(c)[:-2] + suffix + ".o")
                _run(["gcc", *flags, "-std=c11", "-D_GNU_SOURCE", "-c", "-o", o, c], ROOT)
                objs.append(o)
            _run(["g++", *flags, "-std=c++17", "-Wall", "-Imapache_amd/host", "-o", out, src, *objs, "-lpthread",
                  "-lm"], ROOT)
    zsrc = os.path.join(cpp, "test_zstd_stage.cpp")
    for suffix, flags in SANITIZERS.items():  # the zstd host stage (system libzstd.so.1, dlopen'd)
        out = os.path.join(cpp, "test_zstd_stage" + suffix)
        if os.path.exists(zsrc) and (force or _stale(out, [zsrc, os.path.join(HERE, "host", "zstd_stage.hpp")])):
            _run(["g++", *flags, "-std=c++17", "-Wall", "-Imapache_amd/host", "-o", out, zsrc, "-lpthread", "-ldl"],
                 ROOT)
    out = os.path.join(cpp, "test_host_api_asan")
    src = os.path.join(cpp, "test_host_api.cpp")
    if force or _stale(out, deps + [src, os.path.join(HERE, "libmcdc.so")]):
        flags = SANITIZERS["_asan"]
        objs = []
        for c in osrc:
            o = os.path.join(cpp, os.path.basename(c)[:-2] + "_asan.o")
            _run(["gcc", *flags, "-std=c11", "-D_GNU_SOURCE", "-c", "-o", o, c], ROOT)
            objs.append(o)
        _run(["g++", *flags, "-std=c++17", "-Wall", "-Iinclude", "-Imapache_amd/host", "-o", out, src, *objs,
              "-Lmapache_amd", "-lmcdc", "-Wl,-rpath,$ORIGIN/../../mapache_amd", "-lpthread", "-lm"], ROOT)


def build_format_tests(force: bool = False) -> None:
    """tests/cpp/test_zstd_format: the zstd format pieces of csrc/mcdc_zstd.h on
    the host (hipcc for their __host__ __device__ functions), checked with libzstd."""
    src = os.path.join(ROOT, "tests", "cpp", "test_zstd_format.cpp")
    out = os.path.join(ROOT, "tests", "cpp", "test_zstd_format")
    if os.path.exists(src) and (force or _stale(out, [src, os.path.join(HERE, "csrc", "mcdc_zstd.h")])):
        _run([HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-o", out, src, "-ldl"], ROOT)


def build_tools(force: bool = False) -> None:
    for name in ("scanbench",):
        src = os.path.join(ROOT, "tools", f"{name}.hip")
        out = os.path.join(ROOT, "tools", name)
        deps = [src] + [os.path.join(HERE, d) for d in LIB_DEPS]
        if os.path.exists(src) and (force or _stale(out, deps)):
            _run([HIPCC, *CXXFLAGS, "-Iinclude", "-o", out, src], ROOT)


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return os.path.join(ROOT, "oracle", "_build", "liboracle.so")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--ab", action="store_true")
    a = ap.parse_args(argv)
    build_lib(a.force)
    if a.ab:
        build_lib(a.force, ab=True)
    if a.all:
        build_oracle()
        build_host_tests(a.force)
        build_cpu_tests(a.force)
        build_format_tests(a.force)
        build_tools(a.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
