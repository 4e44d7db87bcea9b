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
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MCDC_ARCH", "gfx950")
CXXFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result"]

LIB_SRCS = ["csrc/mcdc_kernels.hip", "csrc/mcdc_blake3.hip", "csrc/mcdc_aead.hip", "csrc/mcdc_api.hip"]
LIB_DEPS = LIB_SRCS + ["csrc/mcdc_internal.h", "csrc/mcdc_blake3.h", "csrc/mcdc_aead.h", "csrc/gear_table.h", "../include/mcdc.h",
                       "host/batcher.hpp"]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, cwd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


def build_lib(force: bool = False, ab: bool = False) -> str:
    out = os.path.join(HERE, "libmcdc_ab.so" if ab else "libmcdc.so")
    deps = [os.path.join(HERE, d) for d in LIB_DEPS]
    if force or _stale(out, deps):
        tmp = out + ".tmp"
        _run([HIPCC, *CXXFLAGS, *(["-DMCDC_AB_KNOBS"] if ab else []), "-fPIC", "-shared", "-I../include", "-o", tmp,
              *LIB_SRCS], HERE)
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
        build_tools(a.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
