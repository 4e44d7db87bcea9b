"""CPU-side C/C++ under sanitizers (SURVEY.md §5 "Race detection /
sanitizers"): the oracle restatement, the crate-shaped host mirror
(mapache_amd/host/fastcdc_v2020.hpp) and the cross-worker batching front-end
(mapache_amd/host/batcher.hpp), built by ``python -m mapache_amd.build --all``
plainly, with AddressSanitizer + UndefinedBehaviorSanitizer, and with
ThreadSanitizer.  No GPU: the batcher's batch function is the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def _run(exe, *args, env=None):
    path = os.path.join(CPP, exe)
    if not os.path.exists(path):
        pytest.fail(f"{exe} not built: run `python -m mapache_amd.build --all`")
    e = dict(os.environ, **(env or {}))
    r = subprocess.run([path, *map(str, args)], capture_output=True, text=True, timeout=600, env=e)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "ALL PASSED" in r.stdout or "OK (0 failures)" in r.stdout, r.stdout[-2000:]
    return r


def test_batcher_threads():
    _run("test_batcher", 1, 4, 8, 16)


def test_batcher_asan_ubsan():
    r = _run("test_batcher_asan", 4, 16, env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert "runtime error" not in r.stderr


def test_batcher_tsan():
    r = _run("test_batcher_tsan", 4, env={"TSAN_OPTIONS": "halt_on_error=1"})
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_host_mirror_and_oracle_asan_ubsan():
    # (the HIP runtime it links is not instrumented; its allocations are not leak-checked)
    r = _run("test_host_api_asan", "cpu", env={"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1"})
    assert "runtime error" not in r.stderr


def test_zstd_stage_threads():
    _run("test_zstd_stage", 8)


def test_zstd_stage_asan_ubsan():
    r = _run("test_zstd_stage_asan", 4, env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert "runtime error" not in r.stderr


def test_zstd_stage_tsan():
    r = _run("test_zstd_stage_tsan", 4, env={"TSAN_OPTIONS": "halt_on_error=1"})
    assert "WARNING: ThreadSanitizer" not in r.stderr
