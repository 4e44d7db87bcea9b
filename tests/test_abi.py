"""The C-ABI library (libmcdc.so) loads, exports every function include/mcdc.h
declares, validates parameters like the crate, and fails loudly (a status,
not a crash and not a CPU fallback) when no HIP device is present."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from mapache_amd import _lib
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "mcdc.h")).read()
    return sorted(set(re.findall(r"\b(mcdc_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert sorted(_lib.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in _declared() if s not in syms]
    assert not missing, missing
    L = _lib.load()
    for s in _declared():
        assert getattr(L, s) is not None


def test_params_check_matches_crate_asserts():
    L = _lib.load()
    ms, ml = ctypes.c_uint64(), ctypes.c_uint64()
    _, _, masks = O.tables()
    assert L.mcdc_params_check(ctypes.byref(_lib.params(16384, 65536, 262144, 1)), ctypes.byref(ms),
                               ctypes.byref(ml)) == 0
    assert ms.value == masks[17] == 0xd90703537000 and ml.value == masks[15] == 0xd90f03530000
    assert L.mcdc_params_check(ctypes.byref(_lib.params(524288, 1 << 20, 8 << 20, 1)), ctypes.byref(ms),
                               ctypes.byref(ml)) == 0
    assert ms.value == masks[21] and ml.value == masks[19]
    for bad in [(63, 256, 1024, 1), (64, 255, 1024, 1), (64, 256, 1023, 1), (1048577, 2 << 20, 4 << 20, 1),
                (64, 4194305, 16 << 20, 1), (64, 256, 16777217, 1), (64, 256, 1024, 4)]:
        assert L.mcdc_params_check(ctypes.byref(_lib.params(*bad)), None, None) == _lib.MCDC_E_PARAMS
        assert _lib.load().mcdc_last_error()  # message set
    assert L.mcdc_params_check(None, None, None) == _lib.MCDC_E_INVALID


def test_digest_matches_oracle_digest():
    d = O.random_bytes(3 << 20, 11)
    c = O.chunk(O.P16, d)
    assert _lib.digest(c) == O.digest_of(c)


def test_abi_version():
    assert _lib.load().mcdc_abi_version() == 5


def test_no_device_fails_loudly():
    """Without a GPU, creating a context is an error status, never a fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.McdcError) as e:
        _lib.Context(0, 1 << 20)
    assert e.value.code == _lib.MCDC_E_DEVICE
    from mapache_amd import FastCDC
    with pytest.raises(_lib.McdcError):
        list(FastCDC(np.zeros(100000, np.uint8), 16384, 65536, 262144))


def test_python_mirror_asserts_like_crate():
    from mapache_amd import FastCDC, StreamCDC
    with pytest.raises(AssertionError, match="min_size >= MINIMUM_MIN"):
        FastCDC(b"", 63, 256, 1024)
    with pytest.raises(AssertionError, match="avg_size <= AVERAGE_MAX"):
        FastCDC(b"", 64, 4194305, 16777216)
    with pytest.raises(AssertionError, match="max_size >= MAXIMUM_MIN"):
        StreamCDC(None, 64, 256, 1023)


def test_cpp_host_api_cpu():
    exe = os.path.join(ROOT, "tests", "cpp", "test_host_api")
    if not os.path.exists(exe):
        from mapache_amd import build
        build.build_host_tests()
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
