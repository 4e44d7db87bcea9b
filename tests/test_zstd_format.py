"""The zstd format pieces of the GPU compressor (mapache_amd/csrc/mcdc_zstd.h:
predefined and per-block FSE tables (table descriptions), sequence bitstream, literal / sequence / block / frame
headers) on the CPU: tests/cpp/test_zstd_format builds frames from synthetic
sequences (every literal-length, match-length and offset code, the 3-byte
sequence-count header) and from a greedy LZ parse of text, random, zero,
periodic and mixed inputs, and decodes every frame with the system libzstd
within mapache's 2^20 window (storage.rs:87-94)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "test_zstd_format")


def test_format_pieces_decode_with_libzstd():
    if not os.path.exists(EXE):
        from mapache_amd import build as B
        B.build_format_tests()
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300)
    if "SKIP" in r.stdout:
        pytest.skip(r.stdout.strip())
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, (r.stdout + r.stderr)[-3000:]
