"""BLAKE3 chunk-ID oracle (oracle/blake3_oracle.c) against the fixtures.

Pins the CPU restatement that the GPU chunk-ID kernels are checked against:
the reference's own KAT (src/utils/mod.rs:426-441), the published
BLAKE3("") / BLAKE3("abc"), recalled official test vectors across the
1024-byte leaf edge (tests/golden/blake3_kat.json, made by make_blake3_kat.py),
and a second, independent statement of the tree (pure Python, recursive).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "blake3_kat.json")))


def _input(k):
    if "pattern_i_mod_251" in k:
        return bytes(i % 251 for i in range(k["pattern_i_mod_251"]))
    return bytes.fromhex(k["input_hex"])


@pytest.mark.parametrize("k", KATS, ids=lambda k: k["source"][:40])
def test_kats(k):
    d = _input(k)
    assert O.blake3(d).hex() == k["blake3"]
    assert O.blake3_py(d).hex() == k["blake3"]


def test_reference_kat_is_the_reference_test():
    k = KATS[0]
    assert k["source"].startswith("reference src/utils/mod.rs")
    assert k["blake3"] == "28ff314ca7c551552d4d2f4be86fd2348749ace0fbda1a051038bdb493c10a4d"
    assert len(bytes.fromhex(k["input_hex"])) == 509


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 3 * 1024 + 1,
                               4096, 5 * 1024 + 7, 8192, 8193, 16384, 16385, 17 * 1024, 33 * 1024 + 3, 65536 + 1])
def test_two_tree_statements_agree(n):
    d = O.random_bytes(n, 77 + n).tobytes()
    assert O.blake3(d) == O.blake3_py(d)


def test_chunk_ids_threads_and_offsets():
    d = O.random_bytes(3 << 20, 5)
    c = O.chunk(O.P16, d)
    one = O.chunk_ids(d, c, threads=1)
    four = O.chunk_ids(d, c, threads=4)
    assert (one == four).all()
    for i in (0, len(c) // 2, len(c) - 1):
        o, ln = int(c["offset"][i]), int(c["length"][i])
        assert bytes(one[i]) == O.blake3(d[o:o + ln].tobytes())
