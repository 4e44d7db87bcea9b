"""Golden boundary vectors (tests/golden/, self-generated from the oracle and
labelled crate-unverified).  CPU: the oracle still reproduces them.  GPU: the
MI355X path reproduces them bit for bit (offsets, lengths and hashes)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden.make_golden import make_input

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fastcdc_v2020_golden.json")))["cases"]


def _expected(case):
    lens = np.array(case["lengths"], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if len(lens) else lens
    return offs, lens, np.array([int(h, 16) for h in case["hashes"]], dtype=np.uint64)


def _ids(c):
    return f"{'/'.join(map(str, c['params']))}-{c['input']['kind']}-{c['input']['len']}"


@pytest.mark.parametrize("case", GOLD, ids=_ids)
def test_oracle_reproduces_golden(case):
    d = make_input(case["input"])
    assert hashlib.sha256(d.tobytes()).hexdigest() == case["sha256"]
    c = O.chunk(O.Params(*case["params"]), d)
    offs, lens, hashes = _expected(case)
    assert (c["offset"] == offs).all() and (c["length"] == lens).all() and (c["hash"] == hashes).all()


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLD, ids=_ids)
def test_gpu_reproduces_golden(case, ctx):
    from mapache_amd import _lib
    d = make_input(case["input"])
    g = ctx.chunk_host(_lib.params(*case["params"]), d)
    offs, lens, hashes = _expected(case)
    assert len(g) == len(lens)
    assert (g["offset"] == offs).all() and (g["length"] == lens).all() and (g["hash"] == hashes).all()
