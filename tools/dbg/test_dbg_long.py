import numpy as np
import pytest
from mapache_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_dbg(ctx):
    p = (64, 256, 1024, 1)
    z = 80 << 20
    d = np.concatenate([O.random_bytes(100_003, 9), np.zeros(z, np.uint8), O.random_bytes(3 << 20, 10)])
    ref = O.chunk(O.Params(*p), d)
    for rep in range(4):
        g = ctx.chunk_host(_lib.params(*p), d)
        bad = np.nonzero((g["offset"] != ref["offset"]) | (g["length"] != ref["length"]) | (g["hash"] != ref["hash"]))[0]
        print("rep", rep, len(g), bad[:10], [hex(int(x)) for x in g["hash"][bad[:5]]], ctx.timing(), flush=True)
        if len(bad):
            i = bad[0]
            print(g[i - 3:i + 3], ref[i - 3:i + 3], flush=True)
