"""Product tables (mapache_amd/csrc/gear_table.h) equal the oracle's
independently derived GEAR and its MASKS."""
import os
import re

from oracle import oracle as O

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mapache_amd", "csrc",
                   "gear_table.h")


def _parse(name):
    txt = open(HDR).read()
    body = re.search(name + r"\[\d+\] = \{(.*?)\};", txt, re.S).group(1)
    return [int(x, 16) for x in re.findall(r"0x([0-9a-f]+)ull", body)]


def test_product_gear_equals_oracle():
    g, _, m = O.tables()
    assert _parse("kGear") == g
    assert _parse("kMasks") == m
