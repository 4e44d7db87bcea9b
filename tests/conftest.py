"""Shared pytest setup: the `gpu` marker and helpers.

CPU tests (``-m "not gpu"``) cover the oracle against golden vectors and
recalled crate KATs, the product tables, the host logic and that the C-ABI
library loads and exports every symbol ``include/mcdc.h`` declares.  GPU tests
(``-m gpu``) are the parity tests proper and call through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmcdc.so on the device)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def ctx():
    """One mcdc context for the whole GPU session (fails loudly without HIP)."""
    from mapache_amd import _lib
    c = _lib.Context(0, 16 << 30)
    yield c
    c.close()
