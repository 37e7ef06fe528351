import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmgdk.so)")


@pytest.fixture(scope="session")
def gdk():
    """The product: libmgdk.so on cuda:0.  Fails loudly if unavailable."""
    from monetdb_amd import gdk as G
    G.init(0)
    return G


@pytest.fixture(scope="session")
def ora():
    from oracle import pyoracle as O
    O.lib()
    return O
