"""Shared pytest configuration.

* registers the ``gpu`` marker (tests that need a real MI355X and the built HIP library);
* puts the repo root (for ``oracle``) and ``tx-fast-hydrology_amd`` (for the product package
  ``tx_fast_hydrology_amd``) on ``sys.path``.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_PARENT = os.path.join(ROOT, "tx-fast-hydrology_amd")
for p in (ROOT, PKG_PARENT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libmcroute.so")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load
