"""Shared test setup.  CPU tests: `pytest -m "not gpu"`; MI355X tests: `pytest -m gpu`."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsimplex's HIP path)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "run_last: long whole solves, moved to the end of the run")


def pytest_collection_modifyitems(session, config, items):
    # the full-size C4 / C5 certificates (minutes) run after everything else,
    # so a failure elsewhere shows up first under -x
    items.sort(key=lambda it: 1 if it.get_closest_marker("run_last") else 0)


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc  # oracle/oracle.py (test infrastructure)

    orc.lib()
    return orc


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "highs_optima.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def spx():
    import simplex_method_gpu_amd as s

    s._lib.load()
    return s
