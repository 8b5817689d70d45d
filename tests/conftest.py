"""pytest configuration for the multi-view -> BEV hot path.

`-m gpu` tests need a real MI355X and the in-tree HIP library; everything else
(oracle vs golden fixtures, host logic, C-ABI symbol table, gloo multi-process)
runs on the CPU.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gather_results(procs, q, n: int, timeout: float):
    """n results from spawned rank processes; fails as soon as a rank died instead of waiting out the timeout
    (a rank that raised never puts its result)."""
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < n:
        try:
            out.append(q.get(timeout=5))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead:
                raise AssertionError(f"a rank process exited with {dead} before reporting")
            if time.time() - t0 > timeout:
                raise AssertionError(f"no result from the rank processes within {timeout} s")
    return out
