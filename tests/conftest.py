"""Shared test setup: import paths, the `gpu` marker, graph fixtures.

`-m "not gpu"` tests run anywhere (CPU oracle, host logic, library load/exports, the
CPU-device backend, the gloo multi-process path). `-m gpu` tests are the parity tests
proper: they call the HIP kernels through the C-ABI and compare with the oracle.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pla-gnn_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(pytest.mark.timeout(600))


def random_graph(n, e, seed=0, self_loop=True):
    """Random multigraph COO (duplicates and explicit self-loops allowed, like
    PPI_inter's diagonal), plus DGL self-loops appended when self_loop."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, e).astype(np.int64)
    dst = rng.integers(0, n, e).astype(np.int64)
    if self_loop:
        src = np.concatenate([src, np.arange(n)])
        dst = np.concatenate([dst, np.arange(n)])
    return src, dst


def hub_graph(n, hub_deg, seed=0):
    """Random graph plus node 0 receiving hub_deg in-edges (forces split rows) and node 1
    sending hub_deg out-edges; self-loops appended."""
    rng = np.random.default_rng(seed)
    s = [rng.integers(0, n, 4 * n), rng.integers(0, n, hub_deg), np.ones(hub_deg, np.int64)]
    d = [rng.integers(0, n, 4 * n), np.zeros(hub_deg, np.int64), rng.integers(0, n, hub_deg)]
    src = np.concatenate(s + [np.arange(n)]).astype(np.int64)
    dst = np.concatenate(d + [np.arange(n)]).astype(np.int64)
    return src, dst


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle
