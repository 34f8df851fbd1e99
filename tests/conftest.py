"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, ABI load/exports,
2-rank gloo DP. `-m gpu` runs on an MI355X: HIP kernels vs the oracle through the C-ABI.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels are launched)")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container (run with -m gpu on the MI355X box)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def golden(name: str) -> dict:
    with np.load(GOLDEN / name, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(autouse=True)
def _x6_bounds_record():
    """Bounds-check builds of the library (ops.X6_BOUNDS, tools/run_bounds_check.sh): after every
    test, no convolution gather may have computed an out-of-range index (ops.bounds_record)."""
    yield
    ops = sys.modules.get("oc_cleanrl_amd.ops")
    if ops is None or not ops.X6_BOUNDS or not ops._BOUNDS_REC:
        return
    import torch

    torch.cuda.synchronize()
    for key, rec in ops._BOUNDS_REC.items():
        r = rec.cpu().tolist()
        rec.zero_()
        if r[0]:
            kind = ops.BOUND_KINDS.get(r[1], r[1])
            idx = (r[2] & 0xffffffff) | (r[3] << 32)
            lim = (r[4] & 0xffffffff) | (r[5] << 32)
            pytest.fail(f"{r[0]} out-of-range gather indices on {key}; first: {kind} {idx} "
                        f"(limit {lim})")


@pytest.fixture(scope="session")
def dev():
    import torch

    return torch.device("cuda:0")
