"""The C restatement of the GAE loop agrees bit-for-bit with the reference fixtures."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


@pytest.mark.parametrize("name", sorted(os.path.basename(p) for p in glob.glob(str(GOLDEN / "gae_*.npz"))))
def test_c_gae_bitwise(name):
    from oracle import build

    lib = build.load()
    z = golden(name)
    T, N = z["rewards"].shape
    adv = np.empty((T, N), np.float32)
    ret = np.empty((T, N), np.float32)
    p = lambda a: np.ascontiguousarray(a).ctypes.data  # noqa: E731
    arrs = [np.ascontiguousarray(z[k]) for k in ("rewards", "values", "dones", "next_value", "next_done")]
    lib.oracle_gae(*[a.ctypes.data for a in arrs], T, N, float(z["gamma"]), float(z["gae_lambda"]),
                   adv.ctypes.data, ret.ctypes.data)
    assert np.array_equal(adv.view(np.uint32), z["advantages"].view(np.uint32))
    assert np.array_equal(ret.view(np.uint32), z["returns"].view(np.uint32))
