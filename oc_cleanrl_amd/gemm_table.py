"""The shipped hipBLASLt solution table for the update GEMMs (PyTorch TunableOp, read-only).

The network forward / backward of the update stays on PyTorch's BLAS path (hipBLASLt). Its default
heuristic picks one solution per shape; for the fixed shapes of the benchmarked configs
(2: PPObj at the frame-dedup capacity, 3: NatureCNN, 5: the DQN train step) a timed pick among
hipBLASLt's own solutions is up to 2 % of the config-2 iteration faster (tools/tunable_bench.sh:
774-779k vs 759k env steps/s on one box). `tools/tune_gemms.sh` regenerates the table on an
MI355X (TunableOp with rocBLAS solutions excluded: those won TunableOp's own timing and lost
under hipGraph replay); this module loads it once per process with tuning OFF, so a
shape missing from the table keeps the default solution and nothing is timed at run time.
TunableOp checks the table's validators (PyTorch, HIP, hipBLASLt versions, gfx arch) and ignores
a table from another stack. OCPPO_GEMM_TABLE=0 or Args.gemm_table=False leaves the default.
"""
from __future__ import annotations

import os
import tempfile
from pathlib import Path

import torch

TABLE = Path(__file__).resolve().parent / "tuning" / "tunableop_gfx950.csv"
_state: dict = {}


def use(device) -> bool:
    """Enable the table for this process (idempotent). Returns whether it is in use."""
    if "on" in _state:
        return _state["on"]
    _state["on"] = False
    if (os.environ.get("OCPPO_GEMM_TABLE", "1") == "0" or not TABLE.exists() or
            os.environ.get("PYTORCH_TUNABLEOP_ENABLED") is not None):  # a user's TunableOp wins
        return False
    dev = torch.device(device)
    if dev.type != "cuda" or "gfx950" not in torch.cuda.get_device_properties(dev).gcnArchName:
        return False
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    # results written at exit go to a scratch file, never over the shipped table
    t.set_filename(os.path.join(tempfile.gettempdir(), f"ocppo_tunableop_{os.getpid()}.csv"))
    ok = bool(t.read_file(str(TABLE)))
    if not ok:
        t.enable(False)
    _state["on"] = ok
    return ok
