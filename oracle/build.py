"""Build the oracle's C restatement (oracle/ocppo_oracle.c) with gcc into oracle/_build/.

TEST INFRASTRUCTURE ONLY. The reference (BluemlJ/oc_cleanrl) is pure Python, so there is no
compiled reference to build into oracle/_ref/; parity is pinned by tests/golden/ instead."""
from __future__ import annotations

import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "ocppo_oracle.c"
OUT = HERE / "_build" / "libocppo_oracle.so"


def build(force: bool = False) -> Path:
    if not force and OUT.exists() and OUT.stat().st_mtime >= SRC.stat().st_mtime:
        return OUT
    OUT.parent.mkdir(exist_ok=True)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                    "-o", str(OUT), str(SRC)], check=True)
    return OUT


def load():
    import ctypes

    lib = ctypes.CDLL(str(build()))
    P, I64, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
    lib.oracle_gae.argtypes = [P, P, P, P, P, I64, I64, D, D, P, P]
    lib.oracle_gae.restype = None
    return lib


if __name__ == "__main__":
    print(build(force=True))
