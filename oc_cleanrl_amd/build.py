"""Build libocppo_hip.so (gfx950) in-tree with hipcc, plus the oracle's C restatement.

    python -m oc_cleanrl_amd.build          # incremental: rebuilds when a source is newer
    python -m oc_cleanrl_amd.build --force

The shared library is the C-ABI of include/ocppo.h; it is loaded by oc_cleanrl_amd._lib with
ctypes after torch (so the process has exactly one HIP runtime: torch's libamdhip64.so.7 and ours
share the soname).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
LIB = LIBDIR / "libocppo_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OCPPO_ARCH", "gfx950")

HIP_FLAGS = [
    "-O3",
    "-std=c++17",
    f"--offload-arch={ARCH}",
    "-ffp-contract=off",  # keep PyTorch's per-op f32 rounding (bit-exact GAE)
    "-fPIC",
    "-fvisibility=hidden",  # export exactly the C-ABI (OCPPO_API in include/ocppo.h)
    "-Wall",
    "-Wno-unused-function",
]


# Per-source extra flags. ocppo_gemm.hip: no SLP packing of scalar f32 ops into v_pk_* (same
# results) -- beside MFMAs a packed f32 op costs more issue time than the two scalar ones
# (gemm_x6's operand split: config-2 GEMMs 730 -> 704 us, bench +2.4 %).
FILE_FLAGS = {"ocppo_gemm.hip": ["-fno-slp-vectorize"]}


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_hip(force: bool = False, verbose: bool = False) -> Path:
    srcs = sources()
    deps = srcs + sorted(CSRC.glob("*.h")) + [CSRC / "exports.map"] + [ROOT / "include" / "ocppo.h", Path(__file__)]
    if not force and not _stale(LIB, deps):
        return LIB
    LIBDIR.mkdir(exist_ok=True)
    objdir = LIBDIR / "obj"
    objdir.mkdir(exist_ok=True)
    objs = []
    procs = []
    for src in srcs:
        obj = objdir / (src.stem + ".o")
        objs.append(obj)
        cmd = [HIPCC, *HIP_FLAGS, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((src, out.decode()))
        elif verbose and out:
            print(out.decode())
    if failed:
        msg = "\n".join(f"--- {s.name}\n{o}" for s, o in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
           "-Wl,-rpath,/opt/rocm/lib", f"-Wl,--version-script={CSRC / 'exports.map'}"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_oracle(force: bool = False) -> Path:
    sys.path.insert(0, str(ROOT))
    from oracle import build as oracle_build  # noqa: E402  (test infrastructure, C restatement)

    return oracle_build.build(force=force)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args(argv)
    print(build_hip(force=a.force, verbose=a.verbose))
    if not a.no_oracle:
        print(build_oracle(force=a.force))


if __name__ == "__main__":
    main()
