"""Build an experimental variant of libocppo_hip.so with extra -D flags (never the product):

    python tools/build_variant.py OUT.so [--only SOURCE.hip] -DOCPPO_LOSS_PROBE
    OCPPO_LIB=OUT.so python tools/kernel_bench.py --kernel ppo_loss_prepared --size scaled
"""
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import build as b  # noqa: E402


def main():
    out = Path(sys.argv[1]).resolve()
    defs = sys.argv[2:]
    only = None
    if defs and defs[0] == "--only":  # recompile one source, link the in-tree objects of the rest
        only, defs = defs[1], defs[2:]
    with tempfile.TemporaryDirectory() as td:
        objs = []
        procs = []
        for src in b.sources():
            if only is not None and src.name != only:
                objs.append(b.LIBDIR / "obj" / (src.stem + ".o"))
                continue
            o = Path(td) / (src.stem + ".o")
            objs.append(o)
            procs.append(subprocess.Popen([b.HIPCC, *b.HIP_FLAGS, *b.FILE_FLAGS.get(src.name, []),
                                          *defs, "-c", str(src), "-o", str(o)]))
        assert all(p.wait() == 0 for p in procs)
        subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(out),
                        *map(str, objs), "-Wl,-rpath,/opt/rocm/lib",
                        f"-Wl,--version-script={b.CSRC / 'exports.map'}"], check=True)
    print(out)


if __name__ == "__main__":
    main()
