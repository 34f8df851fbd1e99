"""Bench A/B of a module-level switch in one box session (experiment):
    python tools/ab_toggle.py agents.DEFER_WGRAD_AFTER_FIRST_LAYER 0 [bench args...]
runs bench.py in-process with oc_cleanrl_amd.<module>.<NAME> set to the given value."""
import runpy
import sys
from importlib import import_module
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    target, value = sys.argv[1], sys.argv[2]
    mod, name = target.rsplit(".", 1)
    m = import_module(f"oc_cleanrl_amd.{mod}")
    v = int(value)
    setattr(m, name, bool(v) if isinstance(getattr(m, name), bool) else v)
    sys.argv = [str(ROOT / "bench.py")] + sys.argv[3:]
    runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
