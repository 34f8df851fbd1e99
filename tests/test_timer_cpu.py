"""KernelTimer keeps the closure of each site's FIRST eager launch and replays it after the timed
region (trainer.KernelTimer, bench.py). A closure created inside a loop must bind the loop's
variables at creation time (lambda defaults), else every replay of a site would see the loop's
LAST operands -- the late-binding bug of round 2's config-3 kernel timing (agents.py). Checked
here statically over the package sources and behaviourally on the timer itself (CPU only)."""
import ast
from pathlib import Path

from oc_cleanrl_amd.trainer import KernelTimer

PKG = Path(__file__).resolve().parent.parent / "oc_cleanrl_amd"
TIMER_CALLS = {"bracket", "timed"}


def _loop_targets(node):
    names = set()
    for t in ast.walk(node.target):
        if isinstance(t, ast.Name):
            names.add(t.id)
    return names


def _late_bound_closures(tree):
    """(lineno, name) of every lambda handed to bracket()/timed() inside a for loop of the same
    function that reads a loop variable it does not bind as a default argument."""
    bad = []

    def visit(node, loops):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for ch in node.body:
                visit(ch, [])
            return
        if isinstance(node, ast.For):
            for ch in ast.iter_child_nodes(node):
                visit(ch, loops + [_loop_targets(node)])
            return
        if isinstance(node, ast.Call):
            f = node.func
            fname = f.attr if isinstance(f, ast.Attribute) else getattr(f, "id", None)
            if fname in TIMER_CALLS:
                for arg in node.args:
                    if isinstance(arg, ast.Lambda) and loops:
                        bound = {a.arg for a in arg.args.args}
                        used = {n.id for n in ast.walk(arg.body) if isinstance(n, ast.Name)}
                        live = set().union(*loops)
                        for name in (used & live) - bound:
                            bad.append((node.lineno, name))
        for ch in ast.iter_child_nodes(node):
            visit(ch, loops)

    visit(tree, [])
    return bad


def test_timer_closures_bind_loop_variables():
    bad = {}
    for src in sorted(PKG.glob("*.py")):
        found = _late_bound_closures(ast.parse(src.read_text()))
        if found:
            bad[src.name] = found
    assert not bad, f"late-bound loop variables in timer closures: {bad}"


def test_checker_flags_a_late_bound_closure():
    tree = ast.parse("def f(timer, xs):\n"
                     "    for i, x in enumerate(xs):\n"
                     "        timer.bracket('a', lambda: g(x))\n"
                     "        timer.bracket('b', lambda x=x: g(x))\n")
    assert _late_bound_closures(tree) == [(3, "x")]


def test_timer_keeps_first_closure_with_its_operands():
    t = KernelTimer(enabled=True)
    seen = []
    for it in range(2):  # two "iterations"; counting stops after the first
        for i, x in enumerate((10, 20, 30)):
            t.bracket(f"site{i}", lambda x=x: seen.append(x) or x)
        t.end_iteration()
    assert t.per_iter == {"site0": 1, "site1": 1, "site2": 1}
    seen.clear()
    assert [t.sites[f"site{i}"]() for i in range(3)] == [10, 20, 30]
    assert seen == [10, 20, 30]
    off = KernelTimer(enabled=False)
    assert off.bracket("x", lambda: 5) == 5 and not off.sites
