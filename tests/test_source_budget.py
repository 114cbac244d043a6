"""Source hygiene without the npm registry: tools/lint_js.js (unused imports and declarations, module size) over
every JS tree, and the same size budget for the Python / C++ / HIP sources (no module over ~700 lines)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUDGET = 700


def test_js_sources_pass_lint_js():
    r = subprocess.run(["node", "tools/lint_js.js", "src", "bench", "tools", "tests/js"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 findings" in r.stdout


def _tracked(exts):
    out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout.split()
    return [f for f in out if f.endswith(exts)]


@pytest.mark.parametrize("exts", [(".py",), (".cpp", ".h", ".hip", ".cc")])
def test_native_and_python_modules_fit_the_budget(exts):
    files = _tracked(exts)
    if not files:
        pytest.skip("not a git checkout")
    over = {}
    for f in files:
        with open(os.path.join(ROOT, f), encoding="utf-8") as fh:
            n = sum(1 for _ in fh)
        if n > BUDGET:
            over[f] = n
    assert not over, over
