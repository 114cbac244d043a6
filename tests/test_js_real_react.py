"""The shared React-layer specs on REAL React 18.3.1 + react-dom, offline.

tests/js/shared/*.test.js (every route, both detail sections, the provider
hooks, the renderer's blocks, the React 18 rules the harness React models) run
here a second time against the UMD development builds of react@18.3.1 and
react-dom@18.3.1 — the versions package.json pins — over a minimal DOM
(tests/js/harness/minidom.js, umd-react.js, umd.js; tools/plugin-loader.js with
AMD_TEST_TIER=react-umd). There is no npm registry here, so the builds come
from a Python package of this image that vendors them (dash); the test skips
when none is importable. In networked CI the same specs also run on
react-dom in jsdom with @testing-library/react (vitest.react.config.mts).

One pytest case per spec, as in tests/test_js_suites.py.
"""
import glob
import json
import os
import shutil
import subprocess
import tempfile

import pytest

from headlamp_intel_gpu_plugin_amd.utils.reactumd import umd_dir

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node") or shutil.which("nodejs")
SHARED = sorted(os.path.relpath(p, ROOT) for p in glob.glob(os.path.join(ROOT, "tests", "js", "shared", "*.test.js")))
RUNNER = os.path.join("tools", "minitest.js")
LOADER = ["--no-warnings", "--experimental-loader", "./tools/plugin-loader.js"]

UMD = umd_dir()
ENV = dict(os.environ, AMD_TEST_TIER="react-umd", AMD_REACT_UMD_DIR=UMD or "")
pytestmark = pytest.mark.skipif(not (NODE and UMD), reason="node or the React 18.3.1 UMD builds are not available")


def _node(args, timeout=300):
    return subprocess.run([NODE] + LOADER + [RUNNER] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                          env=ENV)


def _list_ids():
    if not (NODE and UMD and SHARED):
        return []
    with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
        out = f.name
    try:
        r = _node(["--list", "--json", out] + SHARED)
        if r.returncode != 0:
            raise RuntimeError("shared spec collection on real React failed:\n" + r.stdout + r.stderr)
        with open(out) as fh:
            return json.load(fh)
    finally:
        os.unlink(out)


IDS = _list_ids()


@pytest.fixture(scope="session")
def react_results():
    with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
        out = f.name
    try:
        r = _node(["--json", out] + SHARED)
        if not os.path.exists(out) or os.path.getsize(out) == 0:
            pytest.fail("JS runner crashed on real React:\n" + r.stdout + r.stderr)
        with open(out) as fh:
            res = {x["id"]: x for x in json.load(fh)}
        res["__console__"] = r.stdout + r.stderr
        return res
    finally:
        if os.path.exists(out):
            os.unlink(out)


def test_real_react_loads_and_every_shared_file_runs(react_results):
    files = {i.split("::")[0] for i in IDS}
    assert files == set(SHARED), files
    assert len(IDS) >= 80
    # the tier label in the spec names says which React rendered them
    assert all("react-dom-umd" in i for i in IDS), [i for i in IDS if "react-dom-umd" not in i][:3]


def test_real_react_warns_about_nothing(react_results):
    # React's development build reports misuse on console.error as "Warning: …":
    # missing or duplicate keys, invalid DOM nesting or props, updates on
    # unmounted components, setState in render, hook order changes. The shipped
    # renderer, provider and pages must trigger none of them on any spec.
    out = react_results["__console__"]
    warnings = [l for l in out.splitlines() if "Warning:" in l]
    assert not warnings, warnings[:5]


@pytest.mark.parametrize("spec_id", IDS)
def test_shared_spec_on_real_react(spec_id, react_results):
    res = react_results.get(spec_id)
    assert res is not None, f"{spec_id} did not run"
    assert res["ok"], res["error"]
