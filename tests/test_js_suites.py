"""Bridge: every vitest-style JS spec under tests/js runs as its own pytest case.

The shipped plugin logic is JavaScript; these specs run it under the Node
runtime available in this image via tools/minitest.js (a vitest-compatible
runner — vitest itself needs the npm registry). The whole JS suite runs once
per session; each spec id becomes one parametrized case so failures are
reported individually.
"""
import glob
import json
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node") or shutil.which("nodejs")
SPECS = sorted(os.path.relpath(p, ROOT) for p in glob.glob(os.path.join(ROOT, "tests", "js", "*.test.js"))
               + glob.glob(os.path.join(ROOT, "tests", "js", "shared", "*.test.js")))
RUNNER = os.path.join("tools", "minitest.js")
# Resolves 'react' / '@kinvolk/headlamp-plugin/lib' to the harness stand-ins
# and loads the TypeScript entry shims, so the specs import src/index.tsx and
# src/headlamp.ts exactly as Headlamp bundles them.
LOADER = ["--no-warnings", "--experimental-loader", "./tools/plugin-loader.js"]


def _node(args, timeout=120):
    return subprocess.run([NODE] + LOADER + [RUNNER] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


def _list_ids():
    if not NODE or not SPECS:
        return []
    with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
        out = f.name
    try:
        r = _node(["--list", "--json", out] + SPECS)
        if r.returncode != 0:
            raise RuntimeError("JS spec collection failed:\n" + r.stdout + r.stderr)
        with open(out) as fh:
            return json.load(fh)
    finally:
        os.unlink(out)


IDS = _list_ids()


@pytest.fixture(scope="session")
def js_results():
    with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
        out = f.name
    try:
        r = _node(["--json", out] + SPECS, timeout=300)
        if not os.path.exists(out) or os.path.getsize(out) == 0:
            pytest.fail("JS runner crashed:\n" + r.stdout + r.stderr)
        with open(out) as fh:
            return {x["id"]: x for x in json.load(fh)}
    finally:
        if os.path.exists(out):
            os.unlink(out)


def test_node_runtime_present():
    assert NODE, "node is required to run the plugin's JS specs"
    assert len(IDS) >= 150, f"expected the full JS suite, collected {len(IDS)}"


def test_react_layer_specs_collected():
    """The executed React layer (renderer, provider, shipped entry) has its own specs."""
    files = {i.split("::")[0] for i in IDS}
    for f in ("tests/js/react.test.js", "tests/js/provider.test.js", "tests/js/plugin.test.js"):
        assert f in files, f
    assert sum(1 for i in IDS if i.split("::")[0] in files) >= 30


@pytest.mark.parametrize("spec_id", IDS)
def test_js(spec_id, js_results):
    res = js_results.get(spec_id)
    assert res is not None, f"{spec_id} did not run"
    assert res["ok"], res["error"]
