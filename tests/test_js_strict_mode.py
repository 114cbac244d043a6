"""The shared product specs once more with every render under <StrictMode>.

React 18's StrictMode (development) renders each component twice and mounts,
unmounts and re-mounts every effect, to flush out effects that are not
idempotent: a fetch effect without cancellation or de-duplication sends its
request twice, a subscription without cleanup leaks. AMD_TEST_STRICT=1 makes
the render adapters (tests/js/harness/{stub,umd,dom}.js) wrap every render in
StrictMode; the product specs' assertions (request counts, rendered text,
refresh paths) must hold unchanged, on the harness React and on real React
18.3.1 (UMD builds, offline). react-semantics.shared.test.js is left out: it
counts renders and effect runs one by one and has its own StrictMode specs.
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
PRODUCT = sorted(os.path.relpath(p, ROOT) for p in glob.glob(os.path.join(ROOT, "tests", "js", "shared", "*.test.js"))
                 if not p.endswith("react-semantics.shared.test.js"))
LOADER = ["--no-warnings", "--experimental-loader", "./tools/plugin-loader.js"]
UMD = umd_dir()

pytestmark = pytest.mark.skipif(not NODE, reason="node is required")


def _run(env):
    with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
        out = f.name
    try:
        r = subprocess.run([NODE] + LOADER + [os.path.join("tools", "minitest.js"), "--json", out] + PRODUCT, cwd=ROOT,
                           capture_output=True, text=True, timeout=300, env=dict(os.environ, AMD_TEST_STRICT="1", **env))
        if not os.path.exists(out) or os.path.getsize(out) == 0:
            pytest.fail("JS runner crashed under StrictMode:\n" + r.stdout + r.stderr)
        with open(out) as fh:
            return json.load(fh), r.stdout + r.stderr
    finally:
        os.unlink(out)


def _check(results):
    assert len(results) >= 60, len(results)
    failed = [(x["id"], x["error"][:300]) for x in results if not x["ok"]]
    assert not failed, failed[:5]


def test_product_specs_under_strict_mode_on_the_harness_react():
    results, _ = _run({})
    _check(results)


@pytest.mark.skipif(not UMD, reason="the React 18.3.1 UMD builds are not available")
def test_product_specs_under_strict_mode_on_real_react():
    results, console = _run({"AMD_TEST_TIER": "react-umd", "AMD_REACT_UMD_DIR": UMD})
    assert all("react-dom-umd" in x["id"] for x in results)
    _check(results)
    assert "Warning:" not in console, [l for l in console.splitlines() if "Warning:" in l][:5]
