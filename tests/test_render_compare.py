"""tools/render_compare.py: opt-in only (ADR 014), and the pooling of several driver processes' samples."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import render_compare  # noqa: E402


def test_refuses_to_run_the_reference_without_the_flag(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "render_compare.py"), "--out", str(tmp_path / "x")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "--allow-reference-exec" in r.stderr
    assert not (tmp_path / "x.json").exists()


def _run(ref_mounts, amd_mounts):
    def side(ms):
        return {"mount": ms, "rerender": [m / 4 for m in ms], "elements": 10}
    page = {"reference": {"elements": 10, "mountMs": sorted(ref_mounts)[len(ref_mounts) // 2]},
            "amd": {"elements": 8, "mountMs": sorted(amd_mounts)[len(amd_mounts) // 2]},
            "samples": {"reference": side(ref_mounts), "amd": side(amd_mounts),
                        "prebuilt": {"mount": [m * 0.7 for m in amd_mounts], "vm": [m * 0.3 for m in amd_mounts]}}}
    return {"gpuPods": 6, "referenceProviderFilterMs": 0.1, "pages": {"nodes": page}}


def test_pooling_recomputes_the_quantiles_over_every_process_sample():
    runs = [_run([1.0, 1.0, 1.0], [0.9, 0.9, 0.9]), _run([2.0, 2.0, 2.0], [1.1, 1.1, 1.1]), _run([3.0, 3.0, 3.0], [3.0, 3.0, 3.0])]
    p = render_compare.pooled(runs)
    a, ref = p["pages"]["nodes"]["amd"], p["pages"]["nodes"]["reference"]
    assert p["runs"] == 3 and ref["reps"] == 9 and a["reps"] == 9
    assert ref["mountMs"] == 2.0 and ref["mountQ1"] == 1.0 and ref["mountQ3"] == 3.0
    assert a["mountMs"] == 1.1 and a["runMountMs"] == [0.9, 1.1, 3.0]
    assert render_compare.verdict(a, ref) == "≤"
    assert abs(a["vmBuildMs"] - 0.33) < 1e-9 and "samples" not in p["pages"]["nodes"]


def test_verdict():
    ref = {"mountMs": 1.0, "mountQ3": 1.2}
    assert render_compare.verdict({"mountMs": 0.9}, ref) == "≤"
    assert render_compare.verdict({"mountMs": 1.1}, ref) == "≈"
    assert render_compare.verdict({"mountMs": 1.3}, ref) == ">"


# ---------------------------------------------------------------------------
# The realm and the process the reference's pages run in (ADR 014), on
# fixture modules of this repository's own (tests/fixtures/refrealm), never
# the reference's.
# ---------------------------------------------------------------------------

FIXTURE = os.path.join(ROOT, "tests", "fixtures", "refrealm")

REALM_SCRIPT = r"""
import vm from 'vm';
import { createRequire } from 'module';
import worker from './bench/refWorker.cjs';
import { realmInit } from './bench/refIsolated.js';
const require = createRequire(import.meta.url);
const [fixture, umd] = process.argv.slice(2);
(async function () {
  const realm = worker.createRealm(vm, realmInit(fixture, umd));
  const nodes = [{ metadata: { name: 'n0' }, status: { capacity: { 'gpu.intel.com/i915': '8' } } }, { metadata: { name: 'cpu' }, status: {} }];
  const pods = [{ metadata: { name: 'p' }, spec: { containers: [{ resources: { requests: { 'gpu.intel.com/i915': '1' } } }] } }];
  const out = { data: JSON.parse(realm.api.setData(JSON.stringify({ nodes, pods, devicePlugins: [], pluginPods: [], metrics: { chips: [{}, {}] } }))) };
  out.pages = {};
  for (const page of ['overview', 'devicePlugins', 'nodes', 'pods', 'metrics']) {
    out.pages[page] = await worker.cycle(realm.api, { page, waitText: page === 'metrics' ? 'GPU Power Summary' : null, mustShow: 'Intel GPU' },
      () => new Promise((r) => setImmediate(r)));
  }
  const host = { process, require, Function, Object };
  out.audit = worker.audit(vm, realm.ctx, host);
  out.globals = vm.runInContext('[typeof process, typeof require, typeof setImmediate, typeof Buffer, typeof fetch].join()', realm.ctx);
  try { vm.runInContext('(function () {}).constructor("return 1")', realm.ctx); out.codegen = 'allowed'; } catch (e) { out.codegen = e.message; }
  // negative control: one host object handed in is found, with the path to it
  vm.runInContext('globalThis', realm.ctx).handedIn = { cb: function () {} };
  out.control = worker.audit(vm, realm.ctx, host).leaks.slice(0, 3);
  process.stdout.write(JSON.stringify(out));
})().catch((e) => { console.error(e.stack); process.exit(1); });
"""


def _umd_prod():
    from headlamp_intel_gpu_plugin_amd.utils.reactumd import PROD_BUILDS, umd_dir

    return umd_dir(PROD_BUILDS)


def test_the_reference_realm_reaches_nothing_of_the_host(tmp_path):
    """Everything reachable from the realm's global object after every page mounted, waited and re-rendered is the
    realm's own: no `process`, no `require`, no host-realm function or object (bench/refWorker.cjs audit); Node's
    globals are absent and the realm compiles no code from strings. A host object handed in is caught."""
    import json

    import pytest

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary

    umd = _umd_prod()
    if not umd:
        pytest.skip("react@18.3.1 production UMD builds not available")
    script = tmp_path / "realm.mjs"
    script.write_text(REALM_SCRIPT.replace("'./bench/", "'" + ROOT + "/bench/"))
    r = subprocess.run([node_binary(), str(script), FIXTURE, umd], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["data"] == {"gpuNodes": 1, "gpuPods": 1, "chips": 2}
    assert {p: v["elements"] > 0 for p, v in out["pages"].items()} == dict.fromkeys(
        ["overview", "devicePlugins", "nodes", "pods", "metrics"], True)
    assert out["audit"]["leaks"] == [] and out["audit"]["objects"] > 500
    assert out["globals"] == "undefined,undefined,undefined,undefined,undefined"
    assert "Code generation from strings disallowed" in out["codegen"]
    assert out["control"][0] == "globalThis.handedIn: a host-realm object"
    assert out["control"][1] == "globalThis.handedIn.cb: a host-realm function"


ISOLATED_SCRIPT = r"""
import { startWorker, realmInit } from './bench/refIsolated.js';
const [fixture, umd] = process.argv.slice(2);
(async function () {
  const w = startWorker();
  const out = {};
  out.init = await w.call('init', realmInit(fixture, umd));
  out.probe = await w.call('probe');
  await w.call('setData', { json: JSON.stringify({ nodes: [], pods: [], devicePlugins: [], pluginPods: [], metrics: { chips: [] } }) });
  out.cycle = await w.call('cycle', { page: 'metrics', waitText: 'GPU Power Summary', mustShow: 'Intel GPU' });
  out.audit = await w.call('audit');
  await w.close();
  // a call answered late kills the worker: this one, and every later call, rejects
  const w2 = startWorker();
  out.late = await w2.call('init', realmInit(fixture, umd), 1).then(() => 'answered', (e) => e.message);
  out.after = await w2.call('probe').then(() => 'answered', (e) => e.message);
  await w2.close();
  process.stdout.write(JSON.stringify(out));
})().catch((e) => { console.error(e.stack); process.exit(1); });
"""


def _can_isolate():
    try:
        return subprocess.run(["unshare", "--net", "--mount", "--propagation", "private", "--", "true"],
                              capture_output=True, timeout=30).returncode == 0
    except (OSError, subprocess.SubprocessError):
        return False


def test_the_reference_worker_has_no_network_and_writes_nothing(tmp_path):
    """The process bench/refIsolated.js starts for the reference's pages: its writes fail on every mount it tries
    (read-only namespace, RLIMIT_FSIZE 0), its TCP connection out fails (empty network namespace), and its realm
    still renders a page and audits clean. A call answered late kills the worker and fails every later call. Skipped where the container allows no namespaces (ADR 014)."""
    import json

    import pytest

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary

    umd = _umd_prod()
    if not umd or not _can_isolate():
        pytest.skip("no React production UMD builds, or no unshare --net --mount here")
    script = tmp_path / "iso.mjs"
    script.write_text(ISOLATED_SCRIPT.replace("'./bench/", "'" + ROOT + "/bench/"))
    r = subprocess.run([node_binary(), str(script), FIXTURE, umd], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    writes = out["probe"]["writes"]
    assert len(writes) == 3 and set(writes.values()) <= {"EROFS", "EFBIG", "EACCES", "EPERM"}, writes
    assert out["probe"]["connect"] in ("ENETUNREACH", "EHOSTUNREACH", "ENETDOWN"), out["probe"]
    assert out["cycle"]["elements"] > 0
    assert out["audit"]["leaks"] == []
    assert out["late"].startswith("reference worker timed out after 1 ms on init"), out["late"]
    assert out["after"] == out["late"]
    for f in ("/tmp/.ref-probe", "/dev/shm/.ref-probe"):
        assert not os.path.exists(f)
