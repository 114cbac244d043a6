"""npm manifest and lock: direct dependencies pinned, the lock derived from the reference's resolved tree, CI on `npm ci`.

The reference ships package-lock.json and CI runs `npm ci` (reference .github/workflows/ci.yaml:147-167). A lock
cannot be resolved offline here; tools/derive_lock.py derives it from the reference's lock (lockfileVersion 3), which
resolves exactly the versions package.json pins, rewriting only the root entry and dropping what our root no longer
reaches.
"""
import json
import os
import re

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dev_dependencies_are_exact_versions():
    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    for name, ver in pkg["devDependencies"].items():
        assert re.fullmatch(r"\d+\.\d+\.\d+", ver), (name, ver)
    # peer range stays a range: Headlamp provides React at run time
    assert pkg["peerDependencies"]["react"].startswith("^18")


def test_ci_installs_with_npm_ci():
    ci = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yaml")))
    steps = ci["jobs"]["plugin"]["steps"]
    install = next(s for s in steps if s.get("name") == "Install")["run"]
    assert "npm ci" in install and "npm install" not in install


def _lock():
    return json.load(open(os.path.join(ROOT, "package-lock.json")))


def test_lock_root_matches_the_manifest():
    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    lock = _lock()
    root = lock["packages"][""]
    assert lock["lockfileVersion"] == 3 and lock["name"] == pkg["name"] == root["name"]
    assert lock["version"] == pkg["version"] == root["version"]
    for field in ("devDependencies", "peerDependencies", "bin", "engines"):
        assert root.get(field) == pkg.get(field), field


def test_lock_pins_the_declared_versions_with_integrity():
    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    pkgs = _lock()["packages"]
    for name, ver in pkg["devDependencies"].items():
        assert pkgs["node_modules/" + name]["version"] == ver, name
    for path, ent in pkgs.items():
        if not path or ent.get("link"):
            continue
        assert ent.get("integrity", "").startswith("sha"), path
        assert ent.get("resolved", "").startswith("https://registry.npmjs.org/"), path


def test_lock_is_the_derivation_of_the_reference_tree():
    import subprocess
    import sys

    ref = "/root/reference/package-lock.json"
    if not os.path.exists(ref):
        import pytest

        pytest.skip("reference tree not mounted")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "derive_lock.py"), "--check"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lock = _lock()["packages"]
    # our root reaches no Playwright (the reference's root lists it; this plugin has no e2e suite)
    assert not [p for p in lock if "playwright" in p]
    # every kept package is reachable from our root: nothing extraneous
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import derive_lock

    keep = derive_lock.reachable(lock, list(lock[""]["devDependencies"]) + list(lock[""]["peerDependencies"]))
    assert keep == {p for p in lock if p}


def test_offline_plugin_archive_is_installable_and_reproducible(tmp_path):
    """`node tools/bundle.js --package`: `<name>/main.js` + `<name>/package.json` (the layout Headlamp loads from its
    plugins directory), byte-identical across runs so the ArtifactHub checksum is stable."""
    import hashlib
    import subprocess
    import tarfile

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary

    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    shas = []
    for run in ("a", "b"):
        out = tmp_path / run / "main.js"
        r = subprocess.run([node_binary(), os.path.join(ROOT, "tools", "bundle.js"), "--out", str(out), "--package"],
                           cwd=ROOT, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        arc = tmp_path / run / f"{pkg['name']}-{pkg['version']}.tar.gz"
        sha = hashlib.sha256(arc.read_bytes()).hexdigest()
        assert f"sha256:{sha}" in r.stdout
        shas.append(sha)
        with tarfile.open(arc) as t:
            assert t.getnames() == [f"{pkg['name']}/main.js", f"{pkg['name']}/package.json"]
            assert t.extractfile(f"{pkg['name']}/main.js").read() == out.read_bytes()
            meta = json.load(t.extractfile(f"{pkg['name']}/package.json"))
    assert shas[0] == shas[1]
    assert meta["name"] == pkg["name"] and meta["version"] == pkg["version"] and meta["main"] == "main.js"


def _node():
    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary

    return node_binary()


def _validator():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import validate_artifacthub
    finally:
        sys.path.pop(0)
    return validate_artifacthub


def _committed_digest():
    meta = yaml.safe_load(open(os.path.join(ROOT, "artifacthub-pkg.yml")))
    return meta["annotations"]["headlamp/plugin/archive-checksum"].split(":", 1)[1]


def test_committed_archive_checksum_is_this_trees_archive():
    """artifacthub-pkg.yml's archive-checksum is the sha256 of the archive this tree builds (tools/bundle.js is
    deterministic), recomputed here from the sources; `--check` says the same. A source change without
    `node tools/bundle.js --package --stamp` fails this test (reference /root/reference/artifacthub-pkg.yml:101-105)."""
    import subprocess

    v = _validator()
    digest = v.tree_digest(ROOT)
    assert digest == _committed_digest()
    assert v.validate(os.path.join(ROOT, "artifacthub-pkg.yml"), digest) == []
    r = subprocess.run([_node(), os.path.join(ROOT, "tools", "bundle.js"), "--check"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_validator_rejects_placeholder_and_foreign_digests(tmp_path):
    v = _validator()
    shipped = os.path.join(ROOT, "artifacthub-pkg.yml")

    def with_checksum(hexd):
        m = yaml.safe_load(open(shipped))
        m["annotations"]["headlamp/plugin/archive-checksum"] = "sha256:" + hexd
        p = tmp_path / "pkg.yml"
        p.write_text(yaml.safe_dump(m))
        # screenshots resolve against the file's directory: put them beside it
        if not (tmp_path / "docs").exists():
            os.symlink(os.path.join(ROOT, "docs"), tmp_path / "docs")
        return v.validate(str(p), _committed_digest())

    for placeholder in ("0" * 64, "f" * 64, "ab" * 32, "deadbeef" * 8):
        errs = with_checksum(placeholder)
        assert len(errs) == 1 and "placeholder" in errs[0], (placeholder, errs)
    errs = with_checksum("1" + _committed_digest()[1:] if _committed_digest()[0] != "1" else "2" + _committed_digest()[1:])
    assert len(errs) == 1 and "not this tree's archive" in errs[0], errs
    assert with_checksum(_committed_digest()) == []


def test_the_archive_the_release_uploads_loads_and_registers_every_extension_point(tmp_path):
    """The release's steps, in order, on a scratch copy of the output: bundle + package, then tools/verify_archive.js on
    that file — gunzip, untar, evaluate the archive's own main.js with the host library as `pluginLib`: 6 sidebar
    entries, 5 exact routes, 2 detail sections, 1 column processor, each route and section mounted."""
    import subprocess

    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    r = subprocess.run([_node(), os.path.join(ROOT, "tools", "bundle.js"), "--out", str(tmp_path / "main.js"), "--package"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    arc = tmp_path / f"{pkg['name']}-{pkg['version']}.tar.gz"
    r = subprocess.run([_node(), os.path.join(ROOT, "tools", "verify_archive.js"), str(arc), "--version", pkg["version"],
                        "--sha256", _committed_digest()], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["errors"] == []
    assert out["registered"] == {"sidebar": 6, "routes": 5, "detailSections": 2, "columnProcessors": 1}
    assert out["mounted"] == ["/amd-gpu", "/amd-gpu/device-plugins", "/amd-gpu/nodes", "/amd-gpu/pods", "/amd-gpu/metrics",
                              "node-detail", "pod-detail", "headlamp-nodes columns"]
    assert out["entries"] == [f"{pkg['name']}/main.js", f"{pkg['name']}/package.json"]


def test_archive_verifier_fails_an_archive_that_does_not_register_everything(tmp_path):
    import gzip
    import io
    import subprocess
    import tarfile

    pkg = json.load(open(os.path.join(ROOT, "package.json")))

    def archive(main_js, extra=None):
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w", format=tarfile.USTAR_FORMAT) as t:
            files = [(f"{pkg['name']}/main.js", main_js.encode()),
                     (f"{pkg['name']}/package.json", json.dumps({"name": pkg["name"], "version": pkg["version"],
                                                                 "main": "main.js"}).encode())] + (extra or [])
            for name, body in files:
                info = tarfile.TarInfo(name)
                info.size = len(body)
                t.addfile(info, io.BytesIO(body))
        p = tmp_path / "a.tar.gz"
        p.write_bytes(gzip.compress(buf.getvalue()))
        r = subprocess.run([_node(), os.path.join(ROOT, "tools", "verify_archive.js"), str(p)], cwd=ROOT,
                           capture_output=True, text=True, timeout=120)
        return r.returncode, json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else None

    one_route = ("(function (pluginLib) { pluginLib.registerRoute({ path: '/amd-gpu', exact: true, component: function () "
                 "{ return null; } }); return { registered: { routes: 1 } }; })(pluginLib)")
    rc, out = archive(one_route)
    assert rc == 1 and not out["ok"]
    assert any(e.startswith("sidebar") for e in out["errors"]) and any(e.startswith("routes") for e in out["errors"])
    rc, out = archive("throw new Error('boom')")
    assert rc == 1 and any("does not evaluate" in e for e in out["errors"])
    dist = open(os.path.join(ROOT, "dist-offline", "main.js")).read() if os.path.exists(
        os.path.join(ROOT, "dist-offline", "main.js")) else None
    if dist:
        rc, out = archive(dist, [(f"{pkg['name']}/extra.js", b"1")])
        assert rc == 1 and any("entries" in e for e in out["errors"])


def test_deflate_is_deterministic_and_standard():
    """tools/deflate.js: any inflater reads it, and its bytes are pinned (a zlib build would vary across Node versions,
    and the committed archive digest must be reproducible on the release runner)."""
    import gzip
    import hashlib
    import subprocess

    script = ("import { gzipStable } from './tools/deflate.js';"
              "const parts = []; for (let i = 0; i < 4000; i++) parts.push('line ' + (i * 7919 % 1000) + ' of the MI355X fixture\\n');"
              "process.stdout.write(gzipStable(Buffer.from(parts.join(''))).toString('base64'));")
    r = subprocess.run([_node(), "--input-type=module", "-e", script], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    import base64

    gz = base64.b64decode(r.stdout)
    text = "".join(f"line {i * 7919 % 1000} of the MI355X fixture\n" for i in range(4000)).encode()
    assert gzip.decompress(gz) == text
    assert gz[:4] == b"\x1f\x8b\x08\x00" and gz[4:8] == b"\0\0\0\0"  # no mtime
    assert len(gz) < len(text) // 4
    assert hashlib.sha256(gz).hexdigest() == DEFLATE_GOLDEN


DEFLATE_GOLDEN = "42ae0ea4b2f2995f90011e16f1f66fe0572206d93bc7e80b800a047f20cc20f7"


def test_release_publishes_the_verified_archive_and_commits_its_digest_before_tagging():
    wf = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "release.yaml")))
    steps = wf["jobs"]["release"]["steps"]
    runs = [s.get("run", "") for s in steps]
    names = [s.get("name", "") for s in steps]

    def idx(pred):
        return next(i for i, s in enumerate(steps) if pred(s))

    pack = idx(lambda s: "tools/bundle.js" in s.get("run", "") and "--stamp" in s.get("run", ""))
    verify = idx(lambda s: "tools/verify_archive.js" in s.get("run", ""))
    commit = idx(lambda s: "git push origin HEAD:main" in s.get("run", ""))
    tag = idx(lambda s: "git tag" in s.get("run", ""))
    publish = idx(lambda s: "action-gh-release" in s.get("uses", ""))
    assert pack < verify < commit < tag < publish, names
    assert "dist-offline/amd-gpu-$VERSION.tar.gz" in runs[verify]
    assert steps[publish]["with"]["files"] == "dist-offline/amd-gpu-${{ inputs.version }}.tar.gz"
    assert "artifacthub-pkg.yml" in runs[commit]
    assert not any("headlamp-plugin" in r or "npm run build" in r or "npm run package" in r for r in runs)
    ci = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yaml")))
    ci_runs = " ".join(s.get("run", "") for s in ci["jobs"]["plugin"]["steps"])
    assert "validate_artifacthub.py --tree" in ci_runs and "tools/verify_archive.js" in ci_runs


def test_artifacthub_metadata_is_valid_and_matches_the_manifest(tmp_path):
    """CI's ArtifactHub gate (reference .github/workflows/ci.yaml:25-72) accepts the shipped metadata, whose version is
    package.json's, and rejects the mistakes it exists to catch."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from validate_artifacthub import validate
    finally:
        sys.path.pop(0)
    shipped = os.path.join(ROOT, "artifacthub-pkg.yml")
    assert validate(shipped) == []
    meta = yaml.safe_load(open(shipped))
    assert str(meta["version"]) == json.load(open(os.path.join(ROOT, "package.json")))["version"]

    def broken(mutate):
        m = yaml.safe_load(open(shipped))
        mutate(m)
        p = tmp_path / "pkg.yml"
        p.write_text(yaml.safe_dump(m))
        return validate(str(p))

    assert any("SemVer" in e for e in broken(lambda m: m.update(version="1.2")))
    assert any("checksum" in e for e in broken(lambda m: m["annotations"].update({"headlamp/plugin/archive-checksum": "sha256:xyz"})))
    assert any("v9.9.9" in e for e in broken(lambda m: m.update(version="9.9.9")))
    assert any("license" in e for e in broken(lambda m: m.pop("license")))
    # screenshots: present, raw URLs of this repository, files that exist (here: none under tmp_path)
    assert "missing screenshots" in broken(lambda m: m.pop("screenshots"))
    assert any("does not exist" in e for e in broken(lambda m: None))
    assert any("not in amd-gpu-headlamp" in e for e in broken(
        lambda m: m["screenshots"][0].update(url=m["screenshots"][0]["url"].replace("amd-gpu-headlamp/", "someone-else/"))))
    assert any("raw.githubusercontent.com" in e for e in broken(lambda m: m["screenshots"][0].update(url="https://x/y.png")))
    assert validate(str(tmp_path / "missing.yml")) == [f"{tmp_path / 'missing.yml'} not found"]


def test_real_react_tier_is_configured_and_the_shared_specs_are_runner_agnostic():
    """vitest.react.config.mts renders tests/js/shared/ with the real React in jsdom (no 'react' alias, only the
    Headlamp library mocked); those specs import no harness internals; CI runs the tier."""
    import glob

    cfg = open(os.path.join(ROOT, "vitest.react.config.mts")).read()
    assert "environment: 'jsdom'" in cfg and "tests/js/shared/**/*.test.js" in cfg
    assert "find: /^react$/" not in cfg and "stubs', 'react.js'" not in cfg
    assert "harness', 'dom.js'" in cfg and "@testing-library/react" in open(os.path.join(ROOT, "tests", "js", "harness", "dom.js")).read()
    shared = glob.glob(os.path.join(ROOT, "tests", "js", "shared", "*.test.js"))
    assert shared
    for f in shared:
        src = open(f).read()
        imports = re.findall(r"^import .* from '([^']+)';", src, re.M)
        assert "amd-test-harness" in imports, f
        assert not [i for i in imports if "stubs/" in i or i == "react"], (f, imports)
    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    assert pkg["scripts"]["test:react"] == "vitest run --config vitest.react.config.mts"
    for dep in ("jsdom", "@testing-library/react", "react-dom"):
        assert dep in pkg["devDependencies"], dep
    ci = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yaml")))
    runs = [s.get("run", "") for s in ci["jobs"]["plugin"]["steps"]]
    assert "npm run test:react" in runs
