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
