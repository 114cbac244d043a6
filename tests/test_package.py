"""npm manifest: direct dependencies pinned, CI installs from the lock when one exists.

The reference ships package-lock.json and CI runs `npm ci` (reference .github/workflows/ci.yaml:147-167). A lock
cannot be generated offline here, so the pins in package.json are the reproducibility floor until CI's first
networked run produces one (uploaded as an artifact by .github/workflows/ci.yaml).
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


def test_ci_prefers_npm_ci_when_locked():
    ci = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yaml")))
    steps = ci["jobs"]["plugin"]["steps"]
    install = next(s for s in steps if s.get("name") == "Install")["run"]
    assert "package-lock.json" in install and "npm ci" in install
    assert any(s.get("uses", "").startswith("actions/upload-artifact") for s in steps)


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
    assert validate(str(tmp_path / "missing.yml")) == [f"{tmp_path / 'missing.yml'} not found"]
