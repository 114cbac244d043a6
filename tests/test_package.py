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
