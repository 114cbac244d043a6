#!/usr/bin/env python3
"""Validate artifacthub-pkg.yml (required fields, SemVer, archive annotations, screenshots).

Used by CI and the release job; exits non-zero with one line per problem.

    python3 tools/validate_artifacthub.py [artifacthub-pkg.yml] [--tree]

`--tree` also rebuilds the plugin archive this tree ships (`node tools/bundle.js --digest`: the deterministic bundle +
tar + gzip of tools/bundle.js) and requires the committed archive-checksum to be its sha256: ArtifactHub indexes main, so
the digest on main must be the one of the archive the release publishes from it (reference
/root/reference/artifacthub-pkg.yml:101-105 commits its real digest).
"""
import os
import re
import subprocess
import sys

import yaml


def placeholder_digest(hexdigest):
    """A digest nobody computed: one repeated hex digit (the all-zero stand-in) or a short repeating pattern."""
    h = str(hexdigest).lower()
    return any(h == h[:n] * (64 // n) for n in (1, 2, 4, 8))


def tree_digest(root=None):
    """sha256 hex of the archive this tree ships, from tools/bundle.js (needs Node)."""
    root = root or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    try:
        from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary
        node = node_binary()
    except Exception:  # the package is not importable (bare CI step): the node on PATH
        node = "node"
    finally:
        sys.path.pop(0)
    r = subprocess.run([node, os.path.join(root, "tools", "bundle.js"), "--digest"], cwd=root, capture_output=True,
                       text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError("tools/bundle.js --digest failed: " + r.stderr.strip())
    m = re.match(r"^sha256:([0-9a-f]{64})$", r.stdout.strip())
    if not m:
        raise RuntimeError("tools/bundle.js --digest printed " + repr(r.stdout))
    return m.group(1)


def validate(path="artifacthub-pkg.yml", expect_digest=None):
    """Problems with the metadata at `path`; with `expect_digest` (hex), also unless its checksum is that digest."""
    errors = []
    try:
        with open(path) as f:
            pkg = yaml.safe_load(f) or {}
    except FileNotFoundError:
        return [f"{path} not found"]
    except yaml.YAMLError as e:
        return [f"{path} is invalid YAML: {e}"]
    for field in ("version", "name", "description", "homeURL", "license", "category"):
        if not pkg.get(field):
            errors.append(f"missing required field: {field}")
    version = str(pkg.get("version", ""))
    if version and not re.match(r"^\d+\.\d+\.\d+$", version):
        errors.append(f"version {version!r} is not SemVer X.Y.Z")
    ann = pkg.get("annotations") or {}
    url = ann.get("headlamp/plugin/archive-url", "")
    checksum = ann.get("headlamp/plugin/archive-checksum", "")
    if not url:
        errors.append("missing annotation headlamp/plugin/archive-url")
    elif version and f"v{version}" not in url:
        errors.append(f"archive-url does not reference v{version}")
    if not re.match(r"^sha256:[0-9a-f]{64}$", str(checksum)):
        errors.append(f"archive-checksum {checksum!r} is not sha256:<64 hex>")
    elif placeholder_digest(str(checksum)[7:]):
        errors.append(f"archive-checksum {checksum!r} is a placeholder, not the archive's digest "
                      "(run: node tools/bundle.js --package --stamp)")
    elif expect_digest and str(checksum)[7:] != expect_digest:
        errors.append(f"archive-checksum {checksum!r} is not this tree's archive sha256:{expect_digest} "
                      "(run: node tools/bundle.js --package --stamp)")
    if not ann.get("headlamp/plugin/version-compat"):
        errors.append("missing annotation headlamp/plugin/version-compat")
    errors.extend(screenshot_errors(pkg, os.path.dirname(os.path.abspath(path))))
    return errors


# ArtifactHub shows what `url` serves; the files are this repository's docs/screenshots, published from main.
RAW_RE = re.compile(r"^https://raw\.githubusercontent\.com/([^/]+)/([^/]+)/[^/]+/(docs/screenshots/[\w.-]+\.(?:svg|png))$")


def screenshot_errors(pkg, root):
    """`screenshots:` — at least one; each a title and a raw.githubusercontent.com URL of this repository
    (homeURL's owner/name) naming a file that exists under docs/screenshots."""
    shots = pkg.get("screenshots")
    if not shots:
        return ["missing screenshots"]
    if not isinstance(shots, list):
        return ["screenshots is not a list"]
    home = re.match(r"^https://github\.com/([^/]+)/([^/]+?)/?$", str(pkg.get("homeURL", "")))
    errors = []
    for i, s in enumerate(shots):
        if not isinstance(s, dict) or not str(s.get("title", "")).strip():
            errors.append(f"screenshots[{i}] has no title")
            continue
        url = str(s.get("url", ""))
        m = RAW_RE.match(url)
        if not m:
            errors.append(f"screenshots[{i}] url {url!r} is not a raw.githubusercontent.com docs/screenshots/*.svg|png URL")
            continue
        if home and (m.group(1), m.group(2)) != (home.group(1), home.group(2)):
            errors.append(f"screenshots[{i}] url is not in {home.group(1)}/{home.group(2)} (homeURL)")
        if not os.path.isfile(os.path.join(root, m.group(3))):
            errors.append(f"screenshots[{i}] file {m.group(3)} does not exist")
    return errors


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--tree"]
    errs = validate(args[0] if args else "artifacthub-pkg.yml", tree_digest() if "--tree" in sys.argv[1:] else None)
    for e in errs:
        print(f"::error::{e}")
    if errs:
        sys.exit(1)
    print("artifacthub-pkg.yml valid")
