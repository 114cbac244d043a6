#!/usr/bin/env python3
"""Validate artifacthub-pkg.yml (required fields, SemVer, archive annotations, screenshots).

Used by CI; exits non-zero with one line per problem.
"""
import os
import re
import sys

import yaml


def validate(path="artifacthub-pkg.yml"):
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
    errs = validate(sys.argv[1] if len(sys.argv) > 1 else "artifacthub-pkg.yml")
    for e in errs:
        print(f"::error::{e}")
    if errs:
        sys.exit(1)
    print("artifacthub-pkg.yml valid")
