#!/usr/bin/env python3
"""Validate artifacthub-pkg.yml (required fields, SemVer, archive annotations).

Used by CI; exits non-zero with one line per problem.
"""
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
    return errors


if __name__ == "__main__":
    errs = validate(sys.argv[1] if len(sys.argv) > 1 else "artifacthub-pkg.yml")
    for e in errs:
        print(f"::error::{e}")
    if errs:
        sys.exit(1)
    print("artifacthub-pkg.yml valid")
