#!/usr/bin/env python3
"""Derive package-lock.json from the reference plugin's resolved tree (offline).

This build container has no npm registry, so `npm install` cannot resolve a
tree here. The reference plugin commits a lockfile (lockfileVersion 3) that
resolves exactly the toolchain this plugin pins in package.json:
@kinvolk/headlamp-plugin 0.13.1, react / react-dom 18.3.1, vitest 3.2.4,
jsdom 24.1.3, @testing-library/* and react-router-dom 5.3.4. The lock here
is that tree with

* the root entry rewritten from OUR package.json (name, version, license,
  bin, engines, dependency specs), and
* every package no longer reachable from our root dropped (the reference's
  root also lists @playwright/test, which this plugin does not use),

following npm's resolution (a dependency of `a/node_modules/b` is looked up in
`a/node_modules/b/node_modules`, then each ancestor's `node_modules`, then the
top level). Nothing is downloaded and no entry's resolved URL or integrity
hash is changed.

    python tools/derive_lock.py [--check]

`--check` exits 1 when the committed lock differs from a fresh derivation.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE_LOCK = os.environ.get("REFERENCE_LOCK", "/root/reference/package-lock.json")
ROOT_FIELDS = ("name", "version", "license", "bin", "engines", "dependencies", "devDependencies",
               "peerDependencies", "optionalDependencies")


def resolve(packages, from_path, dep):
    """Path of the package `dep` as required from the package at `from_path` ('' = root)."""
    base = from_path
    while True:
        cand = (base + "/" if base else "") + "node_modules/" + dep
        if cand in packages:
            return cand
        if not base:
            return None
        # strip the last "node_modules/<name>" (scoped names have a slash)
        i = base.rfind("node_modules/")
        base = base[:i].rstrip("/") if i > 0 else ""


def reachable(packages, root_deps):
    seen = set()
    stack = [("", d) for d in root_deps]
    while stack:
        frm, dep = stack.pop()
        path = resolve(packages, frm, dep)
        if path is None or path in seen:
            continue
        seen.add(path)
        ent = packages[path]
        if ent.get("link"):
            tgt = ent.get("resolved")
            if tgt and tgt in packages and tgt not in seen:
                seen.add(tgt)
        for field in ("dependencies", "optionalDependencies", "peerDependencies"):
            for d in ent.get(field, {}):
                optional_peer = ent.get("peerDependenciesMeta", {}).get(d, {}).get("optional")
                if field == "peerDependencies" and optional_peer:
                    continue
                stack.append((path, d))
    return seen


def derive(ref_lock, pkg):
    packages = ref_lock["packages"]
    root = {k: pkg[k] for k in ROOT_FIELDS if k in pkg}
    deps = list(pkg.get("dependencies", {})) + list(pkg.get("devDependencies", {})) + list(pkg.get("peerDependencies", {}))
    missing = [d for d in deps if resolve(packages, "", d) is None]
    if missing:
        raise SystemExit(f"not in the reference tree: {missing}")
    keep = reachable(packages, deps)
    out = {"name": pkg["name"], "version": pkg["version"], "lockfileVersion": ref_lock["lockfileVersion"],
           "requires": True, "packages": {"": root}}
    for path, ent in packages.items():
        if path and path in keep:
            out["packages"][path] = ent
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    pkg = json.load(open(os.path.join(ROOT, "package.json")))
    lock = derive(json.load(open(REFERENCE_LOCK)), pkg)
    text = json.dumps(lock, indent=2) + "\n"
    path = os.path.join(ROOT, "package-lock.json")
    if a.check:
        same = os.path.exists(path) and open(path).read() == text
        print("package-lock.json is current" if same else "package-lock.json differs from a fresh derivation")
        return 0 if same else 1
    with open(path, "w") as f:
        f.write(text)
    print(f"package-lock.json: {len(lock['packages']) - 1} packages")
    return 0


if __name__ == "__main__":
    sys.exit(main())
