#!/usr/bin/env python3
"""A/B of the plugin's cold page opens on a large cluster: two commits, one fake control plane, CPU profiles.

    python tools/ab_cold_open.py [--base ee2699e] [--nodes 1000] [--opens 5] [--rounds 2]
                                 [--out profiles/r6_ab_cold1k_cpu]

Checks the base commit out into a git worktree, starts ONE fake control plane (this tree's: the same server for both
sides, no injected latency), and runs each side's own bench/driver.js ``coldPages`` (a fresh schedule per open:
empty caches, a new client; every page, ``--opens`` times) under ``node --cpu-prof``, alternating base / head for
``--rounds`` rounds. Reports per page the p50 of first content / content / complete (ms), and each side's CPU self
time grouped by where the code lives: the plugin's arrival facts, cluster index, list tracking and store,
telemetry client, views; the bench's response decode; Node internals; GC and idle.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary  # noqa: E402

PAGES = ["overview", "devicePlugins", "nodes", "pods", "metrics"]

# Where a function's self time goes, by the file it lives in (first match wins).
GROUPS = [
    ("arrival facts", ("src/api/amdPods.js", "src/api/amdNodes.js", "src/api/operatorFacts.js", "src/api/nodeSummaries.js",
                       "src/api/derivedCache.js", "src/api/k8sCore.js", "src/api/topology.js")),
    ("cluster index", ("src/api/clusterIndex.js",)),
    ("lists + store", ("src/api/listCache.js", "src/api/clusterStore.js", "src/api/providerCore.js", "src/api/selectors.js",
                       "src/api/requests.js", "src/api/cluster.js", "src/api/settings.js")),
    ("telemetry client", ("src/api/metrics.js", "src/api/promClient.js", "src/api/promql.js", "src/api/telemetry.js",
                          "src/api/clusterSnapshots.js", "src/api/scopedSnapshots.js", "src/api/ownerSnapshots.js",
                          "src/api/seriesFetch.js", "src/api/series.js")),
    ("views", ("src/view/",)),
    ("bench: response decode", ("bench/common.js",)),
    ("bench: other", ("bench/",)),
]


def group_of(url: str, fn: str) -> str:
    if fn in ("(garbage collector)",):
        return "GC"
    if fn in ("(idle)", "(program)", "(root)"):
        return "idle / program"
    for name, prefixes in GROUPS:
        if any(p in url for p in prefixes):
            return name
    if "/src/" in url:
        return "other plugin"
    return "Node internals / V8"


def self_times(profile_path: str) -> dict:
    prof = json.load(open(profile_path))
    nodes = {n["id"]: n for n in prof["nodes"]}
    dt = {}
    for sid, d in zip(prof.get("samples", []), prof.get("timeDeltas", [])):
        dt[sid] = dt.get(sid, 0) + d
    out = {}
    for nid, us in dt.items():
        cf = nodes[nid]["callFrame"]
        g = group_of(cf.get("url", ""), cf.get("functionName", ""))
        out[g] = out.get(g, 0.0) + us / 1000.0
    return out


def top_functions(profile_path: str, k: int = 8) -> list:
    prof = json.load(open(profile_path))
    nodes = {n["id"]: n for n in prof["nodes"]}
    acc = {}
    for sid, d in zip(prof.get("samples", []), prof.get("timeDeltas", [])):
        cf = nodes[sid]["callFrame"]
        url = cf.get("url", "")
        if "/src/" not in url:
            continue
        key = f"{cf.get('functionName') or '(anonymous)'} ({url.split('/src/')[1]}:{cf.get('lineNumber', 0) + 1})"
        acc[key] = acc.get(key, 0) + d / 1000.0
    return sorted(acc.items(), key=lambda kv: -kv[1])[:k]


def run_side(tree: str, url: str, opens: int, prof_dir: str) -> dict:
    os.makedirs(prof_dir, exist_ok=True)
    p = subprocess.Popen([node_binary(), "--cpu-prof", f"--cpu-prof-dir={prof_dir}", os.path.join(tree, "bench", "driver.js"),
                          "--serve", "--url", url], cwd=tree, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, bufsize=1)
    p.stdin.write(json.dumps({"cmd": "coldPages", "schedule": "amd", "n": opens}) + "\n")
    p.stdin.flush()
    line = p.stdout.readline()
    p.stdin.write(json.dumps({"cmd": "quit"}) + "\n")
    p.stdin.flush()
    p.wait(120)
    out = json.loads(line)
    if "error" in out:
        raise RuntimeError(out["error"])
    return out["pages"]


def p50(xs):
    return statistics.median(xs) if xs else float("nan")


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--base", default="ee2699e")
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--opens", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6_ab_cold1k_cpu"))
    args = ap.parse_args()
    from headlamp_intel_gpu_plugin_amd.sim.serve import ControlPlaneProcess

    base_rev = subprocess.run(["git", "rev-parse", "--short", args.base], cwd=ROOT, capture_output=True, text=True,
                              check=True).stdout.strip()
    head_rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=ROOT, capture_output=True, text=True,
                              check=True).stdout.strip()
    wt = os.path.join(tempfile.gettempdir(), "ab-" + base_rev)
    if not os.path.isdir(wt):
        subprocess.run(["git", "worktree", "add", "-f", wt, base_rev], cwd=ROOT, check=True, capture_output=True)
    sides = {"base": wt, "head": ROOT}
    lat = {s: {p: {"first": [], "content": [], "complete": []} for p in PAGES} for s in sides}
    cpu = {s: {} for s in sides}
    tops = {s: {} for s in sides}
    work = tempfile.mkdtemp(prefix="ab-cold-")
    with ControlPlaneProcess(args.nodes, source="both", latency_ms=0.0) as srv:
        for r in range(args.rounds):
            for s in (["base", "head"] if r % 2 == 0 else ["head", "base"]):
                d = os.path.join(work, f"{s}-{r}")
                pages = run_side(sides[s], srv.url, args.opens, d)
                for p in PAGES:
                    pg = pages[p]
                    # the first open of a process pays module load and JIT warm-up: left out
                    lat[s][p]["first"] += pg["firstMs"][1:]
                    lat[s][p]["content"] += pg["contentMs"][1:]
                    lat[s][p]["complete"] += pg["latencies"][1:]
                for f in glob.glob(os.path.join(d, "*.cpuprofile")):
                    for g, v in self_times(f).items():
                        cpu[s][g] = cpu[s].get(g, 0.0) + v
                    for k, v in top_functions(f, 30):
                        tops[s][k] = tops[s].get(k, 0.0) + v
                print(f"[ab] round {r} {s} done", file=sys.stderr, flush=True)
    res = {"base": base_rev, "head": head_rev, "nodes": args.nodes, "opens": args.opens, "rounds": args.rounds,
           "latency": {s: {p: {k: p50(v) for k, v in lat[s][p].items()} for p in PAGES} for s in sides},
           "cpuMs": cpu, "topPlugin": {s: sorted(tops[s].items(), key=lambda kv: -kv[1])[:12] for s in sides}}
    with open(args.out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    md = [f"A/B at {args.nodes} GPU nodes: base `{base_rev}` vs head `{head_rev}`, each side's own bench/driver.js "
          f"`coldPages` against one fake control plane (no injected latency), {args.opens} cold opens of every page per "
          f"process (the first left out), {args.rounds} processes per side alternating, `node --cpu-prof`.", "",
          "| Page | first content base → head (ms) | content base → head (ms) | complete base → head (ms) |",
          "|---|---:|---:|---:|"]
    for p in PAGES:
        b, h = res["latency"]["base"][p], res["latency"]["head"][p]
        md.append(f"| {p} | {b['first']:.0f} → {h['first']:.0f} | {b['content']:.0f} → {h['content']:.0f} | "
                  f"{b['complete']:.0f} → {h['complete']:.0f} |")
    groups = sorted(set(cpu["base"]) | set(cpu["head"]), key=lambda g: -(cpu["head"].get(g, 0) + cpu["base"].get(g, 0)))
    md += ["", "CPU self time over all opens of both processes of a side (ms):", "",
           "| Where | base | head | head − base |", "|---|---:|---:|---:|"]
    for g in groups:
        b, h = cpu["base"].get(g, 0.0), cpu["head"].get(g, 0.0)
        md.append(f"| {g} | {b:.0f} | {h:.0f} | {h - b:+.0f} |")
    plugin = [g for g in groups if g in {n for n, _ in GROUPS[:5]} or g == "other plugin"]
    pb = sum(cpu["base"].get(g, 0.0) for g in plugin)
    ph = sum(cpu["head"].get(g, 0.0) for g in plugin)
    md.append(f"| **plugin total** | **{pb:.0f}** | **{ph:.0f}** | **{ph - pb:+.0f}** |")
    for s in ("base", "head"):
        md += ["", f"Top plugin functions, {s} (self ms):", ""]
        md += [f"- {k}: {v:.0f}" for k, v in res["topPlugin"][s]]
    with open(args.out + ".md", "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))
    return 0


if __name__ == "__main__":
    sys.exit(main())
