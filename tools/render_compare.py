#!/usr/bin/env python3
"""The reference's own pages vs this plugin's, rendered on real React 18.3.1 at 1 to 1,000 GPU nodes.

    python tools/render_compare.py --allow-reference-exec [--sizes 1,2,4,8] [--reps 101] [--warm 50] [--runs 3]
                                   [--out profiles/r5_render_compare]

OPT-IN: this runs the reference's page components, which are untrusted public content (ADR 014). Without
``--allow-reference-exec`` it refuses. With it, bench/driver.js (this plugin's pages) starts the process that runs the
reference's (bench/refIsolated.js): no network, read-only mounts, no capabilities, no file it can open, V8's
``--disallow-code-generation-from-strings``; inside it the reference's modules, React and the DOM stand-in are built
from source text in a realm of their own (bench/refWorker.cjs), with no ``process``, ``require``, ``import()``,
timers, file system or network, and no code generation from strings. It gets text and answers with numbers.

Per page and size: ``--warm`` untimed mounts of each side, then ``--reps`` (at least 15) interleaved
reference / new pairs, the order alternating; mount and re-render p50 with the interquartile range. ``--runs``
driver processes measure each size, and their samples are pooled: a process's JIT and heap state moves every figure
it takes, so one process is one draw of that state.

Per size: the fake control plane (no injected latency: this measures render, not requests) serves a synthetic
cluster; bench/driver.js ``refRender`` mounts each of the five reference pages — read unmodified from
``--reference`` (default /root/reference) and transpiled at run time by bench/tsx.js — and each of this plugin's,
on the react@18.3.1 / react-dom@18.3.1 production UMD builds (bench/referenceRender.js has the data mapping).
Writes ``<out>.json`` and ``<out>.md``.

The reference's sources are not in this repository and not on the GPU box, so this runs where they are (this
container's CPU); the figures of both plugins come from the same host, each side's from its own process, the pairs
interleaved. Both processes also mount one calibration tree (a 100-row table) on their own React, so the two
environments' speed is on record next to the figures.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PAGES = [("overview", "Overview"), ("devicePlugins", "Device Plugins"), ("nodes", "GPU Nodes"), ("pods", "GPU Pods"),
         ("metrics", "Metrics")]


def measure(n: int, reference: str, reps: int, warm: int, pages=None) -> dict:
    from headlamp_intel_gpu_plugin_amd.sim.serve import ControlPlaneProcess
    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import Driver
    from headlamp_intel_gpu_plugin_amd.utils.reactumd import PROD_BUILDS, umd_dir

    umd = umd_dir(PROD_BUILDS)
    if not umd:
        raise SystemExit("the React 18.3.1 production UMD builds are not available in this image")
    with ControlPlaneProcess(n, source="both", latency_ms=0.0) as srv:
        drv = Driver(srv.url, node_flags=["--disallow-code-generation-from-strings"],
                     env={"PATH": os.environ.get("PATH", "/usr/bin:/bin")})
        try:
            r = drv.call("refRender", referenceDir=reference, umdDir=umd, reps=reps, warm=warm, allowReferenceExec=True,
                         pages=pages, timeout=3000)
        finally:
            drv.close()
    if r.get("error"):
        raise RuntimeError(r["error"])
    return r["render"]


def quantile(xs, p):
    v = sorted(xs)
    idx = (len(v) - 1) * p
    lo, hi = int(idx), min(int(idx) + 1, len(v) - 1)
    return v[lo] + (v[hi] - v[lo]) * (idx - lo)


def pooled(runs: list) -> dict:
    """One size's result from several driver processes: each page's samples pooled, p50 / IQR recomputed."""
    out = {k: v for k, v in runs[0].items() if k != "pages"}
    out["runs"] = len(runs)
    cal = [r["calibration"] for r in runs if "calibration" in r]
    if cal:
        out["calibration"] = {"rows": cal[0]["rows"], "elements": cal[0]["elements"],
                              "referenceRealmMs": [c["referenceRealmMs"] for c in cal],
                              "driverRealmMs": [c["driverRealmMs"] for c in cal]}
    out["pages"] = {}
    for page in runs[0]["pages"]:
        per = [r["pages"][page] for r in runs]
        res = {}
        for side in ("reference", "amd"):
            mount = [x for p in per for x in p["samples"][side]["mount"]]
            rer = [x for p in per for x in p["samples"][side]["rerender"]]
            res[side] = {"elements": per[0][side]["elements"], "reps": len(mount),
                         "mountMs": quantile(mount, 0.5), "mountQ1": quantile(mount, 0.25), "mountQ3": quantile(mount, 0.75),
                         "rerenderMs": quantile(rer, 0.5), "rerenderQ1": quantile(rer, 0.25), "rerenderQ3": quantile(rer, 0.75)}
        res["amd"]["reactOnlyMs"] = quantile([x for p in per for x in p["samples"]["prebuilt"]["mount"]], 0.5)
        res["amd"]["vmBuildMs"] = quantile([x for p in per for x in p["samples"]["prebuilt"]["vm"]], 0.5)
        # each process's own p50s, to show the spread between processes
        res["amd"]["runMountMs"] = [p["amd"]["mountMs"] for p in per]
        res["reference"]["runMountMs"] = [p["reference"]["mountMs"] for p in per]
        out["pages"][page] = res
    return out


def verdict(a: dict, ref: dict) -> str:
    """'≤' when the new mount p50 is at most the reference's, '≈' within its interquartile range, else '>'."""
    if a["mountMs"] <= ref["mountMs"]:
        return "≤"
    return "≈" if a["mountMs"] <= ref.get("mountQ3", ref["mountMs"]) else ">"


def table(rows) -> list:
    head = ["GPU nodes", "GPU pods"] + [f"{t}: elements ref → new; mount p50 [IQR] ref → new (ms); re-render p50 ref → new"
                                        for _, t in PAGES] + ["Reference provider filter per watch event (ms)",
                                                              "Calibration tree mount, reference's realm / driver's (ms)"]
    md = ["| " + " | ".join(head) + " |", "|---:|---:|" + "---|" * (len(head) - 2)]
    for n, r in rows:
        cells = [str(n), str(r["gpuPods"])]
        for k, _ in PAGES:
            a, ref = r["pages"][k]["amd"], r["pages"][k]["reference"]
            iqr = lambda x: f"[{x['mountQ1']:.2f}–{x['mountQ3']:.2f}]" if "mountQ1" in x else ""
            split = f" (vm {a['vmBuildMs']:.2f} + React {a['reactOnlyMs']:.2f})" if "vmBuildMs" in a else ""
            cells.append(f"{ref['elements']} → {a['elements']}; {ref['mountMs']:.2f} {iqr(ref)} → {a['mountMs']:.2f} {iqr(a)} "
                         f"{verdict(a, ref)}{split}; {ref['rerenderMs']:.2f} → {a['rerenderMs']:.2f}")
        cells.append(f"{r['referenceProviderFilterMs']:.1f}")
        cal = r.get("calibration")
        cells.append(" · ".join(f"{a:.2f} / {b:.2f}" for a, b in zip(cal["referenceRealmMs"], cal["driverRealmMs"])) if cal else "—")
        md.append("| " + " | ".join(cells) + " |")
    return md


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--sizes", default="1,2,4,8")
    p.add_argument("--reps", type=int, default=101)
    p.add_argument("--warm", type=int, default=50)
    p.add_argument("--runs", type=int, default=3, help="driver processes per size, their samples pooled")
    p.add_argument("--reference", default="/root/reference")
    p.add_argument("--pages", default=None, help="comma-separated page keys (default: all five); a partial run prints no table")
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "r5_render_compare"))
    p.add_argument("--allow-reference-exec", action="store_true",
                   help="run the reference's page components (untrusted) in the isolated worker process")
    args = p.parse_args()
    if not args.allow_reference_exec:
        raise SystemExit("render_compare runs the reference's sources (untrusted public content): "
                         "pass --allow-reference-exec to run them in the isolated worker process (ADR 014)")
    if not os.path.isdir(os.path.join(args.reference, "src", "components")):
        raise SystemExit(f"no reference sources under {args.reference}")
    rows = []
    for s in args.sizes.split(","):
        n = int(s)
        t = time.time()
        pages = args.pages.split(",") if args.pages else None
        r = pooled([measure(n, args.reference, args.reps, args.warm, pages) for _ in range(max(1, args.runs))])
        if pages:
            for k, v in r["pages"].items():
                a, ref = v["amd"], v["reference"]
                print(f"[render_compare] {n} nodes {k}: ref {ref['mountMs']:.3f} [{ref['mountQ1']:.3f}-{ref['mountQ3']:.3f}] "
                      f"({ref['elements']} el) new {a['mountMs']:.3f} [{a['mountQ1']:.3f}-{a['mountQ3']:.3f}] ({a['elements']} el) "
                      f"{verdict(a, ref)} vm {a['vmBuildMs']:.3f} react {a['reactOnlyMs']:.3f}; cal {r.get('calibration')}",
                      file=sys.stderr, flush=True)
            continue
        rows.append((n, r))
        print(f"[render_compare] {n} nodes: {time.time() - t:.1f} s", file=sys.stderr, flush=True)
        with open(args.out + ".json", "w") as f:
            json.dump({"host": os.uname().nodename, "node": "v12", "rows": [{"gpu_nodes": n, **r} for n, r in rows]}, f,
                      indent=1)
    md = ["Each page mounted on react@18.3.1 + react-dom@18.3.1 production UMD builds into a minimal JS DOM: "
          f"{args.warm} untimed warm mounts of each side, then {max(15, args.reps)} interleaved reference / new pairs "
          f"(order alternating), in each of {max(1, args.runs)} driver processes, samples pooled; p50 with the "
          "interquartile range. ≤: new p50 at most the reference's; ≈: within its "
          "IQR; >: above it. Reference = its page component (read from its sources, transpiled at run time) with "
          "its data in context, its per-render aggregation included; re-render = a watch event (a new context "
          "value). New = this plugin's page, mount including the view-model built from a cold memo; re-render = "
          "the same watch event (a new store snapshot of the same data). First page of each pager. The last column "
          "is the reference provider's re-filtering of both whole lists on every watch event "
          "(IntelGpuDataContext.tsx:200-208), on top of the page's re-render.", ""] + table(rows)
    with open(args.out + ".md", "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))
    return 0


if __name__ == "__main__":
    sys.exit(main())
