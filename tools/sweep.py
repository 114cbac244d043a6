#!/usr/bin/env python3
"""Scaling curve + BASELINE configs: run bench.py per point and tabulate.

    python tools/sweep.py --out gpurun_out/sweep [--steps 30] [--rtt-ms 20] [--beyond 16,32,64,256,1000]
    python tools/sweep.py --stress --out gpurun_out/stress [--stress-nodes 16,64,256,1000] [--events 1000]

``--stress``: the cluster-size axis under watch churn (bench/stress.js) —
16/64/256/1000 GPU nodes × 8, 30 plain pods per node, 50 pod watch events/s —
per delivery mode (identity / rewrapped / reparsed): CPU ms per event for the
shipped store + all five page view-models vs a replay of the reference's
per-event recompute, per event kind, heap growth and list bytes. Writes
``stress.json`` and ``stress.md``.

Points: synthetic clusters of 1, 2, 4 and 8 nodes × 8 MI355X (one process,
``--nodes N``) and the five BASELINE.json presets. Writes ``sweep.json`` and
``sweep.md`` (the table that goes into BASELINE.md).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

POINTS = [("nodes", "1"), ("nodes", "2"), ("nodes", "4"), ("nodes", "8"),
          ("preset", "cpu-only"), ("preset", "1x1"), ("preset", "1x8"), ("preset", "4x8"), ("preset", "8x8"),
          ("hwmon", "8")]

PRESET_LABEL = {
    "cpu-only": "#1 CPU-only cluster, 0 GPU nodes",
    "1x1": "#2 single 1×MI355X node",
    "1x8": "#3 single 8×MI355X node, 4 GPU pods",
    "4x8": "#4 4 nodes × 8 MI355X + exporter",
    "8x8": "#5 8 nodes × 8 MI355X (detail/columns)",
}


def label_of(r):
    if r["kind"] == "nodes":
        return f"{r['point']}-node scaling point"
    if r["kind"] == "hwmon":
        return f"{r['point']} nodes × 8 MI355X, node-exporter hwmon only (no exporter series)"
    return PRESET_LABEL[r["point"]]


def run(kind, val, args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--rtt-ms", str(args.rtt_ms)]
    # hwmon: a cluster whose Prometheus holds node-exporter's amdgpu series only (the plugin's fallback source)
    cmd += ["--nodes", val, "--source", "node-exporter"] if kind == "hwmon" else [f"--{kind}", val]
    if args.extra:
        cmd += args.extra.split()
    # bench progress lines (stderr) pass through: a long point stays visibly alive
    r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, text=True, timeout=1800)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)} failed (rc {r.returncode}); see its stderr above")
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


PAGE_COLS = [("overview", "Overview"), ("devicePlugins", "Device Plugins"), ("nodes", "GPU Nodes"),
             ("pods", "GPU Pods"), ("metrics", "Metrics")]


def cold_mean(line):
    cp = line.get("cold_open_per_page_p50_ms")
    if not cp:
        return "—"
    ref = sum(v["reference"] for v in cp.values()) / len(cp)
    amd = sum(v["amd"] for v in cp.values()) / len(cp)
    return f"{ref:.0f} → {amd:.0f}"


def table(rows):
    """Markdown table led by the per-page Refresh-click p50s (reference → new)."""
    head = ["Config", "GPU nodes"] + [f"{t} ref → new (ms)" for _, t in PAGE_COLS] + [
        "Mean per page ref → new (ms)", "Speed-up", "All-pages composite ref → new (ms)",
        "Cold open, mean per page ref → new (ms)", "Cold open, all pages ref → new (ms)", "Route switch ref → new (ms)",
        "GPU nodes rendered", "GPU pods rendered",
        "GPUs monitored", "Live GPU telemetry"]
    md = ["| " + " | ".join(head) + " |", "|---|---:|" + "---|" * (len(head) - 2)]
    for r in rows:
        l = r["line"]
        pp = l["per_page_refresh_p50_ms"]
        comp = l["all_pages_refresh"]
        label = label_of(r)
        cells = [label, str(l["config"]["nodes"])]
        cells += [f"{pp[k]['reference']:.1f} → {pp[k]['amd']:.1f}" for k, _ in PAGE_COLS]
        cells += [f"{l['baseline']['value_ms']:.1f} → {l['value']:.1f}", f"{l['baseline']['value_ms'] / l['value']:.1f}×",
                  f"{comp['reference_p50_ms']:.1f} → {comp['amd_p50_ms']:.1f}",
                  cold_mean(l),
                  f"{l['cold_open_p50_ms']['reference']:.0f} → {l['cold_open_p50_ms']['amd']:.0f}"
                  + server_share(l["cold_open_p50_ms"].get("amd_server_ms"), l["cold_open_p50_ms"]["amd"]),
                  f"{l['route_switch_p50_ms']['reference']:.0f} → {l['route_switch_p50_ms']['amd']:.1f}",
                  str(l["rendered"]["gpu_nodes"]), str(l["rendered"]["gpu_pods"]), str(l["rendered"]["gpus_monitored"]),
                  "yes" if l.get("live_telemetry") else "no"]
        md.append("| " + " | ".join(cells) + " |")
    return md


#: A figure whose fake-server share (X-Server-Ms of its slowest request) is above this measures the harness.
SERVER_SHARE_FLAG = 0.25


def server_share(server_ms, figure_ms):
    """'s N%' — the fake server's share of a figure — with ⚠ above SERVER_SHARE_FLAG; '' when unknown."""
    if server_ms is None or not figure_ms:
        return ""
    share = server_ms / figure_ms
    return f", s {share * 100:.0f}%" + (" ⚠" if share > SERVER_SHARE_FLAG else "")


def cold_table(rows):
    """Per page at each point: cold open, reference → new first content / new complete (ms), the new open's
    Prometheus requests (query + query_range + probe), and the fake server's share of the new complete figure
    (``s N%``: the open's slowest request's own server time over the figure; ⚠ above SERVER_SHARE_FLAG)."""
    head = ["Config", "GPU nodes"] + [f"{t}: ref → first / complete (ms), Prometheus requests, server share"
                                      for _, t in PAGE_COLS]
    md = ["| " + " | ".join(head) + " |", "|---|---:|" + "---|" * (len(head) - 2)]
    for r in rows:
        l = r["line"]
        cp = l.get("cold_open_per_page_p50_ms") or {}
        label = label_of(r)
        cells = [label, str(l["config"]["nodes"])]
        for k, _ in PAGE_COLS:
            v = cp.get(k)
            if not v or "amd_first_content" not in v:
                cells.append("—")
                continue
            by = v.get("amd_requests_by_kind") or {}
            prom = sum(by.get(x, 0) for x in ("query", "query_range", "probe"))
            cells.append(f"{v['reference']:.0f} → {v['amd_first_content']:.0f} / {v['amd']:.0f}, {prom}"
                         + server_share(v.get("amd_server_ms"), v["amd"]))
        md.append("| " + " | ".join(cells) + " |")
    return md


def render_table(rows):
    """Per page at each point: harness-React elements and mount / re-render ms, plus the cold Node detail open."""
    head = ["GPU nodes"] + [f"{t}: elements, mount / re-render ms" for _, t in PAGE_COLS] + [
        "Cold Node detail ref → new: ms, KB, requests",
        "Node detail after a page, as wired: ms, KB, requests, list hooks (cluster-wide)"]
    md = ["| " + " | ".join(head) + " |", "|---:|" + "---|" * (len(head) - 1)]
    for r in rows:
        l = r["line"]
        rp = l.get("render_per_page") or {}
        cells = [str(l["config"]["nodes"])]
        for k, _ in PAGE_COLS:
            v = rp.get(k)
            cells.append(f"{v['elements']}, {v['mount_ms']:.1f} / {v['rerender_ms']:.1f}" if v else "—")
        d = l.get("detail_open") or {}
        a, ref = d.get("nodeDetailCold"), d.get("nodeDetailColdReference")
        cells.append(f"{ref['p50_ms']:.0f} → {a['p50_ms']:.0f}; {ref['bytes'] / 1e3:.0f} → {a['bytes'] / 1e3:.0f}; "
                     f"{ref['requests']:.0f} → {a['requests']:.0f}" if a and ref and a["p50_ms"] is not None else "—")
        w = d.get("nodeDetailWired")
        cells.append(f"{w['p50_ms']:.0f}; {w['bytes'] / 1e3:.0f}; {w['requests']:.0f}; {w.get('lists', 0):.0f} "
                     f"({w.get('cluster_wide_lists', 0):.0f})" if w and w.get("p50_ms") is not None else "—")
        md.append("| " + " | ".join(cells) + " |")
    return md


def react_dom_table(rows):
    """Per page at each point: real React 18.3.1 (production) elements and mount / re-render ms."""
    if not any(r["line"].get("render_per_page_react_dom") for r in rows):
        return []
    head = ["GPU nodes"] + [f"{t}: elements, mount / re-render ms" for _, t in PAGE_COLS]
    md = ["", "Render on real React 18.3.1 + react-dom (production UMD builds, minimal JS DOM, median of 9):", "",
          "| " + " | ".join(head) + " |", "|---:|" + "---|" * (len(head) - 1)]
    for r in rows:
        rp = r["line"].get("render_per_page_react_dom") or {}
        cells = [str(r["line"]["config"]["nodes"])]
        for k, _ in PAGE_COLS:
            v = rp.get(k)
            cells.append(f"{v['elements']}, {v['mount_ms']:.1f} / {v['rerender_ms']:.1f}" if v else "—")
        md.append("| " + " | ".join(cells) + " |")
    return md


MODES = ["identity", "rewrapped", "reparsed"]
KINDS = ["modified", "gpu-modified", "added", "gpu-added", "deleted", "gpu-deleted"]


def stress(args):
    os.makedirs(args.out, exist_ok=True)
    res = {}
    for mode in MODES:
        out = os.path.join(args.out, f"stress_{mode}.json")
        cmd = ["node", "--expose-gc", os.path.join(ROOT, "bench", "stress.js"), "--nodes", args.stress_nodes,
               "--events", str(args.events), "--rate", "50", "--mode", mode, "--out", out]
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=1800)
        if r.returncode != 0:
            raise RuntimeError(f"{' '.join(cmd)} failed:\n{r.stderr[-3000:]}")
        print(r.stderr.strip(), flush=True)
        res[mode] = json.load(open(out))
    with open(os.path.join(args.out, "stress.json"), "w") as f:
        json.dump(res, f, indent=1)
    md = ["| Delivery | GPU nodes | Pods | Events | New p50 / p95 / mean (ms) | Reference replay p50 / p95 (ms) | "
          "p50 speed-up | Index rebuilds / patches | Heap growth (MB) | Pod list (MB) |",
          "|---|---:|---:|---:|---|---|---:|---|---:|---:|"]
    for mode in MODES:
        for p in res[mode]["points"]:
            a, ref = p["amd"], p["reference"]
            c = p["storeCounters"]
            md.append(f"| {mode} | {p['nodes']} | {p['pods']} | {p['events']} | {a['p50']:.3f} / {a['p95']:.3f} / "
                      f"{a['mean']:.3f} | {ref['p50']:.2f} / {ref['p95']:.2f} | {ref['p50'] / a['p50']:.0f}× | "
                      f"{c['indexBuilds']} / {c['indexPatches']} | {p['heapGrowthBytes'] / 1e6:.1f} | "
                      f"{p['podListBytes'] / 1e6:.1f} |")
    md += ["", "Per event kind, identity delivery (new p50 / p95 ms):", "",
           "| GPU nodes | " + " | ".join(KINDS) + " |", "|---:|" + "---|" * len(KINDS)]
    for p in res["identity"]["points"]:
        cells = []
        for k in KINDS:
            v = p["amdByKind"].get(k)
            cells.append(f"{v['p50']:.3f} / {v['p95']:.3f} (n={v['n']})" if v else "—")
        md.append(f"| {p['nodes']} | " + " | ".join(cells) + " |")
    with open(os.path.join(args.out, "stress.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="gpurun_out/sweep")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rtt-ms", type=float, default=20.0)
    p.add_argument("--extra", default="")
    p.add_argument("--stress", action="store_true", help="watch-churn stress of the cluster-size axis instead")
    p.add_argument("--stress-nodes", default="16,64,256,1000")
    p.add_argument("--events", type=int, default=1000)
    p.add_argument("--beyond", default="", help="extra node counts past the BASELINE configs, e.g. 16,32,64,256,1000; hN = N nodes, node-exporter hwmon only")
    p.add_argument("--only-beyond", action="store_true", help="skip the BASELINE points (run --beyond only)")
    args = p.parse_args()
    if args.stress:
        return stress(args)
    os.makedirs(args.out, exist_ok=True)
    rows = []
    # --beyond 16,64,h256: "hN" is an N-node cluster whose Prometheus holds node-exporter's hwmon series only
    points = ([] if args.only_beyond else POINTS) + [("hwmon", v.strip()[1:]) if v.strip().startswith("h") else ("nodes", v.strip())
                                                     for v in args.beyond.split(",") if v.strip()]
    for kind, val in points:
        line = run(kind, val, args)
        rows.append({"kind": kind, "point": val, "line": line})
        print(f"{kind}={val}: per-page p50 {line['value']} ms vs ref {line['baseline']['value_ms']} ms", flush=True)
        with open(os.path.join(args.out, "sweep.json"), "w") as f:
            json.dump(rows, f, indent=1)
    md = (table(rows) + ["", "Cold open per page (progressive: a page renders once the lists it draws are in):", ""]
          + cold_table(rows) + ["", "Render (harness React, first page of each view) and the cold Node detail open:", ""]
          + render_table(rows) + react_dom_table(rows))
    with open(os.path.join(args.out, "sweep.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
