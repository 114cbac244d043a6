#!/usr/bin/env python3
"""Scaling curve + BASELINE configs: run bench.py per point and tabulate.

    python tools/sweep.py --out gpurun_out/sweep [--steps 30] [--rtt-ms 20]

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
          ("preset", "cpu-only"), ("preset", "1x1"), ("preset", "1x8"), ("preset", "4x8"), ("preset", "8x8")]

PRESET_LABEL = {
    "cpu-only": "#1 CPU-only cluster, 0 GPU nodes",
    "1x1": "#2 single 1×MI355X node",
    "1x8": "#3 single 8×MI355X node, 4 GPU pods",
    "4x8": "#4 4 nodes × 8 MI355X + exporter",
    "8x8": "#5 8 nodes × 8 MI355X (detail/columns)",
}


def run(kind, val, args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--rtt-ms", str(args.rtt_ms), f"--{kind}", val]
    if args.extra:
        cmd += args.extra.split()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)} failed:\n{r.stderr[-3000:]}")
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


PAGE_COLS = [("overview", "Overview"), ("devicePlugins", "Device Plugins"), ("nodes", "GPU Nodes"),
             ("pods", "GPU Pods"), ("metrics", "Metrics")]


def table(rows):
    """Markdown table led by the per-page Refresh-click p50s (reference → new)."""
    head = ["Config", "GPU nodes"] + [f"{t} ref → new (ms)" for _, t in PAGE_COLS] + [
        "Mean per page ref → new (ms)", "Speed-up", "All-pages composite ref → new (ms)",
        "Cold open ref → new (ms)", "Route switch ref → new (ms)", "GPU nodes rendered", "GPU pods rendered",
        "GPUs monitored", "Live GPU telemetry"]
    md = ["| " + " | ".join(head) + " |", "|---|---:|" + "---|" * (len(head) - 2)]
    for r in rows:
        l = r["line"]
        pp = l["per_page_refresh_p50_ms"]
        comp = l["all_pages_refresh"]
        label = f"{r['point']}-node scaling point" if r["kind"] == "nodes" else PRESET_LABEL[r["point"]]
        cells = [label, str(l["config"]["nodes"])]
        cells += [f"{pp[k]['reference']:.1f} → {pp[k]['amd']:.1f}" for k, _ in PAGE_COLS]
        cells += [f"{l['baseline']['value_ms']:.1f} → {l['value']:.1f}", f"{l['baseline']['value_ms'] / l['value']:.1f}×",
                  f"{comp['reference_p50_ms']:.1f} → {comp['amd_p50_ms']:.1f}",
                  f"{l['cold_open_p50_ms']['reference']:.0f} → {l['cold_open_p50_ms']['amd']:.0f}",
                  f"{l['route_switch_p50_ms']['reference']:.0f} → {l['route_switch_p50_ms']['amd']:.1f}",
                  str(l["rendered"]["gpu_nodes"]), str(l["rendered"]["gpu_pods"]), str(l["rendered"]["gpus_monitored"]),
                  "yes" if l.get("live_telemetry") else "no"]
        md.append("| " + " | ".join(cells) + " |")
    return md


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="gpurun_out/sweep")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rtt-ms", type=float, default=20.0)
    p.add_argument("--extra", default="")
    args = p.parse_args()
    os.makedirs(args.out, exist_ok=True)
    rows = []
    for kind, val in POINTS:
        line = run(kind, val, args)
        rows.append({"kind": kind, "point": val, "line": line})
        print(f"{kind}={val}: per-page p50 {line['value']} ms vs ref {line['baseline']['value_ms']} ms", flush=True)
        with open(os.path.join(args.out, "sweep.json"), "w") as f:
            json.dump(rows, f, indent=1)
    md = table(rows)
    with open(os.path.join(args.out, "sweep.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
