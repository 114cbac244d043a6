"""Render every plugin view of a synthetic MI355X cluster to static HTML and SVG.

    python tools/screenshots.py [--nodes 2] [--out docs/screenshots]

The reference ships hand-drawn SVG mock-ups (docs/screenshots/*.svg, published
through artifacthub-pkg.yml's `screenshots:`); these are the real view-models
(src/view/pages/*.js) of a fake 2-node cluster, rendered through
src/view/html.js — the same path the benchmark counts rows on — and drawn by
src/view/svg.js as the pictures ArtifactHub and the README show, so they stay
in sync with the code.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from headlamp_intel_gpu_plugin_amd.models.cluster import EPOCH  # noqa: E402
from headlamp_intel_gpu_plugin_amd.sim.apiserver import ServerThread, make_fake  # noqa: E402
from headlamp_intel_gpu_plugin_amd.utils.nodebridge import Driver  # noqa: E402

# Fixed clock one day after the synthetic cluster epoch, so ages render deterministically.
NOW_MS = int((EPOCH.timestamp() + 86400) * 1000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "docs", "screenshots"))
    a = ap.parse_args()
    # Reproducible files: Prometheus evaluates at the same instant the data layer's clock reads, and "Last
    # Fetched" (browser-local time) is rendered in UTC.
    os.environ["TZ"] = "UTC"
    fc = make_fake(a.nodes, source="amd-exporter", latency_ms=0)
    fc.now = lambda: NOW_MS / 1000.0
    with ServerThread(fc) as srv, Driver(srv.url) as d:
        files = d.call("snapshot", dir=os.path.abspath(a.out), now=NOW_MS)["files"]
    for f in files:
        print(os.path.relpath(f, ROOT))


if __name__ == "__main__":
    main()
