"""tools/screenshots.py renders every view of a fake cluster through the shipped view-models, to HTML and to the
SVG pictures artifacthub-pkg.yml's `screenshots:` publishes (src/view/svg.js)."""
import os
import subprocess
import sys
import xml.etree.ElementTree as ET

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VIEWS = ["01-overview", "02-device-plugins", "03-gpu-nodes", "04-gpu-pods", "05-metrics", "06-node-detail",
         "07-pod-detail"]
SVG = "{http://www.w3.org/2000/svg}"


def render(out, *args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "screenshots.py"), *args, "--out", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]


def svg_text(path):
    """Every <text> of an SVG file, in document order (parsing it: the file is well-formed XML)."""
    root = ET.parse(path).getroot()
    assert root.tag == SVG + "svg"
    return [t.text or "" for t in root.iter(SVG + "text")]


def test_screenshots_render_every_view(tmp_path):
    render(tmp_path, "--nodes", "2")
    names = sorted(os.listdir(tmp_path))
    assert names == sorted([v + ".html" for v in VIEWS] + [v + ".svg" for v in VIEWS])
    html = {n: (tmp_path / n).read_text() for n in names if n.endswith(".html")}
    assert "<h1>AMD GPU — Overview</h1>" in html["01-overview.html"]
    assert "GPU Node Summary" in html["03-gpu-nodes.html"]
    assert "mi355x-001" in html["03-gpu-nodes.html"]
    assert "<h2>AMD GPU</h2>" in html["06-node-detail.html"]
    assert "<h2>AMD GPU Resources</h2>" in html["07-pod-detail.html"]
    assert "GPU Power Summary" in html["05-metrics.html"]


def test_svg_pictures_draw_the_view_models(tmp_path):
    """The SVGs carry the same page: its title, its section titles and its rows as text; bars and statuses as
    shapes; a size that fits what was drawn."""
    render(tmp_path, "--nodes", "2")
    nodes = svg_text(tmp_path / "03-gpu-nodes.svg")
    assert nodes[0] == "AMD GPU — Nodes"
    for want in ("GPU Node Summary", "mi355x-000", "mi355x-001", "Hottest GPU", "Show xGMI matrix"):
        assert want in nodes, want
    assert any(t.startswith("GPU 0 ml/train-000-0") for t in nodes)  # the slot strip's owners
    assert svg_text(tmp_path / "01-overview.svg")[0] == "AMD GPU — Overview"
    assert "Plugin Daemon Pods" in svg_text(tmp_path / "02-device-plugins.svg")
    assert "GPU Power Summary" in svg_text(tmp_path / "05-metrics.svg")
    assert "AMD GPU" in svg_text(tmp_path / "06-node-detail.svg")
    root = ET.parse(tmp_path / "03-gpu-nodes.svg").getroot()
    height = float(root.get("height"))
    bottoms = [float(r.get("y")) + float(r.get("height")) for r in root.iter(SVG + "rect")]
    assert max(bottoms) <= height and height - max(b for b in bottoms if b < height) < 100
    assert sum(1 for c in root.iter(SVG + "circle")) == 2  # the two Ready statuses
    metrics = ET.parse(tmp_path / "05-metrics.svg").getroot()
    assert sum(1 for _ in metrics.iter(SVG + "path")) >= 3  # power history sparklines


def test_committed_screenshots_match_the_code(tmp_path):
    """docs/screenshots are rendered on a fixed clock (tools/screenshots.py), so they must equal a fresh render:
    a view-model change that is not re-rendered into the docs fails here."""
    render(tmp_path)
    docs = os.path.join(ROOT, "docs", "screenshots")
    committed = sorted(n for n in os.listdir(docs) if n.endswith((".html", ".svg")))
    assert committed == sorted(os.listdir(tmp_path))
    assert len([n for n in committed if n.endswith(".svg")]) >= 5
    stale = [n for n in committed if open(os.path.join(docs, n)).read() != (tmp_path / n).read_text()]
    assert not stale, f"re-render with `python tools/screenshots.py`: {stale}"


def test_artifacthub_publishes_the_committed_svgs():
    """Every `screenshots:` entry of artifacthub-pkg.yml names one of docs/screenshots' SVGs (the validator CI runs
    checks the same), and every page of the plugin has one."""
    pkg = yaml.safe_load(open(os.path.join(ROOT, "artifacthub-pkg.yml")))
    files = [s["url"].rsplit("/", 1)[1] for s in pkg["screenshots"]]
    assert len(files) >= 5
    for f in files:
        assert f.endswith(".svg") and os.path.isfile(os.path.join(ROOT, "docs", "screenshots", f)), f
    assert {f[:-4] for f in files} >= set(VIEWS[:5])
