"""tools/screenshots.py renders every view of a fake cluster through the shipped view-models."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_screenshots_render_every_view(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "screenshots.py"), "--nodes", "2", "--out",
                        str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    names = sorted(os.listdir(tmp_path))
    assert names == ["01-overview.html", "02-device-plugins.html", "03-gpu-nodes.html", "04-gpu-pods.html",
                     "05-metrics.html", "06-node-detail.html", "07-pod-detail.html"]
    html = {n: (tmp_path / n).read_text() for n in names}
    assert "<h1>AMD GPU — Overview</h1>" in html["01-overview.html"]
    assert "GPU Node Summary" in html["03-gpu-nodes.html"]
    assert "mi355x-001" in html["03-gpu-nodes.html"]
    assert "<h2>AMD GPU</h2>" in html["06-node-detail.html"]
    assert "<h2>AMD GPU Resources</h2>" in html["07-pod-detail.html"]
    assert "GPU Power Summary" in html["05-metrics.html"]


def test_committed_screenshots_match_the_code(tmp_path):
    """docs/screenshots are rendered on a fixed clock (tools/screenshots.py), so they must equal a fresh render:
    a view-model change that is not re-rendered into the docs fails here."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "screenshots.py"), "--out", str(tmp_path)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    docs = os.path.join(ROOT, "docs", "screenshots")
    committed = sorted(n for n in os.listdir(docs) if n.endswith(".html"))
    assert committed == sorted(os.listdir(tmp_path))
    stale = [n for n in committed if open(os.path.join(docs, n)).read() != (tmp_path / n).read_text()]
    assert not stale, f"re-render with `python tools/screenshots.py`: {stale}"
