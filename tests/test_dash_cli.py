"""bin/amd-gpu-dash.js: the plugin's data layer + view-models in a terminal, against the fake cluster."""
import json
import os
import subprocess

import pytest

from headlamp_intel_gpu_plugin_amd.sim.apiserver import ServerThread, make_fake
from headlamp_intel_gpu_plugin_amd.utils.nodebridge import node_binary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "amd-gpu-dash.js")


def run(*args, timeout=60):
    return subprocess.run([node_binary(), CLI] + list(args), capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.fixture(scope="module")
def url():
    fc = make_fake(2, source="amd-exporter", latency_ms=1)
    with ServerThread(fc) as srv:
        yield srv.url


def test_all_pages_render(url):
    r = run("--url", url, "--page", "all")
    assert r.returncode == 0, r.stderr
    for title in ("AMD GPU — Overview", "AMD GPU — Device Plugins", "AMD GPU — Nodes", "AMD GPU — Pods",
                  "AMD GPU — Metrics"):
        assert "# " + title in r.stdout
    assert "mi355x-001" in r.stdout and "xGMI topology (measured; link throughput measured)" in r.stdout and "Assigned GPUs" in r.stdout


def test_json_is_the_view_model(url):
    r = run("--url", url, "--page", "nodes", "--json")
    assert r.returncode == 0, r.stderr
    vm = json.loads(r.stdout)
    assert vm["title"] == "AMD GPU — Nodes"
    assert [s["title"] for s in vm["items"] if s["t"] == "section"][:3] == ["GPU Node Summary", "mi355x-000", "mi355x-001"]
    pager = [s for s in vm["items"] if s["t"] == "pager"][0]
    assert pager["noun"] == "GPU nodes" and pager["page"] == 0 and pager["from"] == 0


def test_unreachable_prometheus_and_bad_arguments(url):
    r = run("--url", url, "--page", "metrics", "--prometheus", "monitoring/none:9090")
    assert r.returncode == 0 and "GPU Power Summary" in r.stdout  # falls back to the built-in candidates
    assert run("--page", "nope").returncode == 2
    assert run("--prometheus", "not-a-service").returncode == 2
    dead = run("--url", "http://127.0.0.1:9", "--page", "overview", "--timeout", "500")
    assert dead.returncode == 0 and "Error" in dead.stdout  # the page's own error state, not a crash


def test_single_pages_ask_only_for_their_telemetry(url):
    pods = run("--url", url, "--page", "pods")
    assert pods.returncode == 0 and "Assigned GPUs" in pods.stdout and "mi355x-000: GPU 0" in pods.stdout
    nodes = run("--url", url, "--page", "nodes")
    assert nodes.returncode == 0 and "xGMI topology (measured; link throughput measured)" in nodes.stdout


def test_overview_sends_no_prometheus_request():
    fc = make_fake(1, source="amd-exporter", latency_ms=1)
    with ServerThread(fc) as srv:
        r = run("--url", srv.url, "--page", "overview")
        assert r.returncode == 0 and "Error" not in r.stdout
        assert fc.stats().get("prometheus", 0) == 0 and fc.stats()["apiserver"] >= 3


def test_device_plugins_lists_operator_pods_only():
    """As its plugin route: the DeviceConfigs and the operator pods, never the node list or every pod."""
    fc = make_fake(2, source="amd-exporter", latency_ms=1)
    with ServerThread(fc) as srv:
        r = run("--url", srv.url, "--page", "device-plugins")
        assert r.returncode == 0, r.stderr
        assert "DeviceConfig: gpu-operator" in r.stdout and "gpu-operator-device-plugin-" in r.stdout
        with fc.lock:
            paths = [p for p, _ in fc.requests]
        assert "/api/v1/pods" not in paths and "/api/v1/nodes" not in paths, paths
        assert "/api/v1/namespaces/kube-amd-gpu/pods" in paths


def test_detail_sections_with_power_history(url):
    node = run("--url", url, "--page", "node:mi355x-001")
    assert node.returncode == 0, node.stderr
    assert node.stdout.startswith("AMD GPU\n") and "Peak GPU Power (30 min)" in node.stdout and "xGMI topology" in node.stdout
    history = [l for l in node.stdout.splitlines() if "power samples" in l]
    assert history and any(c in history[0] for c in "▁▂▃▄▅▆▇█")  # the sparkline of the window
    pod = run("--url", url, "--page", "pod:ml/train-000-2")
    assert pod.returncode == 0, pod.stderr
    assert "AMD GPU Resources" in pod.stdout and "GPU Energy (30 min)" in pod.stdout and "Assigned GPUs" in pod.stdout
    missing = run("--url", url, "--page", "node:cpu-0")
    assert missing.returncode == 0 and "No AMD GPU section for node cpu-0" in missing.stdout
    js = run("--url", url, "--page", "pod:ml/train-000-2", "--json")
    assert json.loads(js.stdout)["title"] == "AMD GPU Resources"
    assert run("--page", "pod:no-slash").returncode == 2


def test_pager_flags_select_the_page_and_filter(url):
    r = run("--url", url, "--page", "nodes", "--json", "--filter", "001")
    assert r.returncode == 0, r.stderr
    vm = json.loads(r.stdout)
    assert [s["title"] for s in vm["items"] if s["t"] == "section"][1:] == ["mi355x-001"]
    pager = [s for s in vm["items"] if s["t"] == "pager"][0]
    assert pager["matched"] == 1 and pager["filter"] == "001"
    two = json.loads(run("--url", url, "--page", "nodes", "--json", "--per-page", "1", "--page-number", "2").stdout)
    assert [s["title"] for s in two["items"] if s["t"] == "section"][1:] == ["mi355x-001"]
    assert run("--url", url, "--page-number", "0").returncode == 2


def test_sort_flag_orders_the_nodes(url):
    r = run("--url", url, "--page", "nodes", "--json", "--sort", "attention")
    assert r.returncode == 0, r.stderr
    pager = [i for i in json.loads(r.stdout)["items"] if i["t"] == "pager"][0]
    assert pager["sort"] == "attention" and [o["value"] for o in pager["sorts"]][0] == "name"
    text = run("--url", url, "--page", "nodes", "--sort", "in-use")
    assert text.returncode == 0 and "sorted: Most GPUs in use" in text.stdout
    bad = run("--url", url, "--sort", "hottest")
    assert bad.returncode == 2 and "bad --sort" in bad.stderr
    pods = run("--url", url, "--page", "pods", "--sort", "gpus")
    assert pods.returncode == 0 and "sorted: Most GPUs held" in pods.stdout


def test_sort_power_lets_prometheus_rank_the_page(url):
    for page, noun in (("nodes", "GPU nodes reporting"), ("metrics", "GPU nodes reporting"), ("pods", "GPU pods drawing power")):
        r = run("--url", url, "--page", page, "--json", "--sort", "power")
        assert r.returncode == 0, r.stderr
        pager = [i for i in json.loads(r.stdout)["items"] if i["t"] == "pager"][0]
        assert pager["sort"] == "power" and pager["noun"] == noun, (page, pager)
        assert pager["total"] > 0, (page, pager)
    text = run("--url", url, "--page", "pods", "--sort", "power")
    assert text.returncode == 0 and "sorted: Highest GPU power" in text.stdout, text.stdout[-800:]


def test_svg_draws_a_page_or_a_detail_section(url):
    """--svg: the page's view-model as the SVG picture docs/screenshots holds (src/view/svg.js), once."""
    import xml.etree.ElementTree as ET

    r = run("--url", url, "--page", "nodes", "--svg")
    assert r.returncode == 0, r.stderr
    root = ET.fromstring(r.stdout)
    texts = [t.text for t in root.iter("{http://www.w3.org/2000/svg}text")]
    assert texts[0] == "AMD GPU — Nodes" and "GPU Node Summary" in texts and "mi355x-001" in texts
    d = run("--url", url, "--page", "node:mi355x-000", "--svg")
    assert d.returncode == 0, d.stderr
    assert "AMD GPU" in [t.text for t in ET.fromstring(d.stdout).iter("{http://www.w3.org/2000/svg}text")]
    for bad in (["--svg", "--json"], ["--svg", "--page", "all"], ["--svg", "--watch", "5"]):
        assert run("--url", url, *bad).returncode == 2
