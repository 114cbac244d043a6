"""Native amdgpu-exporter daemon (ops/csrc/amdgpu_exporter.cpp).

CPU tests run the binary with no GPU (it must still answer, with no GPU series);
the GPU test checks real MI355X series and the single-device relabelling mode.
"""
import os
import re
import shutil
import signal
import subprocess
import time
import urllib.error
import urllib.request

import pytest

from headlamp_intel_gpu_plugin_amd.ops import build as native_build
from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition

HAS_HIPCC = bool(shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc"))
pytestmark = pytest.mark.skipif(not HAS_HIPCC, reason="hipcc not available")


@pytest.fixture(scope="module")
def exe():
    return native_build.build(["amdgpu-exporter"])["amdgpu-exporter"]


@pytest.fixture()
def server(exe):
    p = subprocess.Popen([exe, "--port", "0", "--bind", "127.0.0.1", "--hostname", "mi355x-test"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert "listening on" in line, line + p.stderr.read()
    port = int(line.split("127.0.0.1:")[1].split()[0])
    yield p, f"http://127.0.0.1:{port}"
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
        p.wait(10)


def test_once_prints_help_and_types(exe):
    r = subprocess.run([exe, "--once", "--hostname", "n0"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "# TYPE gpu_power_usage gauge" in r.stdout
    assert "# HELP gpu_xgmi_link_hops" in r.stdout


def test_rejects_bad_arguments(exe):
    assert subprocess.run([exe, "--bogus"], capture_output=True, timeout=30).returncode == 2
    assert subprocess.run([exe, "--port", "70000"], capture_output=True, timeout=30).returncode == 2


def test_http_endpoints(server):
    _, url = server
    with urllib.request.urlopen(url + "/healthz", timeout=10) as r:
        assert r.status == 200 and r.read() == b"ok\n"
    with urllib.request.urlopen(url + "/metrics", timeout=10) as r:
        assert r.headers["Content-Type"].startswith("text/plain")
        body = r.read().decode()
    assert "# TYPE gpu_total_vram gauge" in body
    for name, labels, _ in parse_exposition(body):
        assert labels["hostname"] == "mi355x-test"
    with pytest.raises(urllib.error.HTTPError) as e:
        urllib.request.urlopen(url + "/nope", timeout=10)
    assert e.value.code == 404


def test_sigterm_stops_cleanly(server):
    p, _ = server
    p.send_signal(signal.SIGTERM)
    assert p.wait(10) == 0


@pytest.mark.gpu
def test_exporter_reports_mi355x(exe):
    r = subprocess.run([exe, "--once", "--hostname", "n0"], capture_output=True, text=True, timeout=60)
    rows = parse_exposition(r.stdout)
    names = {n for n, _, _ in rows}
    assert {"gpu_total_vram", "gpu_power_usage"} <= names, names
    total = [v for n, l, v in rows if n == "gpu_total_vram" and l["gpu_id"] == "0"][0]
    assert 280e9 / 2**20 < total <= 288 * 1024
    labels = [l for n, l, _ in rows if n == "gpu_power_usage" and l["gpu_id"] == "0"][0]
    # HIP's device name is empty on this ROCm; the probe names the board from sysfs / device id.
    assert labels["card_model"] == "AMD Instinct MI355X", labels
    assert re.fullmatch(r"[0-9A-F]{16}", labels["serial_number"]), labels
    slow = [v for n, l, v in rows if n == "gpu_junction_temperature_slowdown" and l["gpu_id"] == "0"]
    assert slow and 90 <= slow[0] <= 120, slow  # amd-smi: slowdown_hotspot_temperature 100 C
    part = [l for n, l, _ in rows if n == "gpu_partition_info"]
    assert part and part[0]["compute_partition"] in {"SPX", "DPX", "QPX", "CPX"}, part
    assert part[0]["memory_partition"] in {"NPS1", "NPS2", "NPS4", "NPS8"}, part
    one = subprocess.run([exe, "--once", "--hostname", "n0", "--device", "0", "--gpu-label", "7"],
                         capture_output=True, text=True, timeout=60)
    ids = {l["gpu_id"] for n, l, _ in parse_exposition(one.stdout)}
    assert ids == {"7"}
    time.sleep(0)


def test_exporter_process_and_device_relabel(exe):
    from headlamp_intel_gpu_plugin_amd.parallel.agent import (ExporterProcess, NodeAgent, Scraper, device_to_node,
                                                              live_series)

    p = ExporterProcess(hostname="host-a").start()
    try:
        assert "# TYPE gpu_power_usage gauge" in p.scrape()
    finally:
        p.stop()
    assert p.proc.returncode == 0
    # A host-wide exporter's device 0 belongs to rank 0's synthetic node.
    agent = NodeAgent("host-a", lambda: {"power_w": 321.0, "vram_total_b": 2.0 ** 30}).start()
    try:
        live = live_series(["mi355x-003"])
        s = Scraper([(agent.url, device_to_node({"0": "mi355x-003"}))], live, now=lambda: 100.0)
        s.scrape_once()
        assert s.scrapes == 1
        assert live[("mi355x-003", 0)]["gpu_power_usage"].at(100.0)[1] == 321.0
        assert live[("mi355x-003", 0)]["gpu_total_vram"].at(100.0)[1] == 1024.0
        assert device_to_node({"0": "n"})({"gpu_id": "5"}) is None
    finally:
        agent.stop()
