"""End to end: what a GPU reports is what the dashboard shows.

One chain, with nothing stubbed between its ends: a sampler behind a per-node ``/metrics`` endpoint (``NodeAgent``,
the exporter's text format) → the scraper appending to the fake Prometheus's live series (``Scraper``, as
Prometheus scrapes the exporter) → the plugin's shipped data layer over HTTP (``bench/driver.js`` ``snapshot``:
``src/api/clusterStore.js`` + ``src/api/metrics.js``) → the Metrics page's view-model rendered to HTML
(``src/view/pages/metricsPage.js`` → ``src/view/html.js``). The GPU 0 row of the page is read back from that HTML.

* CPU: a fixed sample, so every figure on the row is checked exactly (power, cap, HBM used / total, GFX and HBM
  activity, junction temperature).
* GPU (MI355X box): ``probe.sample(0)`` of the real card. Static figures (power cap, HBM capacity) must be the
  card's exactly; the live ones lie between direct reads taken before and after (with a margin for power, which
  moves within the second). ``tests/test_ground_truth.py`` pins the probe to sysfs / hwmon; this pins the dashboard
  to the probe.

Reference analog: none — the reference's tests mock the metrics layer (src/components/MetricsPage.test.tsx).
"""
import html
import re
import time

import pytest

from headlamp_intel_gpu_plugin_amd.parallel.agent import NodeAgent, Scraper, live_series
from headlamp_intel_gpu_plugin_amd.sim.apiserver import ServerThread, make_fake
from headlamp_intel_gpu_plugin_amd.utils.nodebridge import Driver

GIB = 1 << 30
NODE = "mi355x-000"  # the single node of BASELINE preset #2 (1x1)

UNITS = {"B": 1, "KiB": 1 << 10, "MiB": 1 << 20, "GiB": GIB, "TiB": 1 << 40}
ROW = re.compile(r"GPU 0 \| ([\d.]+) W / ([\d.]+) W \(\d+%\) \| ([\d.]+) (B|KiB|MiB|GiB|TiB) / ([\d.]+) (B|KiB|MiB|GiB|TiB)"
                 r" \(\d+%\) \| (\d+)% \| (\d+)% \| (\d+) °C")


def dashboard_row(sampler, tmp_path):
    """The Metrics page's GPU 0 row after the chain has scraped `sampler` a few times: the parsed figures."""
    live = live_series([NODE])
    fc = make_fake(1, source="amd-exporter", latency_ms=0, live=live, preset="1x1")
    agent = NodeAgent(NODE, sampler).start()
    scraper = Scraper({NODE: agent.url}, live, interval=0.2).start()
    try:
        t0 = time.time()
        while scraper.scrapes < 3 and time.time() - t0 < 20:
            time.sleep(0.05)
        assert scraper.scrapes >= 3 and scraper.errors == 0, (scraper.scrapes, scraper.errors)
        with ServerThread(fc) as server:
            drv = Driver(server.url)
            try:
                out = drv.call("snapshot", "amd", dir=str(tmp_path), timeout=120)
            finally:
                drv.close()
    finally:
        scraper.stop()
        agent.stop()
    page = [f for f in out["files"] if f.endswith("05-metrics.html")][0]
    with open(page) as f:
        text = html.unescape(re.sub(r"(\s*\|\s*)+", " | ", re.sub(r"<[^>]+>", " | ", f.read())))
    m = ROW.search(text)
    assert m, text[-1500:]
    g = m.groups()
    assert f"{NODE} — 1 × MI355X" in text
    # HBM as formatBytes (src/api/k8sCore.js) shows it: three significant digits in the largest unit.
    return {"power": float(g[0]), "cap": float(g[1]), "used_b": float(g[2]) * UNITS[g[3]],
            "total_b": float(g[4]) * UNITS[g[5]], "gfx": float(g[6]), "umc": float(g[7]), "temp": float(g[8])}


def test_dashboard_shows_exactly_what_the_exporter_reports(tmp_path):
    sample = {"power_w": 321.5, "power_cap_w": 1234.0, "gfx_busy_pct": 42.0, "mem_busy_pct": 17.0,
              "temp_junction_c": 61.0, "temp_junction_slowdown_c": 95.0, "vram_used_b": 12.5 * GIB,
              "vram_total_b": 287.98 * GIB}
    row = dashboard_row(lambda: sample, tmp_path)
    assert row == {"power": 321.5, "cap": 1234.0, "used_b": 12.5 * GIB, "total_b": 288.0 * GIB, "gfx": 42.0,
                   "umc": 17.0, "temp": 61.0}


@pytest.mark.gpu
def test_dashboard_shows_the_real_mi355x(tmp_path):
    from headlamp_intel_gpu_plugin_amd.ops import probe

    before = probe.sample(0)
    row = dashboard_row(lambda: probe.sample(0), tmp_path)
    after = probe.sample(0)
    # Static: the card's own figures, as the page formats them (cap to 0.1 W, capacity to three digits).
    assert row["cap"] == pytest.approx(before["power_cap_w"], abs=0.051)
    assert row["total_b"] == pytest.approx(before["vram_total_b"], rel=0.005)
    assert row["total_b"] > 250 * GIB, row  # 288 GB HBM3E per MI355X
    # Live: between direct reads taken around the chain (power: ±20 % + 20 W, it moves within the second).
    lo_p = min(before["power_w"], after["power_w"])
    hi_p = max(before["power_w"], after["power_w"])
    assert lo_p * 0.8 - 20 <= row["power"] <= hi_p * 1.2 + 20, (row, before, after)
    lo_t = min(before["temp_junction_c"], after["temp_junction_c"])
    hi_t = max(before["temp_junction_c"], after["temp_junction_c"])
    assert lo_t - 5 <= row["temp"] <= hi_t + 5, (row, before, after)
    lo_u = min(before["vram_used_b"], after["vram_used_b"])
    hi_u = max(before["vram_used_b"], after["vram_used_b"])
    assert lo_u * 0.995 - (64 << 20) <= row["used_b"] <= hi_u * 1.005 + (64 << 20), (row, before, after)
