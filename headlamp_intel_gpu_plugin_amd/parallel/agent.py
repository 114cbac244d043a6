"""Per-node telemetry agents and the scraper that feeds the fake Prometheus.

One process per GPU (torchrun): rank ``r`` plays synthetic node ``r``. Its
:class:`NodeAgent` serves ``/metrics`` in AMD Device Metrics Exporter format,
sampled live from its own MI355X through the native probe
(``ops/csrc/amdgpu_probe.cpp``) — the DaemonSet-per-node exporter of a real
cluster. Rank 0's :class:`Scraper` pulls every agent on a fixed interval, as
Prometheus would, and pushes the samples into the TSDB series of
(node r, GPU 0); the node's other seven GPUs stay synthetic because each rank
owns exactly one physical device.
"""
from __future__ import annotations

import http.server
import threading
import time
import urllib.request
from typing import Callable, Dict, List, Optional, Tuple

from ..ops.probe import parse_exposition
from ..sim.promql import Series

#: exporter metric → (sample key, scale)
LIVE_FIELDS = {
    "gpu_power_usage": ("power_w", 1.0),
    "gpu_gfx_activity": ("gfx_busy_pct", 1.0),
    "gpu_umc_activity": ("mem_busy_pct", 1.0),
    "gpu_junction_temperature": ("temp_junction_c", 1.0),
    "gpu_used_vram": ("vram_used_b", 1.0 / (1024 * 1024)),
    "gpu_total_vram": ("vram_total_b", 1.0 / (1024 * 1024)),
}


def render_sample(node: str, gpu: int, sample: Dict[str, Optional[float]]) -> str:
    """One GPU's sample as exporter text (None fields omitted)."""
    lines = []
    for name, (key, scale) in LIVE_FIELDS.items():
        v = sample.get(key)
        if v is None:
            continue
        lines.append(f'{name}{{hostname="{node}",gpu_id="{gpu}"}} {v * scale:.6g}')
    return "\n".join(lines) + "\n"


class NodeAgent:
    """HTTP ``/metrics`` endpoint for one node, backed by ``sampler()``."""

    def __init__(self, node: str, sampler: Callable[[], Dict[str, Optional[float]]], host: str = "127.0.0.1",
                 port: int = 0):
        self.node = node
        self.sampler = sampler
        agent = self

        class Handler(http.server.BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802 (http.server API)
                if self.path.rstrip("/") != "/metrics":
                    self.send_error(404)
                    return
                try:
                    body = render_sample(agent.node, 0, agent.sampler()).encode()
                except Exception as e:  # report, don't kill the server thread
                    self.send_error(500, str(e))
                    return
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *args):
                pass

        self._srv = http.server.ThreadingHTTPServer((host, port), Handler)
        self._srv.daemon_threads = True
        self.url = f"http://{host}:{self._srv.server_address[1]}/metrics"
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True, name=f"agent-{node}")

    def start(self) -> "NodeAgent":
        self._thread.start()
        return self

    def stop(self) -> None:
        self._srv.shutdown()
        self._srv.server_close()


def live_series(nodes: List[str]) -> Dict[Tuple[str, int], Dict[str, Series]]:
    """Empty pushed series for GPU 0 of each node (``models.telemetry.populate(live=...)``)."""
    out = {}
    for node in nodes:
        out[(node, 0)] = {name: Series({"__name__": name, "hostname": node, "gpu_id": "0"}) for name in LIVE_FIELDS}
    return out


class Scraper:
    """Pulls every agent every ``interval`` s and appends to the live series."""

    def __init__(self, targets: Dict[str, str], live: Dict[Tuple[str, int], Dict[str, Series]], interval: float = 2.0,
                 now: Callable[[], float] = time.time):
        self.targets = targets
        self.live = live
        self.interval = interval
        self.now = now
        self.scrapes = 0
        self.errors = 0
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, daemon=True, name="scraper")

    def scrape_once(self) -> None:
        t = self.now()
        for node, url in self.targets.items():
            try:
                with urllib.request.urlopen(url, timeout=2) as r:
                    text = r.read().decode()
            except OSError:
                self.errors += 1
                continue
            for name, labels, value in parse_exposition(text):
                series = self.live.get((labels.get("hostname", node), int(labels.get("gpu_id", "0"))), {}).get(name)
                if series is not None:
                    series.push(t, value)
            self.scrapes += 1

    def _loop(self) -> None:
        while not self._stop.is_set():
            self.scrape_once()
            self._stop.wait(self.interval)

    def start(self) -> "Scraper":
        self.scrape_once()
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(5)
