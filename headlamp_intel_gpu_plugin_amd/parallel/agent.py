"""Per-node telemetry agents and the scraper that feeds the fake Prometheus.

One process per GPU (torchrun): rank ``r`` plays synthetic node ``r`` and owns
HIP device ``r``. Live telemetry comes from the native ``amdgpu-exporter``
daemon (:class:`ExporterProcess`, ops/csrc/amdgpu_exporter.cpp) — the
DaemonSet-per-node exporter of a real cluster — started once on the host and
exporting every visible MI355X; :class:`NodeAgent` is the in-process Python
equivalent (one GPU, probe-backed) used by smoke tests. Rank 0's
:class:`Scraper` pulls the targets on a fixed interval, as Prometheus would,
and pushes each sample into the TSDB series of (node r, GPU 0) for device r;
the node's other seven GPUs stay synthetic because each rank owns exactly one
physical device.
"""
from __future__ import annotations

import http.server
import math
import os
import signal
import subprocess
import threading
import time
import urllib.request
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

from ..ops.probe import parse_exposition
from ..sim.promql import Series

#: exporter metric → (sample key, scale)
LIVE_FIELDS = {
    "gpu_power_usage": ("power_w", 1.0),
    "gpu_power_cap": ("power_cap_w", 1.0),
    "gpu_gfx_activity": ("gfx_busy_pct", 1.0),
    "gpu_umc_activity": ("mem_busy_pct", 1.0),
    "gpu_junction_temperature": ("temp_junction_c", 1.0),
    "gpu_junction_temperature_slowdown": ("temp_junction_slowdown_c", 1.0),
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


class ExporterProcess:
    """The native ``amdgpu-exporter`` daemon as a child process on an ephemeral port."""

    def __init__(self, hostname: str, device: Optional[int] = None, gpu_label: Optional[str] = None,
                 topology: bool = True, sysfs_only: bool = False):
        from ..ops import build as native_build

        # Builds (under the build lock) only when missing or stale, e.g. on a
        # box that received the sources without the in-tree binaries.
        exe = native_build.build(["amdgpu-exporter"]).get("amdgpu-exporter", "")
        if not exe or not os.path.exists(exe):
            raise RuntimeError("amdgpu-exporter could not be built (hipcc / ROCm missing?)")
        self.cmd = [exe, "--port", "0", "--bind", "127.0.0.1", "--hostname", hostname]
        if device is not None:
            self.cmd += ["--device", str(device)]
            if gpu_label is not None:
                self.cmd += ["--gpu-label", gpu_label]
        if not topology:
            self.cmd.append("--no-topology")
        if sysfs_only:
            self.cmd.append("--sysfs-only")
        self.proc: Optional[subprocess.Popen] = None
        self.url = ""

    def start(self, timeout: float = 60.0) -> "ExporterProcess":
        self.proc = subprocess.Popen(self.cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        deadline = time.monotonic() + timeout
        line = ""
        while time.monotonic() < deadline and "listening on" not in line:
            line = self.proc.stdout.readline()
            if not line and self.proc.poll() is not None:
                raise RuntimeError("amdgpu-exporter exited: " + self.proc.stderr.read()[-2000:])
        if "listening on" not in line:
            self.stop()
            raise RuntimeError("amdgpu-exporter did not start")
        port = int(line.split("127.0.0.1:")[1].split()[0])
        self.url = f"http://127.0.0.1:{port}/metrics"
        return self

    def scrape(self, timeout: float = 10.0) -> str:
        with urllib.request.urlopen(self.url, timeout=timeout) as r:
            return r.read().decode()

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)


def live_series(nodes: List[str]) -> Dict[Tuple[str, int], Dict[str, Series]]:
    """Empty pushed series for GPU 0 of each node (``models.telemetry.populate(live=...)``)."""
    out = {}
    for node in nodes:
        out[(node, 0)] = {name: Series({"__name__": name, "hostname": node, "gpu_id": "0"}) for name in LIVE_FIELDS}
    return out


#: maps a scraped series' labels to the (node, gpu) it belongs to, or None to drop it
Relabel = Callable[[Dict[str, str]], Optional[Tuple[str, int]]]


def _by_hostname(default_node: str) -> Relabel:
    return lambda labels: (labels.get("hostname", default_node), int(labels.get("gpu_id", "0")))


def device_to_node(node_of_device: Dict[str, str]) -> Relabel:
    """Relabel a host-wide exporter: series of HIP device ``d`` → (node of rank d, GPU 0)."""
    return lambda labels: (node_of_device[labels["gpu_id"]], 0) if labels.get("gpu_id") in node_of_device else None


#: A grid-scheduled scrape this late after its grid point is still stamped with it.
ALIGN_SLACK_S = 0.5


class Scraper:
    """Pulls every target every ``interval`` s and appends to the live series.

    ``targets`` is ``{node: url}`` (per-node agents, labels used as-is) or a
    list of ``(url, relabel)`` pairs. With ``align`` the scrapes are scheduled
    on the ``interval`` grid (a target's scrapes are one interval apart in
    Prometheus too, and the fake's synthetic series are sampled on the same
    grid), so the fake's query caches turn over once per interval, not once
    per scrape of a faster loop. A scrape taken on the grid (within
    ALIGN_SLACK_S after a grid point, the loop's wake-up delay) is stamped
    with the grid time; one taken off it — the first, when the scraper starts
    — keeps its own time, so no sample is dated more than ALIGN_SLACK_S
    before it was read.
    """

    def __init__(self, targets: Union[Dict[str, str], Sequence[Tuple[str, Relabel]]],
                 live: Dict[Tuple[str, int], Dict[str, Series]], interval: float = 2.0,
                 now: Callable[[], float] = time.time, align: bool = False):
        if isinstance(targets, dict):
            targets = [(url, _by_hostname(node)) for node, url in targets.items()]
        self.targets = list(targets)
        self.live = live
        self.interval = interval
        self.now = now
        self.align = align
        self.scrapes = 0
        self.errors = 0
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, daemon=True, name="scraper")

    def scrape_once(self) -> None:
        t = self.now()
        if self.align:
            grid = math.floor(t / self.interval) * self.interval
            if t - grid <= ALIGN_SLACK_S:
                t = grid
        for url, relabel in self.targets:
            try:
                with urllib.request.urlopen(url, timeout=2) as r:
                    text = r.read().decode()
            except OSError:
                self.errors += 1
                continue
            for name, labels, value in parse_exposition(text):
                key = relabel(labels)
                series = self.live.get(key, {}).get(name) if key is not None else None
                if series is not None:
                    series.push(t, value)
            self.scrapes += 1

    def _loop(self) -> None:
        while not self._stop.is_set():
            if self.align:
                # Wake on the next grid point (a little after it, so the grid time has passed).
                wait = self.interval - (self.now() % self.interval) + 0.01
                if self._stop.wait(wait):
                    break
                self.scrape_once()
                continue
            self.scrape_once()
            self._stop.wait(self.interval)

    def start(self) -> "Scraper":
        self.scrape_once()
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(5)
