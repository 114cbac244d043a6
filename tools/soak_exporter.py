#!/usr/bin/env python3
"""Soak the native amdgpu-exporter: scrape it hard while the GPU is busy.

    python tools/soak_exporter.py --seconds 180 --hz 20 [--out gpurun_out/soak.json]
                                  [--sysfs-only] [--slow 8] [--stalled 4]

Starts the daemon and a workload pod (Burner), scrapes /metrics at ``--hz``
for ``--seconds``, and reports scrape latency percentiles, errors, the
daemon's RSS over time (leak check) and how the live power / GFX readings
moved under load. Prints a progress line every 15 s.

Hostile peers, running for the whole soak next to the scraper: ``--slow N``
clients that trickle a request header one byte per second (each reconnects
when the daemon drops it at its per-request deadline), and ``--stalled N``
clients that send a request and never read the answer. The scrape latency
with them present is what a Prometheus server sees while the exporter is
under such an attack (the daemon's worker pool + deadlines, SECURITY.md).
"""

import argparse
import json
import os
import socket
import sys
import threading
import time
import urllib.parse
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import psutil  # noqa: E402

from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition  # noqa: E402
from headlamp_intel_gpu_plugin_amd.parallel.agent import ExporterProcess  # noqa: E402


def pct(xs, p):
    s = sorted(xs)
    return s[min(len(s) - 1, int(p * (len(s) - 1)))] if s else None


class Hostile:
    """Slow-loris and stalled-reader peers against host:port until stop()."""

    def __init__(self, url: str, slow: int, stalled: int):
        u = urllib.parse.urlparse(url)
        self.addr = (u.hostname, u.port)
        self.stop_ev = threading.Event()
        self.dropped = 0  # slow connections the daemon closed (deadline)
        self.threads = [threading.Thread(target=self._slow, daemon=True) for _ in range(slow)]
        self.threads += [threading.Thread(target=self._stalled, daemon=True) for _ in range(stalled)]

    def start(self):
        for t in self.threads:
            t.start()
        return self

    def _slow(self):
        req = b"GET /metrics HTTP/1.1\r\nHost: x\r\nX-Pad: " + b"a" * 4000
        while not self.stop_ev.is_set():
            try:
                with socket.create_connection(self.addr, timeout=5) as s:
                    for i in range(len(req)):
                        if self.stop_ev.wait(1.0):
                            return
                        s.sendall(req[i:i + 1])
            except OSError:
                self.dropped += 1

    def _stalled(self):
        while not self.stop_ev.is_set():
            try:
                with socket.create_connection(self.addr, timeout=5) as s:
                    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
                    s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
                    self.stop_ev.wait(10.0)  # never read
            except OSError:
                pass

    def stop(self):
        self.stop_ev.set()
        for t in self.threads:
            t.join(6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--hz", type=float, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-burn", action="store_true")
    ap.add_argument("--sysfs-only", action="store_true", help="run the daemon as the DaemonSet does (no HIP)")
    ap.add_argument("--slow", type=int, default=0, help="slow-loris peers")
    ap.add_argument("--stalled", type=int, default=0, help="peers that never read the response")
    a = ap.parse_args()
    exp = ExporterProcess(hostname="soak", sysfs_only=a.sysfs_only).start()
    hostile = Hostile(exp.url, a.slow, a.stalled).start() if (a.slow or a.stalled) else None
    proc = psutil.Process(exp.proc.pid)
    burner = None
    if not a.no_burn:
        from headlamp_intel_gpu_plugin_amd.ops.workload import Burner

        burner = Burner(device=0, size=8192, gemms=2, triad_mb=512).start()
    lat, errors, rss, power, gfx = [], 0, [], [], []
    t_end = time.monotonic() + a.seconds
    next_report = time.monotonic() + 15
    period = 1.0 / a.hz
    try:
        while time.monotonic() < t_end:
            t0 = time.perf_counter()
            try:
                with urllib.request.urlopen(exp.url, timeout=5) as r:
                    body = r.read().decode()
                lat.append((time.perf_counter() - t0) * 1e3)
                for n, lb, v in parse_exposition(body):
                    if lb.get("gpu_id") == "0" and n == "gpu_power_usage":
                        power.append(v)
                    if lb.get("gpu_id") == "0" and n == "gpu_gfx_activity":
                        gfx.append(v)
            except OSError:
                errors += 1
            if len(lat) % 20 == 0:
                rss.append(proc.memory_info().rss / 2**20)
            if time.monotonic() > next_report:
                print(f"{len(lat)} scrapes, p50 {pct(lat, .5):.2f} ms, rss {rss[-1] if rss else 0:.1f} MiB,"
                      f" power {power[-1] if power else 0:.0f} W", flush=True)
                next_report += 15
            time.sleep(max(0.0, period - (time.perf_counter() - t0)))
    finally:
        if hostile:
            hostile.stop()
        if burner:
            burner.stop()
        exp.stop()
    third = max(1, len(rss) // 3)
    doc = {
        "seconds": a.seconds, "hz": a.hz, "scrapes": len(lat), "errors": errors,
        "latency_ms": {"p50": pct(lat, .5), "p99": pct(lat, .99), "max": max(lat) if lat else None},
        "rss_mib": {"first_third_mean": sum(rss[:third]) / third, "last_third_mean": sum(rss[-third:]) / third,
                    "max": max(rss) if rss else None},
        "power_w": {"min": min(power) if power else None, "max": max(power) if power else None},
        "gfx_pct": {"min": min(gfx) if gfx else None, "max": max(gfx) if gfx else None},
        "burner_iterations": burner.iterations if burner else 0,
        "sysfs_only": a.sysfs_only,
        "hostile": {"slow": a.slow, "stalled": a.stalled, "slow_dropped_by_daemon": hostile.dropped if hostile else 0},
    }
    print(json.dumps(doc))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
