"""The fake control plane as a process of its own.

In a real deployment the kube-apiserver and Prometheus run on other hosts
than the browser and the GPU jobs. ``bench.py`` used to run the fake one as a
thread of rank 0 — the interpreter that also runs the workload pod's launch
thread — so every request it answered could wait for that process's GIL.
This module runs the fake control plane (and its telemetry scraper) in a
child process instead; it never imports torch or touches a GPU.

    python -m headlamp_intel_gpu_plugin_amd.sim.serve --nodes 4 --source both --latency-ms 20 \\
        [--preset 4x8] [--exporter http://127.0.0.1:PORT/metrics --device-map '{"0": "mi355x-000"}']

Prints one JSON line ``{"url", "gpu_nodes", "gpus_per_node"}`` once it
listens, then answers line commands on stdin: ``stats`` →
``{"server_requests": {...}, "scrapes": n}``; ``quit`` (or EOF) → exit.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from typing import Dict, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--nodes", type=int, default=1)
    p.add_argument("--source", default="both", choices=["amd-exporter", "node-exporter", "both"])
    p.add_argument("--latency-ms", type=float, default=20.0)
    p.add_argument("--preset", default=None)
    p.add_argument("--exporter", default=None, help="amdgpu-exporter /metrics URL scraped into the live series")
    p.add_argument("--device-map", default="{}", help='JSON {"<hip device>": "<node>"}: device d → GPU 0 of that node')
    p.add_argument("--interval", type=float, default=15.0,
                   help="scrape interval (s), on its grid: deploy/exporter's ServiceMonitor scrapes every 15 s")
    p.add_argument("--rules", action="store_true",
                   help="answer instant queries from background re-evaluations (apiserver.py: recording rules)")
    args = p.parse_args(argv)

    from ..parallel.agent import Scraper, device_to_node, live_series
    from .apiserver import ServerThread, make_fake

    node_of_device: Dict[str, str] = json.loads(args.device_map)
    live = live_series(list(node_of_device.values())) if args.exporter and node_of_device else None
    fc = make_fake(args.nodes, source=args.source, latency_ms=args.latency_ms, live=live, preset=args.preset,
                   rules=args.rules)
    scraper = (Scraper([(args.exporter, device_to_node(node_of_device))], live, interval=args.interval,
                       align=True).start()
               if live else None)
    server = ServerThread(fc).start()
    try:
        print(json.dumps({"url": server.url, "gpu_nodes": len(fc.cluster.gpu_nodes),
                          "gpus_per_node": fc.cluster.spec.gpus_per_node}), flush=True)
        for line in sys.stdin:
            cmd = line.strip()
            if cmd == "stats":
                with fc.lock:
                    work = sorted(w for _, w in fc.requests)
                    slowest = sorted(fc.requests, key=lambda r: -r[1])[:5]
                print(json.dumps({"server_requests": fc.stats(), "scrapes": scraper.scrapes if scraper else 0,
                                  "rule_evaluations": fc.rule_evals,
                                  # server-side work per request (ms), on top of the injected latency
                                  "server_work_ms": {"p50": round(work[len(work) // 2] * 1e3, 3) if work else None,
                                                     "max": round(work[-1] * 1e3, 3) if work else None,
                                                     "slowest": [[p[:120], round(w * 1e3, 3)] for p, w in slowest]}}),
                      flush=True)
            elif cmd == "quit":
                break
    finally:
        server.stop()
        if scraper:
            scraper.stop()
    return 0


class ControlPlaneProcess:
    """Parent-side handle of ``python -m headlamp_intel_gpu_plugin_amd.sim.serve``."""

    def __init__(self, nodes: int, *, source: str = "both", latency_ms: float = 20.0, preset: Optional[str] = None,
                 exporter_url: Optional[str] = None, node_of_device: Optional[Dict[str, str]] = None,
                 interval: float = 15.0, rules: bool = True):
        self.cmd = [sys.executable, "-m", "headlamp_intel_gpu_plugin_amd.sim.serve", "--nodes", str(nodes),
                    "--source", source, "--latency-ms", str(latency_ms), "--interval", str(interval)]
        if rules:
            self.cmd.append("--rules")
        if preset:
            self.cmd += ["--preset", preset]
        if exporter_url and node_of_device:
            self.cmd += ["--exporter", exporter_url, "--device-map", json.dumps(node_of_device)]
        self.proc: Optional[subprocess.Popen] = None
        self.info: Dict = {}

    def start(self) -> "ControlPlaneProcess":
        env = dict(os.environ)
        env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        self.proc = subprocess.Popen(self.cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=ROOT,
                                     env=env)
        line = self.proc.stdout.readline()
        if not line:
            self.proc.wait(10)
            raise RuntimeError(f"fake control plane exited with status {self.proc.returncode}")
        self.info = json.loads(line)
        return self

    @property
    def url(self) -> str:
        return self.info["url"]

    def stats(self) -> Dict:
        self.proc.stdin.write("stats\n")
        self.proc.stdin.flush()
        return json.loads(self.proc.stdout.readline())

    def stop(self) -> None:
        if self.proc is None or self.proc.poll() is not None:
            return
        try:
            self.proc.stdin.write("quit\n")
            self.proc.stdin.flush()
            self.proc.wait(15)
        except (OSError, subprocess.TimeoutExpired):
            self.proc.kill()
            self.proc.wait(5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


if __name__ == "__main__":
    sys.exit(main())
