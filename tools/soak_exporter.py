#!/usr/bin/env python3
"""Soak the native amdgpu-exporter: scrape it hard while the GPU is busy.

    python tools/soak_exporter.py --seconds 180 --hz 20 [--out gpurun_out/soak.json]

Starts the daemon and a workload pod (Burner), scrapes /metrics at ``--hz``
for ``--seconds``, and reports scrape latency percentiles, errors, the
daemon's RSS over time (leak check) and how the live power / GFX readings
moved under load. Prints a progress line every 15 s.
"""
import argparse
import json
import os
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import psutil  # noqa: E402

from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition  # noqa: E402
from headlamp_intel_gpu_plugin_amd.parallel.agent import ExporterProcess  # noqa: E402


def pct(xs, p):
    s = sorted(xs)
    return s[min(len(s) - 1, int(p * (len(s) - 1)))] if s else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--hz", type=float, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-burn", action="store_true")
    a = ap.parse_args()
    exp = ExporterProcess(hostname="soak").start()
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
    }
    print(json.dumps(doc))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
