"""Attribute the latency of one telemetry sample on a GPU box.

Times every sysfs file the probe reads for device 0 (plain Python reads, so
each read releases the GIL), then ``probe.device_info(0)`` (hipGetDeviceProperties)
and ``probe.sample(0)``, and finally a GIL-starvation check: a thread spinning
short Python work while another thread calls ``probe.sample`` in a loop. The
longest gap the spinner sees is how long ``sample`` held the GIL.

    python tools/diag/sample_latency.py > gpurun_out/diag/sample_latency.json
"""
from __future__ import annotations

import glob
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from headlamp_intel_gpu_plugin_amd.ops import probe  # noqa: E402


def timed_read(path: str):
    t0 = time.perf_counter()
    try:
        with open(path, "rb") as f:
            f.read()
        ok = True
    except OSError:
        ok = False
    return (time.perf_counter() - t0) * 1e3, ok


def summary(xs):
    xs = sorted(xs)
    return {"n": len(xs), "min": round(xs[0], 3), "p50": round(statistics.median(xs), 3), "max": round(xs[-1], 3)}


def main() -> None:
    out = {"module": "current"}
    if len(sys.argv) > 1 and sys.argv[1] == "--old":
        # The round-2 binding (GIL held across the sample), built from git
        # history into tools/diag/_old_probe/ for an A/B on the same box.
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "_old_probe"))
        import _amdgpu_probe as old

        probe._mod = old
        out["module"] = old.__file__
    info = probe.device_info(0)
    bdf = info["bdf"]
    dev = f"/sys/bus/pci/devices/{bdf}"
    files = [f"{dev}/{n}" for n in ("gpu_busy_percent", "mem_busy_percent", "mem_info_vram_used", "mem_info_vram_total",
                                      "current_compute_partition", "current_memory_partition")]
    files += sorted(glob.glob(f"{dev}/ras/aca_*")) + sorted(glob.glob(f"{dev}/ras/*_err_count"))
    files += [f"{dev}/ras/gpu_vram_bad_pages"]
    for h in sorted(glob.glob(f"{dev}/hwmon/hwmon*")):
        files += [f"{h}/{n}" for n in ("power1_average", "power1_input", "power1_cap", "freq1_input", "freq2_input")]
        files += sorted(glob.glob(f"{h}/temp*_input")) + sorted(glob.glob(f"{h}/temp*_crit"))
    per_file = {}
    for rep in range(5):
        for p in files:
            ms, ok = timed_read(p)
            if ok:
                per_file.setdefault(p.replace(dev + "/", ""), []).append(ms)
    out["per_file_ms"] = {k: summary(v) for k, v in per_file.items()}
    out["slowest_files"] = sorted(((v["max"], k) for k, v in out["per_file_ms"].items()), reverse=True)[:8]

    di = []
    for _ in range(10):
        t0 = time.perf_counter()
        probe.device_info(0)
        di.append((time.perf_counter() - t0) * 1e3)
    out["device_info_ms"] = summary(di)

    sm = []
    for _ in range(20):
        t0 = time.perf_counter()
        probe.sample(0)
        sm.append((time.perf_counter() - t0) * 1e3)
    out["sample_ms"] = summary(sm)

    # GIL starvation: spinner records the longest interval between iterations.
    stop = threading.Event()
    gaps = []

    def spin():
        last = time.perf_counter()
        worst = 0.0
        while not stop.is_set():
            now = time.perf_counter()
            worst = max(worst, now - last)
            last = now
            sum(range(50))
        gaps.append(worst * 1e3)

    t = threading.Thread(target=spin)
    t.start()
    sampled = []
    for _ in range(20):
        t0 = time.perf_counter()
        probe.sample(0)
        sampled.append((time.perf_counter() - t0) * 1e3)
    stop.set()
    t.join()
    out["concurrent"] = {"sample_ms": summary(sampled), "spinner_longest_gap_ms": round(gaps[0], 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
