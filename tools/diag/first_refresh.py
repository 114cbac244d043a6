"""Attribute the latency of the smoke's FIRST dashboard refresh.

The driver's round-2 smoke once read 996 ms for the first refresh where
every other run read 11-19 ms (profiles/r2b_smoke.log 804 ms, r2l 1407 ms).
This replays the smoke's setup in one process — HIP initialised and a few
GEMMs run through torch (as smoke() does), the probe-backed NodeAgent, the
1 s Scraper and the in-process fake apiserver — and records, for the first
refreshes:

* each request's client-side span (Node driver, epoch ms) relative to its step;
* the apiserver's own handler time per request;
* the apiserver event loop's scheduling lag (a 1 ms ticker on that loop);
* every Python GC pause in the process (gc.callbacks), with its generation.

    python tools/diag/first_refresh.py [--no-gpu] > gpurun_out/diag/first_refresh.json
"""
from __future__ import annotations

import asyncio
import gc
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> None:
    use_gpu = "--no-gpu" not in sys.argv
    gc_events = []
    gc_open = {}

    def on_gc(phase, info):
        now = time.time() * 1e3
        if phase == "start":
            gc_open[threading.get_ident()] = now
        else:
            t0 = gc_open.pop(threading.get_ident(), now)
            gc_events.append({"start": t0, "ms": round(now - t0, 3), "gen": info.get("generation"),
                              "collected": info.get("collected")})

    gc.callbacks.append(on_gc)
    setup_t0 = time.time()
    if use_gpu:
        import torch

        from headlamp_intel_gpu_plugin_amd.ops import probe, workload

        dev = torch.device("cuda", 0)
        a = torch.randn(256, 512, device=dev, dtype=torch.bfloat16)
        b = torch.randn(384, 512, device=dev, dtype=torch.bfloat16)
        workload.gemm_bf16_nt(a, b)
        torch.cuda.synchronize()
        sampler = lambda: probe.sample(0)  # noqa: E731
    else:
        sampler = lambda: {"power_w": 100.0}  # noqa: E731

    from headlamp_intel_gpu_plugin_amd.parallel.agent import NodeAgent, Scraper, live_series
    from headlamp_intel_gpu_plugin_amd.sim.apiserver import ServerThread, make_fake
    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import Driver

    node = "mi355x-000"
    agent = NodeAgent(node, sampler).start()
    live = live_series([node])
    fc = make_fake(1, source="both", latency_ms=5, live=live)
    scraper = Scraper({node: agent.url}, live, interval=1.0).start()
    lags = []
    with ServerThread(fc) as server:
        async def ticker():
            last = time.perf_counter()
            while True:
                await asyncio.sleep(0.001)
                now = time.perf_counter()
                lag = (now - last) * 1e3 - 1.0
                if lag > 5.0:
                    lags.append({"at": round(time.time() * 1e3, 3), "lag_ms": round(lag, 3)})
                last = now

        tick = asyncio.run_coroutine_threadsafe(ticker(), server._loop)
        setup_ms = (time.time() - setup_t0) * 1e3
        drv = Driver(server.url)
        try:
            t_open = time.time() * 1e3
            out = drv.call("steps", "amd", n=5, rawSpans=True)
        finally:
            drv.close()
        tick.cancel()
    scraper.stop()
    agent.stop()
    t_end = time.time() * 1e3
    starts = out.get("stepStarts") or []
    spans = []
    for sp in out.get("spans") or []:
        step = max([i for i, s in enumerate(starts) if s <= sp["start"]] or [0])
        spans.append({"step": step, "name": sp["name"], "from_step_ms": round(sp["start"] - starts[step], 3),
                      "ms": round(sp["end"] - sp["start"], 3), "ok": sp["ok"]})
    work = [{"path": p[:60], "work_ms": round(w * 1e3, 3)} for p, w in list(fc.requests)]
    result = {
        "gpu": use_gpu,
        "setup_ms": round(setup_ms, 1),
        "latencies_ms": [round(x, 2) for x in out["latencies"]],
        "render_ms": [round(x, 2) for x in out.get("renderMs", [])],
        "spans": spans,
        "server_work_max_ms": max((w["work_ms"] for w in work), default=None),
        "server_work_top": sorted(work, key=lambda w: -w["work_ms"])[:5],
        "loop_lags_over_5ms": [l for l in lags if l["at"] >= t_open],
        "gc_pauses_during_run": [g for g in gc_events if g["start"] >= t_open and g["start"] <= t_end],
        "gc_pauses_setup_max_ms": max((g["ms"] for g in gc_events if g["start"] < t_open), default=None),
        "gc_counts": gc.get_count(),
        "gc_objects": len(gc.get_objects()),
        "scrapes": scraper.scrapes,
    }
    print(json.dumps(result, indent=1))


if __name__ == "__main__":
    main()
