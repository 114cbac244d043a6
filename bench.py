#!/usr/bin/env python3
"""Headline benchmark: p50 dashboard refresh + rows rendered on a synthetic MI355X cluster.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

BASELINE.json metric: "p50 dashboard refresh (ms) + GPU nodes/pods rendered at
1/2/4/8-node cluster". One rank per GPU; rank r plays node r of an N-node
cluster of 8×MI355X nodes (weak scaling: per-node work is fixed as N grows).

* rank 0 starts the fake kube-apiserver + Prometheus (service proxy) as a
  child process (sim/serve.py: its own interpreter, like a control plane on
  other hosts) with an injected per-request round-trip latency
  (``--rtt-ms``, default 20 ms), identical for both schedules measured;
* every rank with a GPU runs (unless ``--no-burn``) a workload "pod" running
  the MFMA GEMM + HBM triad kernels on its own MI355X; rank 0 starts the
  native ``amdgpu-exporter`` daemon (C++/HIP, one for the host) and scrapes
  it every 15 s on the scrape grid (the interval of deploy/exporter's
  ServiceMonitor) into the TSDB, HIP device r → GPU 0 of node r, so GPU 0 of
  every node reports real power / HBM / activity;
* rank 0 drives the SHIPPED plugin data layer (src/, Node.js) over real HTTP:
  the reference plugin's request schedule is replayed first as the measured
  baseline (untimed), then the flagship schedule runs W warm-up refreshes and
  EXACTLY K timed refreshes bracketed by barrier + torch.cuda.synchronize()
  on every rank; ms_per_step is the MAX over ranks.

A timed STEP = one pass through the five routes (Overview, Device Plugins,
GPU Nodes, GPU Pods, Metrics) clicking each page's own Refresh button: the
time from the click to that page's data committed and the page rebuilt and
rendered is one sample. ``value`` = the mean over the five pages of each
page's p50 click latency (``per_page_refresh_p50_ms`` has them one by one,
next to the reference's). The reference's buttons run different chains per
page — the provider's 4 serial requests on the first four, the Metrics page's
probe + 4 queries on the last — and each is replayed as wired.

The "all pages" composite (every page's data + all views rebuilt in one go,
which no single reference button does) is reported as a secondary figure.
Render in the timed click = view-model → HTML string (the IR renderer's
output). Untimed, every page is also mounted and re-rendered through the
shipped React renderer, on the harness React and on real React 18.3.1
production builds (``render_per_page`` / ``render_per_page_react_dom``).
Data is synthetic (no cluster, no network); say so in the JSON.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "p50 dashboard refresh (ms) + GPU nodes/pods rendered at 1/2/4/8-node cluster"


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1, help="ranks / synthetic nodes (one GPU per rank)")
    p.add_argument("--steps", type=int, default=30, help="timed refreshes")
    p.add_argument("--warmup", type=int, default=5, help="untimed warm-up refreshes")
    p.add_argument("--rtt-ms", type=float, default=20.0, help="injected per-request round trip")
    p.add_argument("--nodes", type=int, default=None, help="override synthetic node count (default: --gpus; 0 = CPU-only)")
    p.add_argument("--preset", default=None, choices=["cpu-only", "1x1", "1x8", "4x8", "8x8"],
                   help="BASELINE.json config preset instead of N x 8 nodes")
    p.add_argument("--ref-steps", type=int, default=None, help="reference-schedule refreshes (default: --steps)")
    p.add_argument("--no-burn", action="store_true", help="do not run the GPU workload pods")
    p.add_argument("--no-live", action="store_true", help="synthetic telemetry only (no native probe)")
    p.add_argument("--source", default="both", choices=["both", "amd-exporter", "node-exporter"],
                   help="GPU series the fake Prometheus holds: the Device Metrics Exporter's, node-exporter's amdgpu "
                        "hwmon / DRM series (the plugin's fallback source), or both")
    p.add_argument("--control-plane", default="process", choices=["process", "thread"],
                   help="run the fake apiserver/Prometheus in a child process (default) or a thread of rank 0")
    p.add_argument("--out", default=None, help="also write the full result JSON here")
    p.add_argument("--order", default="reference-first", choices=["reference-first", "amd-first"],
                   help="which schedule's phases run first (the figures must not depend on it)")
    return p.parse_args(argv)


def _p50(xs):
    """p50 of a list of ms (rounded), None for none."""
    from headlamp_intel_gpu_plugin_amd.utils.stats import summarize

    return round(summarize(xs)["p50"], 3) if xs else None


def main(argv=None) -> int:
    args = parse_args(argv)

    from headlamp_intel_gpu_plugin_amd.models.cluster import gpu_node_name
    from headlamp_intel_gpu_plugin_amd.parallel import dist as D
    from headlamp_intel_gpu_plugin_amd.utils.stats import summarize

    info = D.init()
    n_nodes = args.nodes if args.nodes is not None else max(args.gpus, info.world)
    node_name = gpu_node_name(info.rank)
    gpu = info.device is not None

    # --- workload pod per rank; one native exporter for the host ----------
    burner = exporter = None
    # The live probe exports Device Metrics Exporter series: not on a node-exporter-only cluster.
    live_on = gpu and not args.no_live and args.source != "node-exporter"
    if gpu and not args.no_burn:
        from headlamp_intel_gpu_plugin_amd.ops.workload import Burner

        # ~1.7 ms of GPU work per iteration (2 x 8192^3 bf16 GEMM on the 8-phase
        # kernel + a 1.5 GB triad): few launches, little GIL time on rank 0.
        burner = Burner(device=info.device.index, size=8192, gemms=2, triad_mb=512).start()
    ranks = D.all_gather_object(info, (node_name, info.device.index if gpu else None))

    def quiet_sync():
        """torch.cuda.synchronize() with the workload pod paused between
        iterations, so the sync waits for the bench's own work only."""
        if burner:
            burner.pause()
        D.sync_device(info)
        if burner:
            burner.resume()

    if live_on and info.is_main:
        from headlamp_intel_gpu_plugin_amd.parallel.agent import ExporterProcess

        # The C++ amdgpu-exporter daemon exports every MI355X on the host
        # (one process, whatever the rank count); HIP device d belongs to
        # the rank that owns it, i.e. to that rank's synthetic node.
        exporter = ExporterProcess(hostname=socket.gethostname()).start()
        if "gpu_total_vram{" not in exporter.scrape():
            exporter.stop()
            raise RuntimeError("GPU present but amdgpu-exporter exports no device")

    result = None
    elapsed = 0.0
    if info.is_main:
        from headlamp_intel_gpu_plugin_amd.utils.nodebridge import Driver

        node_of_device = {str(d): n for n, d in ranks if d is not None} if exporter else {}
        if args.control_plane == "process":
            # Its own interpreter, like a real apiserver / Prometheus on other
            # hosts: no request waits for this process's GIL (workload pod).
            from headlamp_intel_gpu_plugin_amd.sim.serve import ControlPlaneProcess

            server = ControlPlaneProcess(n_nodes, source=args.source, latency_ms=args.rtt_ms, preset=args.preset,
                                         exporter_url=exporter.url if exporter else None,
                                         node_of_device=node_of_device).start()
            n_nodes, gpus_per_node = server.info["gpu_nodes"], server.info["gpus_per_node"]
            scraper = None
        else:
            from headlamp_intel_gpu_plugin_amd.parallel.agent import Scraper, device_to_node, live_series
            from headlamp_intel_gpu_plugin_amd.sim.apiserver import ServerThread, make_fake

            live = live_series(list(node_of_device.values())) if node_of_device else None
            fc = make_fake(n_nodes, source=args.source, latency_ms=args.rtt_ms, live=live, preset=args.preset)
            n_nodes, gpus_per_node = len(fc.cluster.gpu_nodes), fc.cluster.spec.gpus_per_node
            scraper = (Scraper([(exporter.url, device_to_node(node_of_device))], live, interval=15.0, align=True).start()
                       if node_of_device else None)
            server = ServerThread(fc).start()
        drv = Driver(server.url)
        # The reference schedule runs in a Node process of its own: neither
        # schedule's figures depend on the heap and JIT state the other left
        # (the 1,000-node composite moved by 18% with the order otherwise).
        ref_drv = Driver(server.url)

        def call(*a, driver=None, **k):
            """drv.call + a progress line on stderr (a long 1,000-node run stays visibly alive)."""
            t = time.perf_counter()
            r = (driver or drv).call(*a, **k)
            print(f"[bench] {a[0]} {a[1] if len(a) > 1 else ''} {time.perf_counter() - t:.1f} s", file=sys.stderr, flush=True)
            return r

        try:
            ref_steps = args.ref_steps if args.ref_steps is not None else args.steps
            # Untimed cold opens of each schedule right before its measured ones:
            # the fake Prometheus evaluates in Python, and its first passes over a
            # 30-minute window of 1,000 nodes take seconds each (up to 10 s of
            # server work, queued on its one evaluation thread; cached afterwards),
            # which a real Prometheus does not. Both schedules are warmed the same way.
            def reference_phases():
                """Measured baseline: the reference plugin's schedule (untimed region), in its own driver process."""
                call("cold", "reference", n=2, driver=ref_drv)
                out = {"ref_cold": call("cold", "reference", n=3, driver=ref_drv),
                       "ref_cold_pages": call("coldPages", "reference", n=5, driver=ref_drv)}
                call("pages", "reference", n=max(1, args.warmup), driver=ref_drv)
                out["ref_pages"] = call("pages", "reference", n=ref_steps, driver=ref_drv)
                out["ref"] = call("steps", "reference", n=max(3, ref_steps // 2), driver=ref_drv)
                out["ref_switch"] = call("switch", "reference", n=3, driver=ref_drv)
                ref_drv.close()
                return out

            if args.order == "reference-first":
                R = reference_phases()
            # Flagship schedule.
            call("cold", "amd", n=2)
            amd_cold = call("cold", "amd", n=3)
            amd_cold_pages = call("coldPages", "amd", n=5)
            call("pages", "amd", n=max(1, args.warmup))
            D.barrier(info)
            quiet_sync()
            t0 = time.perf_counter()
            amd_pages = drv.call("pages", "amd", n=args.steps)
            quiet_sync()
            D.barrier(info)
            elapsed = time.perf_counter() - t0
            # Untimed: every page mounted in the harness React and re-rendered
            # after a refresh (element count, mount / re-render ms); and on real
            # React 18.3.1 (production builds) when this image vendors them.
            from headlamp_intel_gpu_plugin_amd.utils.reactumd import PROD_BUILDS, umd_dir
            react_out = call("pages", "amd", n=1, react=True, reactUmdDir=umd_dir(PROD_BUILDS))
            amd_react = react_out.get("react") or {}
            amd_react_dom = react_out.get("reactDom") or {}
            # Secondary: the all-pages composite refresh.
            drv.call("steps", "amd", n=1)
            amd = call("steps", "amd", n=max(3, args.steps // 2))
            amd_switch = call("switch", "amd", n=5)
            detail_out = call("detail", "amd", n=5)
            detail = detail_out["detail"]
            if args.order == "amd-first":
                R = reference_phases()
            ref_cold, ref_cold_pages, ref_pages, ref, ref_switch = (R[k] for k in (
                "ref_cold", "ref_cold_pages", "ref_pages", "ref", "ref_switch"))
            served = (server.stats() if args.control_plane == "process"
                      else {"server_requests": fc.stats(), "scrapes": scraper.scrapes if scraper else 0})
            for r in (ref_pages, amd_pages, ref, amd, ref_cold_pages, amd_cold_pages):
                if r.get("error"):
                    raise RuntimeError(r["error"])
            result = {"ref": ref, "ref_pages": ref_pages["pages"], "amd_pages": amd_pages["pages"], "ref_cold": ref_cold, "ref_switch": ref_switch,
                      "amd": amd, "amd_cold": amd_cold, "amd_switch": amd_switch, "detail": detail,
                      "ref_cold_pages": ref_cold_pages["pages"], "amd_cold_pages": amd_cold_pages["pages"],
                      "detail_slow": detail_out.get("detailSlow"), "react": amd_react, "react_dom": amd_react_dom,
                      **served}
        finally:
            drv.close()
            ref_drv.close()
            server.stop()
            if scraper:
                scraper.stop()
    else:
        # Agents serve scrapes while rank 0 measures; join its timed region.
        D.barrier(info)
        quiet_sync()
        t0 = time.perf_counter()
        quiet_sync()
        D.barrier(info)
        elapsed = time.perf_counter() - t0

    ms_per_step = D.max_float(info, elapsed * 1000.0 / max(1, args.steps))
    if burner:
        burner.stop()
    if exporter:
        exporter.stop()

    if info.is_main:
        amd_s = summarize(result["amd"]["latencies"])
        ref_s = summarize(result["ref"]["latencies"])
        rows = result["amd"]["rows"]
        pages = list(result["amd_pages"])
        per_page = {}
        for pg in pages:
            a = summarize(result["amd_pages"][pg]["latencies"])
            r = summarize(result["ref_pages"][pg]["latencies"])
            per_page[pg] = {"amd": round(a["p50"], 3), "reference": round(r["p50"], 3),
                            "amd_p95": round(a["p95"], 3), "reference_p95": round(r["p95"], 3),
                            "requests": {"amd": result["amd_pages"][pg]["requestsPerClick"],
                                         "reference": result["ref_pages"][pg]["requestsPerClick"]},
                            "speedup": round(r["p50"] / a["p50"], 2),
                            "server_ms": {"amd": _p50(result["amd_pages"][pg].get("serverMs")),
                                          "reference": _p50(result["ref_pages"][pg].get("serverMs"))}}
        value = sum(per_page[pg]["amd"] for pg in pages) / len(pages)
        ref_value = sum(per_page[pg]["reference"] for pg in pages) / len(pages)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            # v2 (round 2 on): value = mean of the per-page Refresh-click p50s.
            # v1 (round 1) was the p50 of the all-pages composite refresh, now
            # all_pages_refresh; the two are not comparable.
            "metric_version": 2,
            "unit": "ms",
            "n_gpus": info.world if info.world > 1 else args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": round(value / ref_value, 4),
            "value_definition": "mean over the 5 pages of the p50 latency of that page's Refresh click "
                                "(data committed + page rebuilt and rendered); one step = one click per page",
            # The metric is a dashboard latency, not a numeric computation.
            "dtype": "n/a",
            "workload_dtype": "bf16" if gpu and burner else None,
            "dtype_note": "dashboard latency metric; workload_dtype is the MFMA GEMM the GPU pods run meanwhile",
            "data": "synthetic cluster + synthetic/live telemetry (no real cluster or network)",
            "config": {
                "model": "amd-gpu Headlamp plugin on a synthetic 8xMI355X-per-node cluster",
                "nodes": n_nodes,
                "gpus_per_node": gpus_per_node,
                "preset": args.preset,
                "prometheus_series": args.source,
                "global_batch": None,
                "seq_len": None,
                "parallelism": f"rank-per-node x{info.world}",
                "rtt_ms": args.rtt_ms,
                "control_plane": args.control_plane,
            },
            "per_page_refresh_p50_ms": per_page,
            "baseline": {"schedule": "reference plugin request schedule replayed on the same server, per page as wired",
                         "value_ms": round(ref_value, 3)},
            # Secondary: every page's data + every view in one refresh (no
            # single reference button runs this; its replay chains the
            # provider refresh and the Metrics re-fetch).
            "all_pages_refresh": {"amd_p50_ms": round(amd_s["p50"], 3), "amd_p95_ms": round(amd_s["p95"], 3),
                                  "reference_p50_ms": round(ref_s["p50"], 3),
                                  "reference_p95_ms": round(ref_s["p95"], 3),
                                  "requests": {"amd": result["amd"]["requestsPerStep"],
                                               "reference": result["ref"]["requestsPerStep"]}},
            "request_trace_p50_ms": {k: round(v["p50_ms"], 2) for k, v in (result["amd"].get("trace") or {}).items()},
            # Data committed → all views rebuilt and rendered (composite refresh).
            "render_note": ("render in the timed click = view-model IR -> HTML string; React mount / re-render: "
                            "render_per_page (harness React), render_per_page_react_dom (real React 18.3.1)"),
            "render_p50_ms": (round(summarize(result["amd"]["renderMs"])["p50"], 3)
                              if result["amd"].get("renderMs") else None),
            # Each page opened on an empty cache, as each is wired (reference: a
            # fresh provider per route, a full-page Loader until every list and
            # the serial chain are in; Metrics then waits for it to load).
            # amd = the page complete: everything IT draws is in (Metrics: the
            # node list + its telemetry, never the pod list; GPU Nodes / GPU
            # Pods / Metrics ask for their page's telemetry once the node / pod
            # list is in on a cluster larger than one page: a second wave);
            # amd_first_content = the first render with content (progressive
            # pages: a page waits only for the lists it draws);
            # amd_content = the lists + DeviceConfig committed, i.e. everything
            # the reference's page shows.
            "cold_open_per_page_p50_ms": {
                pg: {"amd": round(summarize(result["amd_cold_pages"][pg]["latencies"])["p50"], 3),
                     "amd_first_content": round(summarize(result["amd_cold_pages"][pg]["firstMs"])["p50"], 3),
                     "amd_content": round(summarize(result["amd_cold_pages"][pg]["contentMs"])["p50"], 3),
                     # the fake server's own time on the open's slowest request (X-Server-Ms), p50 over the opens:
                     # the part of the figure that is the synthetic apiserver / Prometheus, not the plugin
                     "amd_server_ms": _p50(result["amd_cold_pages"][pg].get("serverMs")),
                     "reference_server_ms": _p50(result["ref_cold_pages"][pg].get("serverMs")),
                     "reference": round(summarize(result["ref_cold_pages"][pg]["latencies"])["p50"], 3),
                     "requests": {"amd": result["amd_cold_pages"][pg]["requests"],
                                  "reference": result["ref_cold_pages"][pg]["requests"]},
                     # the amd open's requests by kind (nodes, pods, crd, query, query_range, probe)
                     "amd_requests_by_kind": {k: v["n"] for k, v in (result["amd_cold_pages"][pg].get("trace") or {}).items()}}
                for pg in pages},
            # Per page, untimed: the page's view-model mounted in the harness
            # React through the shipped renderer (src/view/react.js), then
            # re-rendered after one refresh; elements = host nodes mounted,
            # html_elements = tags of the IR → HTML render. Bounded by the
            # pager on GPU Nodes / Metrics, whatever the node count.
            "render_per_page": {pg: {"mount_ms": round(v["mountMs"], 3), "rerender_ms": round(v["rerenderMs"], 3),
                                     "elements": v["elements"], "html_elements": v["htmlElements"]}
                                for pg, v in result["react"].items()},
            # The same page on REAL React: react@18.3.1 + react-dom@18.3.1
            # production UMD builds, committed with flushSync into a minimal
            # JS DOM (tests/js/harness/minidom.js; a browser DOM is native).
            # Median of 9 mount / re-render cycles; null when not vendored.
            "render_per_page_react_dom": ({pg: {"mount_ms": round(v["mountMs"], 3), "rerender_ms": round(v["rerenderMs"], 3),
                                                "elements": v["elements"]}
                                           for pg, v in result["react_dom"].items()} or None),
            # Secondary: every page's data (all telemetry + series) in one cold open.
            "cold_open_p50_ms": {"amd": round(summarize(result["amd_cold"]["latencies"])["p50"], 3),
                                 "reference": round(summarize(result["ref_cold"]["latencies"])["p50"], 3),
                                 "amd_server_ms": _p50(result["amd_cold"].get("serverMs")),
                                 "reference_server_ms": _p50(result["ref_cold"].get("serverMs"))},
            "schedule_order": args.order,
            # Part of the cold open spent rebuilding every view from an empty memo.
            "cold_render_p50_ms": (round(summarize(result["amd_cold"]["renderMs"])["p50"], 3)
                                   if result["amd_cold"].get("renderMs") else None),
            "route_switch_p50_ms": {"amd": round(summarize(result["amd_switch"]["latencies"])["p50"], 3),
                                    "reference": round(summarize(result["ref_switch"]["latencies"])["p50"], 3)},
            # Native Pod / Node detail page opened on a warm cluster: the node's
            # telemetry by a hostname-scoped query vs the cluster-wide snapshot.
            # The *Wired modes mount the shipped Node detail wiring and also count its list hooks.
            "detail_open": {k: dict({"p50_ms": round(summarize(v["latencies"])["p50"], 3) if v["latencies"] else None,
                                     "bytes": round(v["bytesPerOpen"]), "requests": v["requestsPerOpen"]},
                                    **{o: v[i] for i, o in (("listsPerOpen", "lists"),
                                                            ("clusterWideListsPerOpen", "cluster_wide_lists"),
                                                            ("deviceConfigRequestsPerOpen", "deviceconfig_requests"),
                                                            ("listPaths", "list_paths"), ("rendered", "rendered"))
                                       if i in v},
                                    **({"server_ms": _p50(v["serverMs"])} if v.get("serverMs") else {}))
                            for k, v in result["detail"].items()},
            "rendered": {"gpu_nodes": rows["gpuNodes"], "gpu_pods": rows["gpuPods"],
                         "gpus_monitored": rows["gpusMonitored"], "gpu_cells": rows["gpuCells"],
                         "pod_table_rows": rows["podTableRows"], "detail_sections": rows["detailSections"]},
            # Both replays fetched the same cluster: the same view-models (this
            # repo's, for both schedules) produce the same row counts. It says
            # nothing about the reference's own pages.
            "replay_fetched_same_rows": all(
                rows[k] == result["ref"]["rows"][k]
                for k in ("gpuNodes", "gpuPods", "gpusMonitored", "podTableRows", "detailSections")),
            "live_telemetry": bool(result["scrapes"]) and n_nodes > 0,
            "telemetry_source": "native amdgpu-exporter (C++/HIP) scraped every 15 s (deploy/exporter ServiceMonitor interval)" if exporter else "synthetic",
            "host": socket.gethostname(),
        }
        print(json.dumps(line), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump({"line": line, "raw": result}, f)
    D.shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
