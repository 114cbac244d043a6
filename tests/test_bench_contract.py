"""bench.py honours the driver contract (one JSON line, required keys), on 1 rank and on 2 gloo ranks."""
import json
import os
import subprocess
import sys

import pytest

from headlamp_intel_gpu_plugin_amd.utils.reactumd import PROD_BUILDS, umd_dir

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(line, n):
    assert REQUIRED <= set(line)
    assert line["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert line["n_gpus"] == n and line["steps"] == 4 and line["warmup"] == 1
    assert line["higher_is_better"] is False and line["scaling"] == "weak" and line["unit"] == "ms"
    assert 0 < line["value"] < 1000
    assert line["ms_per_step"] > 0
    # The flagship schedule must beat the replayed reference schedule.
    assert line["vs_baseline"] < 1.0
    assert line["config"]["nodes"] == n
    assert line["rendered"]["gpu_nodes"] == n
    assert line["rendered"]["gpus_monitored"] == 8 * n
    assert line["replay_fetched_same_rows"] is True
    assert line["metric_version"] == 2
    assert line["dtype"] == "n/a"
    # The headline is per page, each page's click against the reference's
    # wiring of that page's button (not the all-pages composite).
    pp = line["per_page_refresh_p50_ms"]
    assert set(pp) == {"overview", "devicePlugins", "nodes", "pods", "metrics"}
    mean = sum(v["amd"] for v in pp.values()) / 5
    assert abs(line["value"] - mean) < 1e-2
    assert abs(line["baseline"]["value_ms"] - sum(v["reference"] for v in pp.values()) / 5) < 1e-2
    for k in ("overview", "devicePlugins", "nodes", "pods"):
        assert pp[k]["requests"]["reference"] == 4  # CRD, then 3 plugin-pod selectors, in series
    assert pp["metrics"]["requests"]["reference"] == 5  # probe, then 4 queries
    for v in pp.values():
        assert v["amd"] < v["reference"], pp
    assert line["all_pages_refresh"]["requests"]["reference"] == 9
    # Cold open per page: the reference mounts a fresh provider (2 lists + CRD + 3 selectors), and its Metrics
    # page then runs discovery + 4 queries; the new plugin sends one wave (lists, CRD, the page's own query).
    cold = line["cold_open_per_page_p50_ms"]
    assert set(cold) == set(pp)
    for k in ("overview", "devicePlugins", "nodes", "pods"):
        assert cold[k]["requests"]["reference"] == 6
    assert cold["metrics"]["requests"]["reference"] == 6 + 5
    # Each route mounts what its page draws (src/plugin.js PAGE_NEEDS): Overview both lists + the DeviceConfigs;
    # GPU Nodes both lists + its telemetry query, no DeviceConfig request; Metrics the node list + its queries,
    # never the all-namespaces pod list.
    assert cold["overview"]["requests"]["amd"] == 3 and cold["nodes"]["requests"]["amd"] == 3
    assert set(cold["metrics"]["amd_requests_by_kind"]) == {"nodes", "query", "query_range"}, cold["metrics"]
    # Device Plugins: the DeviceConfigs and the operator pods' own lists (their watches' list requests), one wave,
    # no all-namespaces pod list; its Refresh is the DeviceConfig request alone (the operator pods are watched).
    assert set(cold["devicePlugins"]["amd_requests_by_kind"]) == {"operator-pods", "crd"}, cold["devicePlugins"]
    assert pp["devicePlugins"]["requests"]["amd"] == 1
    for v in cold.values():
        assert v["amd"] < v["reference"], cold
        # progressive pages: the first render with content comes no later than the page complete
        assert v["amd_first_content"] <= v["amd"] + 1e-6, cold
    # Every page mounted through the shipped renderer on the harness React and,
    # where this image vendors them, on real React 18.3.1 production builds:
    # the same IR mounts the same host elements on both.
    harness, real = line["render_per_page"], line["render_per_page_react_dom"]
    assert set(harness) == set(pp)
    if umd_dir(PROD_BUILDS):
        assert set(real) == set(pp)
        for k in pp:
            assert real[k]["elements"] == harness[k]["elements"] > 0, (k, real[k], harness[k])
            assert real[k]["mount_ms"] > 0 and real[k]["rerender_ms"] > 0


def test_bench_single_rank():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--rtt-ms", "10"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 1)


def test_bench_node_exporter_only_cluster_is_one_wave():
    """A Prometheus with node-exporter's amdgpu hwmon series only (the fallback source): every GPU is monitored and
    GPU Nodes / Metrics cold-open in one wave — one query (Metrics: plus its range query), no second cluster-wide read."""
    r = subprocess.run([sys.executable, "bench.py", "--nodes", "2", "--source", "node-exporter", "--steps", "2",
                        "--warmup", "1", "--rtt-ms", "5", "--no-burn"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_lines(r.stdout)[-1]
    assert line["config"]["prometheus_series"] == "node-exporter"
    assert line["rendered"]["gpus_monitored"] == 16
    cold = line["cold_open_per_page_p50_ms"]
    assert cold["nodes"]["amd_requests_by_kind"].get("query") == 1, cold["nodes"]
    assert cold["metrics"]["amd_requests_by_kind"].get("query") == 1, cold["metrics"]


def test_bench_two_ranks_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29541", "bench.py", "--gpus", "2",
                        "--steps", "4", "--warmup", "1", "--rtt-ms", "10"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    _check(lines[0], 2)


@pytest.mark.parametrize("n", [4])
def test_bench_node_override(n):
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--rtt-ms", "10", "--nodes", str(n)],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_lines(r.stdout)[0]
    assert line["config"]["nodes"] == n and line["rendered"]["gpu_nodes"] == n


def test_detail_pages_cost_one_node_of_telemetry_whatever_the_cluster_size():
    # Native Pod / Node detail pages fetch their node's telemetry with a
    # hostname-scoped query: one request, the same bytes on 1 and on 16
    # nodes, where the cluster-wide snapshot grows with the GPU count.
    out = {}
    for n in (1, 16):
        r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--rtt-ms", "5",
                            "--nodes", str(n)], cwd=ROOT, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        out[n] = _json_lines(r.stdout)[0]["detail_open"]
    for kind in ("podScoped", "nodeScoped"):
        assert out[1][kind]["requests"] == 1 and out[16][kind]["requests"] == 1
        assert abs(out[16][kind]["bytes"] - out[1][kind]["bytes"]) <= 0.05 * out[1][kind]["bytes"], out
    assert out[16]["podClusterWide"]["bytes"] > 10 * out[16]["podScoped"]["bytes"], out
    # The Pod detail page as wired: node telemetry + the pod's power history, two requests in one wave, bytes
    # independent of the cluster size, latency one round trip (RTT 5 ms here).
    for kind, one in (("podDetail", "podScoped"), ("nodeDetail", "nodeScoped")):
        pd = out[16][kind]
        assert pd["requests"] == 2 and out[1][kind]["requests"] == 2, out
        assert abs(pd["bytes"] - out[1][kind]["bytes"]) <= 0.05 * out[1][kind]["bytes"], out
        assert pd["p50_ms"] < 2 * out[16][one]["p50_ms"] + 5, out
    # A Node detail opened on a cold store (no plugin page visited): its node's pods by field selector, its
    # telemetry and its power history — three requests in ONE wave, the same bytes on 1 and 16 nodes. The
    # reference mounts its full provider there: both cluster-wide lists + CRD + 3 serial requests, growing bytes.
    cold, ref = out[16]["nodeDetailCold"], out[16]["nodeDetailColdReference"]
    assert cold["requests"] == 3 and out[1]["nodeDetailCold"]["requests"] == 3, out
    assert abs(cold["bytes"] - out[1]["nodeDetailCold"]["bytes"]) <= 0.05 * out[1]["nodeDetailCold"]["bytes"], out
    assert cold["p50_ms"] < 2 * out[16]["nodeScoped"]["p50_ms"] + 5, out
    assert ref["requests"] == 6 and ref["bytes"] > 3 * out[1]["nodeDetailColdReference"]["bytes"], out
    assert ref["p50_ms"] > 2 * cold["p50_ms"], out  # 4 serial round trips after the lists against one wave
    # The same open through the shipped wiring (src/plugin.js NodeDetailHost, harness React, list hooks that are
    # real list requests), after GPU Nodes was visited and unmounted — Headlamp's way to a Node page — and cold:
    # one list hook, scoped to the node; no cluster-wide list, no DeviceConfig request; flat bytes.
    for kind in ("nodeDetailWired", "nodeDetailWiredCold"):
        for n in (1, 16):
            w = out[n][kind]
            assert w["rendered"] is True and w["requests"] == 3, (kind, n, w)
            assert w["lists"] == 1 and w["cluster_wide_lists"] == 0 and w["deviceconfig_requests"] == 0, (kind, n, w)
            assert all("fieldSelector=spec.nodeName" in p for p in w["list_paths"]), w
        assert abs(out[16][kind]["bytes"] - out[1][kind]["bytes"]) <= 0.05 * out[1][kind]["bytes"], out
    # The GPU Pods page asks for pod attribution only: one series per allocated GPU.
    assert out[16]["podsPageOwners"]["requests"] == 1
    assert out[16]["podsPageOwners"]["bytes"] < 0.1 * out[16]["podClusterWide"]["bytes"], out


def test_watch_churn_stress_is_incremental():
    # bench/stress.js: the store + all five view-models per pod watch event
    # against a replay of the reference's full recompute. The growth claim
    # rests on the store's WORK COUNTERS, which are deterministic for the
    # seeded event stream; per-event wall time on a shared 8-core box is noise
    # at these sizes (a p50 of 0.1-0.5 ms moves with JIT tiering and other
    # load), so it is only bounded loosely and reported.
    out = os.path.join(ROOT, "gpurun_out", "test_stress.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run(["node", "--expose-gc", "bench/stress.js", "--nodes", "16,128", "--events", "300",
                        "--out", out], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    pts = json.load(open(out))["points"]
    small, big = pts
    assert big["pods"] > 7 * small["pods"]
    for p in pts:
        assert p["consistent"], p
        c = p["storeCounters"]
        pc = c["pods"]
        n, ev = p["pods"], p["events"]
        # The list tracker identity-compares the unchanged prefix / suffix:
        # at most one pointer compare per pod per delivered list.
        assert pc["compared"] <= pc["updates"] * (n + ev), pc
        # Only changed pods are classified: the first list + about one per event.
        assert pc["classified"] < n + 2 * ev, pc
        # GPU-pod events patch the cluster index instead of rebuilding it.
        assert c["indexPatches"] > 5 * c["indexBuilds"], c
    # Classification work per event does not grow with the cluster (O(changed)):
    # the same bound at 588 and at 4,744 pods.
    for p in pts:
        assert (p["storeCounters"]["pods"]["classified"] - p["pods"]) / p["events"] <= 2, p["storeCounters"]
    # Wall time: a loose absolute sanity bound only. The reference replay's mean
    # (it re-filters every pod per event) is reported next to it, not compared:
    # at these sizes the difference is within this box's timing noise.
    assert big["amd"]["p50"] < 5.0, big["amd"]
    print("stress per-event mean ms, amd vs reference replay:", big["amd"]["mean"], big["reference"]["mean"])
