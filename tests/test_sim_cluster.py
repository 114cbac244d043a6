"""Synthetic cluster, fake control plane and their agreement with the JS constants."""
import json
import os
import re
import time
import urllib.error
import urllib.parse
import urllib.request

import pytest

from headlamp_intel_gpu_plugin_amd.models.cluster import (PRESETS, ClusterSpec, SyntheticCluster, gpu_node_name,
                                                          spec_for_nodes)
from headlamp_intel_gpu_plugin_amd.models.telemetry import populate, pci_address
from headlamp_intel_gpu_plugin_amd.sim import promql
from headlamp_intel_gpu_plugin_amd.sim.apiserver import (DEFAULT_PROM_SERVICE, FakeCluster, ServerThread, make_fake,
                                                         parse_field_selector, parse_label_selector)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = open(os.path.join(ROOT, "src", "api", "k8sCore.js")).read()


def js_const(name):
    m = re.search(r"export const " + name + r" = '([^']*)'", JS)
    assert m, name
    return m.group(1)


# ---------------------------------------------------------------------------
# cluster model
# ---------------------------------------------------------------------------

def test_presets_match_baseline_configs():
    assert set(PRESETS) == {"cpu-only", "1x1", "1x8", "4x8", "8x8"}
    assert SyntheticCluster(PRESETS["cpu-only"]).expected_counts()["gpu_nodes"] == 0
    assert SyntheticCluster(PRESETS["1x1"]).expected_counts()["gpus"] == 1


def test_single_node_has_four_gpu_pods_running():
    c = SyntheticCluster(PRESETS["1x8"])
    e = c.expected_counts()
    assert e["running_gpu_pods"] == 4
    assert e["gpus"] == 8 and e["gpus_in_use"] == 6


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_scaling_specs(n):
    c = SyntheticCluster(spec_for_nodes(n))
    assert len(c.gpu_nodes) == n
    assert c.expected_counts()["gpus"] == 8 * n
    names = [p["metadata"]["name"] for p in c.pods]
    assert len(names) == len(set(names))


def test_cluster_is_deterministic():
    a = json.dumps(SyntheticCluster(spec_for_nodes(2)).pods, sort_keys=True)
    b = json.dumps(SyntheticCluster(spec_for_nodes(2)).pods, sort_keys=True)
    assert a == b


def test_labels_and_resources_agree_with_js_constants():
    c = SyntheticCluster(spec_for_nodes(1))
    node = c.gpu_nodes[0]
    assert node["metadata"]["labels"][js_const("AMD_NFD_GPU_LABEL")] == "true"
    assert js_const("LABEL_PRODUCT_NAME") in node["metadata"]["labels"]
    assert node["status"]["capacity"][js_const("AMD_GPU_RESOURCE")] == "8"
    dc = c.device_configs[0]
    assert dc["kind"] == js_const("DEVICE_CONFIG_KIND")
    assert dc["apiVersion"] == js_const("AMD_GPU_OPERATOR_API_GROUP") + "/" + js_const("AMD_GPU_OPERATOR_API_VERSION")
    assert dc["metadata"]["namespace"] == js_const("AMD_GPU_OPERATOR_NAMESPACE")


def test_standalone_plugin_pods_use_js_labels():
    c = SyntheticCluster(ClusterSpec(gpu_nodes=1, standalone_plugin=True, operator=False))
    labels = {p["metadata"]["labels"].get("name") for p in c.pods}
    assert js_const("AMD_DEVICE_PLUGIN_POD_LABEL") in labels
    assert js_const("AMD_NODE_LABELLER_POD_LABEL") in labels
    assert not c.device_configs


def test_partition_labels():
    c = SyntheticCluster(ClusterSpec(gpu_nodes=1, partition="cpx/nps4"))
    labels = c.gpu_nodes[0]["metadata"]["labels"]
    assert labels["amd.com/compute-partitioning-mode"] == "cpx"
    assert c.gpu_nodes[0]["status"]["capacity"]["amd.com/gpu"] == "64"  # 8 boards x 8 CPX partitions


# ---------------------------------------------------------------------------
# telemetry
# ---------------------------------------------------------------------------

def test_exporter_telemetry_series_counts():
    c = SyntheticCluster(spec_for_nodes(2))
    db = promql.TSDB()
    n = populate(db, c, source="amd-exporter")
    assert n == 2 * 8 * (10 + 7 + 7)  # 8 gauges + 2 RAS counters + 7 xGMI throughput + 7 link-hop series per GPU


def test_busy_gpus_draw_more_power_and_carry_pod_labels():
    c = SyntheticCluster(spec_for_nodes(1))
    db = promql.TSDB()
    populate(db, c)
    body = promql.query(db, "gpu_power_usage", 1000.0)
    rows = json.loads(body)["data"]["result"]
    busy = [float(r["value"][1]) for r in rows if "pod" in r["metric"]]
    idle = [float(r["value"][1]) for r in rows if "pod" not in r["metric"]]
    assert len(busy) == 6 and len(idle) == 2
    assert min(busy) > max(idle)
    assert max(busy) <= 1400


def test_node_exporter_telemetry():
    c = SyntheticCluster(spec_for_nodes(1))
    db = promql.TSDB()
    populate(db, c, source="node-exporter")
    r = json.loads(promql.query(db, 'node_hwmon_chip_names{chip_name="amdgpu"}', 1000.0))["data"]["result"]
    assert len(r) == 8
    assert r[0]["metric"]["chip"] == pci_address(0, 0)


def test_xgmi_traffic_only_between_gpus_of_one_pod():
    c = SyntheticCluster(spec_for_nodes(1))
    db = promql.TSDB()
    populate(db, c)
    r = json.loads(promql.query(db, '{__name__=~"xgmi_neighbor_[0-6]_tx_throughput"} > 0', 1000.0))["data"]["result"]
    # pods hold GPUs {0},{1},{2,3},{4,5}: two 2-GPU pods → 2 directed links each
    assert len(r) == 4


# ---------------------------------------------------------------------------
# selectors
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("sel,labels,ok", [
    ("app=web", {"app": "web"}, True),
    ("app==web", {"app": "web"}, True),
    ("app!=web", {"app": "web"}, False),
    ("name in (a,b)", {"name": "b"}, True),
    ("name notin (a,b)", {"name": "b"}, False),
    ("tier", {"tier": "x"}, True),
    ("!tier", {"tier": "x"}, False),
    ("app=web,tier in (fe)", {"app": "web", "tier": "fe"}, True),
    ("", {}, True),
])
def test_label_selector(sel, labels, ok):
    assert parse_label_selector(sel)(labels) is ok


def test_label_selector_rejects_garbage():
    with pytest.raises(ValueError):
        parse_label_selector("a b c")


def test_field_selector():
    pod = {"spec": {"nodeName": "n1"}, "status": {"phase": "Running"}}
    assert parse_field_selector("spec.nodeName=n1")(pod)
    assert not parse_field_selector("status.phase!=Running")(pod)


# ---------------------------------------------------------------------------
# HTTP surface
# ---------------------------------------------------------------------------

@pytest.fixture(scope="module")
def server():
    fc = make_fake(2, source="both", latency_ms=0)
    with ServerThread(fc) as s:
        yield s


def get(server, path):
    try:
        with urllib.request.urlopen(server.url + path, timeout=10) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


PROM = "/api/v1/namespaces/monitoring/services/kube-prometheus-stack-prometheus:9090/proxy/api/v1/"


def test_lists(server):
    st, nodes = get(server, "/api/v1/nodes")
    assert st == 200 and nodes["kind"] == "NodeList" and len(nodes["items"]) == 5
    st, pods = get(server, "/api/v1/pods")
    assert st == 200 and len(pods["items"]) > 50


def test_namespaced_pods_and_selectors(server):
    _, ns = get(server, "/api/v1/namespaces/kube-amd-gpu/pods")
    assert all(p["metadata"]["namespace"] == "kube-amd-gpu" for p in ns["items"])
    q = urllib.parse.quote("app=kube-proxy")
    _, sel = get(server, "/api/v1/pods?labelSelector=" + q)
    assert len(sel["items"]) == 5
    _, fs = get(server, "/api/v1/pods?fieldSelector=" + urllib.parse.quote("spec.nodeName=" + gpu_node_name(1)))
    assert all(p["spec"]["nodeName"] == gpu_node_name(1) for p in fs["items"])
    # The plugin's label-selector request leaves out the operator namespace (disjoint from the namespace request).
    _, every = get(server, "/api/v1/pods")
    _, rest = get(server, "/api/v1/pods?fieldSelector=" + urllib.parse.quote("metadata.namespace!=kube-amd-gpu"))
    assert rest["items"] and all(p["metadata"]["namespace"] != "kube-amd-gpu" for p in rest["items"])
    assert len(rest["items"]) + len(ns["items"]) == len(every["items"])


def test_bad_selector_is_400(server):
    st, body = get(server, "/api/v1/pods?labelSelector=" + urllib.parse.quote("a b"))
    assert st == 400 and body["kind"] == "Status"


def test_deviceconfigs(server):
    st, body = get(server, "/apis/amd.com/v1alpha1/deviceconfigs")
    assert st == 200 and body["items"][0]["kind"] == "DeviceConfig"
    st, body = get(server, "/apis/amd.com/v1alpha1/namespaces/other/deviceconfigs")
    assert st == 200 and body["items"] == []


def test_prometheus_query_and_range(server):
    st, body = get(server, PROM + "query?query=1")
    assert st == 200 and body["status"] == "success"
    st, body = get(server, PROM + "query?query=" + urllib.parse.quote("sum(gpu_power_usage)"))
    assert st == 200 and float(body["data"]["result"][0]["value"][1]) > 0
    st, body = get(server, PROM + "query_range?query=gpu_power_usage&start=1000&end=1060&step=30")
    assert st == 200 and body["data"]["resultType"] == "matrix"


def test_prometheus_errors(server):
    st, body = get(server, PROM + "query?query=" + urllib.parse.quote("sum("))
    assert st == 400 and body["status"] == "error"
    st, body = get(server, PROM + "query_range?query=x&start=a&end=1&step=1")
    assert st == 400


def test_unreachable_prometheus_service_is_503(server):
    st, body = get(server, "/api/v1/namespaces/monitoring/services/prometheus:9090/proxy/api/v1/query?query=1")
    assert st == 503 and body["reason"] == "ServiceUnavailable"


def test_crd_missing_is_404():
    fc = make_fake(1, latency_ms=0, crd_installed=False)
    with ServerThread(fc) as s:
        st, body = get(s, "/apis/amd.com/v1alpha1/deviceconfigs")
    assert st == 404 and body["reason"] == "NotFound"


def test_latency_injection_and_stats():
    import time

    fc = FakeCluster(SyntheticCluster(spec_for_nodes(1)), latency_ms=50, prometheus_up=[DEFAULT_PROM_SERVICE])
    with ServerThread(fc) as s:
        t = time.perf_counter()
        get(s, "/api/v1/nodes")
        dt = time.perf_counter() - t
    assert dt >= 0.05
    assert fc.stats() == {"apiserver": 1, "total": 1}


def test_list_cache_invalidation():
    fc = FakeCluster(SyntheticCluster(spec_for_nodes(1)), latency_ms=0)
    a = fc.nodes_body("")
    assert fc.nodes_body("") is a
    fc.cluster.nodes.pop()
    fc.bump()
    assert fc.nodes_body("") != a


def test_recording_rule_answers_and_server_time(monkeypatch):
    """rules=True (the benchmark's control plane): the first instant query is evaluated for its caller, later ones
    are served the kept answer; the ticker re-evaluates it once its inputs changed, in a lull of client requests and
    no more often than RULE_EVAL_S; every response says its server time (X-Server-Ms)."""
    from headlamp_intel_gpu_plugin_amd.sim import apiserver

    monkeypatch.setattr(apiserver, "RULE_EVAL_S", 0.0)
    monkeypatch.setattr(apiserver, "RULE_IDLE_S", 0.2)
    fc = make_fake(1, source="amd-exporter", latency_ms=0, rules=True)
    clock = [fc.now()]
    fc.now = lambda: clock[0]
    q = PROM + "query?query=" + urllib.parse.quote("sum(gpu_power_usage)")
    with ServerThread(fc) as s:
        with urllib.request.urlopen(s.url + q, timeout=10) as r:
            first = json.loads(r.read())
            assert float(r.headers["X-Server-Ms"]) >= 0
        assert fc.rule_evals == 1 and first["status"] == "success"
        for _ in range(3):
            assert get(s, q)[1] == first
        assert fc.rule_evals == 1  # served, not evaluated
        clock[0] += 60.0  # the sample grid ticks: the kept answer is behind its inputs
        deadline = time.time() + 10
        while fc.rule_evals == 1 and time.time() < deadline:
            time.sleep(0.05)
        assert fc.rule_evals == 2
        assert get(s, q)[1]["data"]["result"]
        # A request of any kind says its server time.
        with urllib.request.urlopen(s.url + "/api/v1/nodes", timeout=10) as r:
            assert float(r.headers["X-Server-Ms"]) >= 0


def test_rule_refreshes_wait_for_a_lull(monkeypatch):
    """A refresh does not start while client requests keep arriving (the evaluation thread cannot pre-empt it),
    unless the answer is RULE_STALE_S old."""
    from headlamp_intel_gpu_plugin_amd.sim import apiserver

    monkeypatch.setattr(apiserver, "RULE_EVAL_S", 0.0)
    monkeypatch.setattr(apiserver, "RULE_IDLE_S", 5.0)
    fc = make_fake(1, source="amd-exporter", latency_ms=0, rules=True)
    clock = [fc.now()]
    fc.now = lambda: clock[0]
    q = PROM + "query?query=" + urllib.parse.quote("count(gpu_power_usage)")
    with ServerThread(fc) as s:
        get(s, q)
        clock[0] += 60.0
        end = time.time() + 1.5
        while time.time() < end:  # a steady stream of requests: no lull of 5 s
            get(s, "/api/v1/nodes")
            time.sleep(0.1)
        assert fc.rule_evals == 1
        monkeypatch.setattr(apiserver, "RULE_STALE_S", 0.0)  # an answer this old is refreshed whatever the load
        end = time.time() + 10
        while fc.rule_evals == 1 and time.time() < end:
            get(s, "/api/v1/nodes")
            time.sleep(0.05)
        assert fc.rule_evals == 2


def test_a_failed_rule_refresh_is_retried_and_an_unstamped_answer_still_refreshes(monkeypatch):
    """A background refresh that raises (its future has no one awaiting it) leaves the query schedulable: the next
    tick evaluates it again. With no input stamp (series sampled at mixed intervals) the answer counts as changed, so
    the age limits still refresh it."""
    from headlamp_intel_gpu_plugin_amd.sim import apiserver

    monkeypatch.setattr(apiserver, "RULE_EVAL_S", 0.0)
    monkeypatch.setattr(apiserver, "RULE_IDLE_S", 0.0)
    fc = make_fake(1, source="amd-exporter", latency_ms=0, rules=True)
    clock = [fc.now()]
    fc.now = lambda: clock[0]
    real = apiserver.promql.query
    calls = []

    def flaky(db, q, t):
        calls.append(q)
        if len(calls) == 2:
            raise RuntimeError("evaluation failed once")
        return real(db, q, t)

    monkeypatch.setattr(apiserver.promql, "query", flaky)
    q = PROM + "query?query=" + urllib.parse.quote("max(gpu_power_usage)")
    with ServerThread(fc) as s:
        assert get(s, q)[1]["status"] == "success"
        clock[0] += 60.0
        deadline = time.time() + 10
        while fc.rule_evals < 2 and time.time() < deadline:
            time.sleep(0.05)
        assert len(calls) >= 3 and fc.rule_evals == 2  # the failure, then the retry
        assert not fc.refreshing or fc.refreshing == {urllib.parse.unquote(q.split("query=")[1])}
        monkeypatch.setattr(apiserver.promql, "cache_stamp", lambda db, t: None)
        before = fc.rule_evals
        deadline = time.time() + 10
        while fc.rule_evals == before and time.time() < deadline:  # clock unchanged: only the missing stamp
            time.sleep(0.05)
        assert fc.rule_evals > before


def test_priority_pool_runs_client_work_before_queued_rule_refreshes():
    """The fake Prometheus's one evaluation thread takes a client request (priority 0) before rule refreshes
    (priority 1) that were queued earlier; equal priorities keep their order."""
    import threading

    from headlamp_intel_gpu_plugin_amd.sim.apiserver import PriorityPool

    pool = PriorityPool("test-pool")
    try:
        gate = threading.Event()
        order = []
        first = pool.submit(1, gate.wait, 10)  # occupies the thread until released
        queued = [pool.submit(1, order.append, f"rule{i}") for i in range(3)]
        client = pool.submit(0, order.append, "client")
        gate.set()
        for f in [first, client] + queued:
            f.result(timeout=10)
        assert order == ["client", "rule0", "rule1", "rule2"]
        # An exception reaches the caller and the thread keeps serving.
        bad = pool.submit(0, lambda: 1 / 0)
        with pytest.raises(ZeroDivisionError):
            bad.result(timeout=10)
        assert pool.submit(0, lambda: 42).result(timeout=10) == 42
    finally:
        pool.shutdown()
