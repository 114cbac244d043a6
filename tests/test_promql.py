"""PromQL-subset evaluator (sim/promql.py) against hand-computed expectations."""
import json
import math

import pytest

from headlamp_intel_gpu_plugin_amd.sim import promql
from headlamp_intel_gpu_plugin_amd.sim.promql import TSDB, Series, parse, query, query_range


@pytest.fixture()
def db():
    d = TSDB()
    for node in ("n0", "n1"):
        for g in range(2):
            base = 100.0 * (1 if node == "n0" else 2) + g
            d.add(Series({"__name__": "gpu_power_usage", "hostname": node, "gpu_id": str(g)}, fn=lambda t, b=base: b))
            d.add(Series({"__name__": "gpu_gfx_activity", "hostname": node, "gpu_id": str(g)}, fn=lambda t: 50.0))
    # counter increasing 2/s
    d.add(Series({"__name__": "energy_total", "chip": "c0", "instance": "i0"}, fn=lambda t: 2.0 * t))
    d.add(Series({"__name__": "chip_names", "chip": "c0", "instance": "i0", "chip_name": "amdgpu"}, fn=lambda t: 1.0))
    d.add(Series({"__name__": "chip_names", "chip": "c1", "instance": "i0", "chip_name": "k10temp"}, fn=lambda t: 1.0))
    return d


def _vec(body):
    if isinstance(body, str):
        body = json.loads(body)
    assert body["status"] == "success", body
    return body["data"]["result"]


def test_scalar_literal(db):
    body = query(db, "1", 1000.0)
    assert body["data"]["resultType"] == "scalar"
    assert body["data"]["result"][1] == "1"


def test_selector_by_name(db):
    assert len(_vec(query(db, "gpu_power_usage", 1000.0))) == 4


def test_label_matchers(db):
    r = _vec(query(db, 'gpu_power_usage{hostname="n1",gpu_id!="0"}', 1000.0))
    assert len(r) == 1 and r[0]["value"][1] == "201"


def test_regex_name_selector(db):
    r = _vec(query(db, '{__name__=~"gpu_power_usage|gpu_gfx_activity"}', 1000.0))
    assert len(r) == 8
    assert {x["metric"]["__name__"] for x in r} == {"gpu_power_usage", "gpu_gfx_activity"}


def test_negative_regex(db):
    r = _vec(query(db, 'chip_names{chip_name!~"k10.*"}', 1000.0))
    assert [x["metric"]["chip"] for x in r] == ["c0"]


def test_sum_by(db):
    r = _vec(query(db, "sum by (hostname) (gpu_power_usage)", 1000.0))
    got = {x["metric"]["hostname"]: float(x["value"][1]) for x in r}
    assert got == {"n0": 201.0, "n1": 401.0}


def test_aggregation_clause_after_body(db):
    r = _vec(query(db, "max(gpu_power_usage) by (hostname)", 1000.0))
    assert {x["metric"]["hostname"]: float(x["value"][1]) for x in r} == {"n0": 101.0, "n1": 201.0}


def test_avg_count_min_without(db):
    assert float(_vec(query(db, "avg(gpu_power_usage)", 1000.0))[0]["value"][1]) == pytest.approx(150.5)
    assert float(_vec(query(db, "count(gpu_power_usage)", 1000.0))[0]["value"][1]) == 4
    r = _vec(query(db, "min without (gpu_id) (gpu_power_usage)", 1000.0))
    assert {x["metric"]["hostname"]: float(x["value"][1]) for x in r} == {"n0": 100.0, "n1": 200.0}


def test_rate_of_counter(db):
    r = _vec(query(db, "rate(energy_total[5m])", 1000.0))
    assert float(r[0]["value"][1]) == pytest.approx(2.0)
    assert "__name__" not in r[0]["metric"]


def test_increase_and_irate(db):
    assert float(_vec(query(db, "increase(energy_total[1m])", 1000.0))[0]["value"][1]) == pytest.approx(120.0)
    assert float(_vec(query(db, "irate(energy_total[1m])", 1000.0))[0]["value"][1]) == pytest.approx(2.0)


def test_over_time_functions(db):
    assert float(_vec(query(db, "avg_over_time(gpu_gfx_activity[5m])", 1000.0))[0]["value"][1]) == 50.0
    assert float(_vec(query(db, "count_over_time(gpu_gfx_activity[1m])", 1005.0))[0]["value"][1]) == 4


def test_group_left_join(db):
    q = 'rate(energy_total[5m]) * on(chip,instance) group_left(chip_name) chip_names{chip_name="amdgpu"}'
    r = _vec(query(db, q, 1000.0))
    assert len(r) == 1
    assert r[0]["metric"]["chip_name"] == "amdgpu"
    assert float(r[0]["value"][1]) == pytest.approx(2.0)


def test_scalar_vector_arithmetic(db):
    r = _vec(query(db, 'gpu_power_usage{hostname="n0",gpu_id="0"} / 2 + 1', 1000.0))
    assert float(r[0]["value"][1]) == 51.0


def test_comparison_filters(db):
    r = _vec(query(db, "gpu_power_usage > 150", 1000.0))
    assert {x["metric"]["hostname"] for x in r} == {"n1"}
    assert all(x["metric"]["__name__"] == "gpu_power_usage" for x in r)


def test_unary_minus(db):
    assert float(_vec(query(db, '-gpu_power_usage{hostname="n0",gpu_id="1"}', 1000.0))[0]["value"][1]) == -101.0


def test_many_to_many_is_an_error(db):
    body = query(db, "gpu_power_usage * on(hostname) gpu_gfx_activity", 1000.0)
    assert body["status"] == "error"


def test_parse_errors_are_reported(db):
    for bad in ("sum(", "gpu_power_usage{hostname=}", "rate(gpu_power_usage)", "@@"):
        assert query(db, bad, 1000.0)["status"] == "error", bad


def test_query_range_matrix(db):
    body = json.loads(query_range(db, "sum by (hostname) (gpu_power_usage)", 1000.0, 1060.0, 30.0))
    res = body["data"]["result"]
    assert body["data"]["resultType"] == "matrix"
    assert len(res) == 2 and all(len(r["values"]) == 3 for r in res)


def test_query_range_rejects_bad_range(db):
    assert query_range(db, "gpu_power_usage", 10.0, 0.0, 1.0)["status"] == "error"
    assert query_range(db, "gpu_power_usage", 0.0, 1e9, 1.0)["status"] == "error"


def test_pushed_series_lookback():
    d = TSDB()
    s = d.add(Series({"__name__": "live"}))
    s.push(100.0, 1.0)
    s.push(110.0, 2.0)
    s.push(105.0, 9.0)  # out of order: dropped
    assert _vec(query(d, "live", 120.0))[0]["value"][1] == "2"
    assert _vec(query(d, "live", 110.0 + promql.LOOKBACK_S + 1)) == []


def test_pushed_series_cap():
    s = Series({"__name__": "x"}, cap=3)
    for t in range(10):
        s.push(float(t), float(t))
    assert s.ts == [7.0, 8.0, 9.0]


def test_select_cache_invalidated_on_add(db):
    assert len(_vec(query(db, "gpu_power_usage", 1.0))) == 4
    db.add(Series({"__name__": "gpu_power_usage", "hostname": "n2", "gpu_id": "0"}, fn=lambda t: 1.0))
    assert len(_vec(query(db, "gpu_power_usage", 1.0))) == 5


def test_nan_and_inf_formatting():
    assert promql._fmt(math.nan) == "NaN"
    assert promql._fmt(math.inf) == "+Inf"
    assert promql._fmt(2.0) == "2"


def test_parse_ast_shapes():
    assert parse("1")[0] == "num"
    node = parse("x[5m]")
    assert node[0] == "sel" and node[2] == 300.0 and node[1][0].value == "x"
    assert parse("sum by (a) (x)")[0] == "agg"


def test_instant_cache_sees_pushes_and_interval_changes():
    db = promql.TSDB()
    live = db.add(promql.Series({"__name__": "gpu_power_usage", "hostname": "n0"}))
    db.add(promql.Series({"__name__": "gpu_power_usage", "hostname": "n1"}, fn=lambda t: t, interval=15))
    live.push(100.0, 1.0)
    q = "gpu_power_usage"

    def values(t):
        return {r["metric"]["hostname"]: float(r["value"][1]) for r in json.loads(promql.query(db, q, t))["data"]["result"]}

    assert values(101.0) == {"n0": 1.0, "n1": 90.0}
    live.push(102.0, 7.0)  # a push invalidates the cached result
    assert values(103.0)["n0"] == 7.0
    assert values(106.0)["n1"] == 105.0  # next 15 s bucket re-evaluates fn series
    body = json.loads(promql.query(db, q, 107.5))
    assert body["data"]["result"][0]["value"][0] == 107.5  # eval timestamp is current, not cached



def test_range_memo_keeps_steps_a_push_cannot_change():
    """A push between two range queries re-evaluates only the steps at or after the pushed sample, and the
    answer equals a fresh evaluation (cache cleared)."""
    db = promql.TSDB()
    live = db.add(promql.Series({"__name__": "gpu_power_usage", "hostname": "n0"}))
    db.add(promql.Series({"__name__": "gpu_power_usage", "hostname": "n1"}, fn=lambda t: t, interval=15))
    for t in range(0, 600, 10):
        live.push(float(t), float(t) / 10)
    q = "sum by (hostname) (gpu_power_usage)"
    first = json.loads(promql.query_range(db, q, 0.0, 600.0, 30.0))
    steps = db._range_cache[q][1]
    assert len(steps) == 21
    before = {t: steps[t] for t in steps}
    live.push(605.0, 99.0)  # changes what is seen from t = 605 on
    again = json.loads(promql.query_range(db, q, 0.0, 630.0, 30.0))
    steps = db._range_cache[q][1]
    assert all(steps[t] is before[t] for t in before if t < 605.0)  # reused, not re-evaluated
    db._range_cache.clear()
    fresh = json.loads(promql.query_range(db, q, 0.0, 630.0, 30.0))
    assert again == fresh
    assert first["data"]["result"][0]["values"][:21] == fresh["data"]["result"][0]["values"][:21]
    # a new series changes every step
    db.add(promql.Series({"__name__": "gpu_power_usage", "hostname": "n2"}, fn=lambda t: 1.0, interval=15))
    promql.query_range(db, q, 0.0, 630.0, 30.0)
    assert len(json.loads(promql.query_range(db, q, 0.0, 630.0, 30.0))["data"]["result"]) == 3


def test_range_memo_drops_steps_that_saw_dropped_samples():
    db = promql.TSDB()
    s = db.add(promql.Series({"__name__": "x"}, cap=5))
    for t in range(0, 50, 10):
        s.push(float(t), 1.0)
    assert len(json.loads(promql.query_range(db, "x", 0.0, 40.0, 10.0))["data"]["result"][0]["values"]) == 5
    s.push(50.0, 2.0)  # drops the sample at 0: what t in [0, 300] saw may change
    again = json.loads(promql.query_range(db, "x", 0.0, 50.0, 10.0))
    db._range_cache.clear()
    assert again == json.loads(promql.query_range(db, "x", 0.0, 50.0, 10.0))


# ---- set operators and label_replace (the paged views' scoped + summary queries) ----

def test_or_keeps_lhs_and_adds_unmatched_rhs_ignoring_the_name(db):
    # Prometheus matches `or` on every label but __name__: gfx rows carry the same
    # hostname/gpu_id sets as the power rows, so none of them is added.
    rows = _vec(query(db, "gpu_power_usage or gpu_gfx_activity", 1000.0))
    assert len(rows) == 4 and {r["metric"]["__name__"] for r in rows} == {"gpu_power_usage"}
    rows = _vec(query(db, 'gpu_power_usage{hostname="n0"} or gpu_gfx_activity{hostname="n1"}', 1000.0))
    assert sorted((r["metric"]["__name__"], r["metric"]["hostname"]) for r in rows) == [
        ("gpu_gfx_activity", "n1"), ("gpu_gfx_activity", "n1"), ("gpu_power_usage", "n0"), ("gpu_power_usage", "n0")]


def test_or_on_name_keeps_both_metrics(db):
    rows = _vec(query(db, "gpu_power_usage or on(__name__, hostname, gpu_id) gpu_gfx_activity", 1000.0))
    assert len(rows) == 8


def test_and_unless(db):
    assert len(_vec(query(db, 'gpu_power_usage and on(hostname) gpu_gfx_activity{hostname="n1"}', 1000.0))) == 2
    rows = _vec(query(db, 'gpu_power_usage unless on(hostname) gpu_gfx_activity{hostname="n1"}', 1000.0))
    assert {r["metric"]["hostname"] for r in rows} == {"n0"}


def test_or_binds_weaker_than_arithmetic(db):
    # (sum * 2) or (count): tagged so both survive
    q = ('label_replace(sum(gpu_power_usage) * 2, "agg", "double", "", "") or '
         'label_replace(count(gpu_power_usage), "agg", "n", "", "")')
    rows = {r["metric"]["agg"]: float(r["value"][1]) for r in _vec(query(db, q, 1000.0))}
    assert rows == {"double": 2 * (100 + 101 + 200 + 201), "n": 4.0}


def test_label_replace_sets_copies_and_removes():
    d = TSDB()
    d.add(Series({"__name__": "up", "instance": "10.0.0.7:9100", "job": "ne"}, fn=lambda t: 1.0))
    q = 'label_replace(up, "host", "$1", "instance", "(.*):.*")'
    (r,) = _vec(query(d, q, 100.0))
    assert r["metric"]["host"] == "10.0.0.7" and r["metric"]["__name__"] == "up"
    (r,) = _vec(query(d, 'label_replace(up, "job", "", "", "")', 100.0))
    assert "job" not in r["metric"]
    (r,) = _vec(query(d, 'label_replace(up, "host", "x", "instance", "nomatch")', 100.0))
    assert "host" not in r["metric"]  # no match: the series is unchanged
    (r,) = _vec(query(d, 'label_replace(up, "host", "${1}-${2}", "instance", "([0-9.]+):([0-9]+)")', 100.0))
    assert r["metric"]["host"] == "10.0.0.7-9100"


def test_summary_query_of_the_metrics_page():
    """metrics.js summaryQuery over an exporter-shaped TSDB: sums, counts and nodes reporting, one tagged row each."""
    import subprocess

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import ROOT, node_binary

    q = subprocess.run([node_binary(), "-e", "Promise.all([import('./src/api/promql.js'), import('./src/api/series.js')]).then(ms => Object.assign({}, ...ms)).then(m => process.stdout.write(m.summaryQuery()))"],
                       cwd=ROOT, capture_output=True, text=True, timeout=60).stdout
    d = TSDB()
    for node in ("a", "b", "c"):
        for g in range(8):
            lab = {"hostname": node, "gpu_id": str(g)}
            d.add(Series({"__name__": "gpu_power_usage", **lab}, fn=lambda t: 500.0))
            d.add(Series({"__name__": "gpu_total_vram", **lab}, fn=lambda t: 294896.0))
            if node != "c":
                d.add(Series({"__name__": "gpu_power_cap", **lab}, fn=lambda t: 1400.0))
    got = {(r["metric"]["agg"], r["metric"]["__name__"]): float(r["value"][1]) for r in _vec(query(d, q, 100.0))}
    assert got[("sum", "gpu_power_usage")] == 24 * 500.0
    assert got[("count", "gpu_power_usage")] == 24 and got[("count", "gpu_power_cap")] == 16
    assert got[("nodes", "gpu_power_usage")] == 3
    assert got[("sum", "gpu_total_vram")] == 24 * 294896.0


def test_size_guarded_small_cluster_query():
    """metrics.js smallClusterQuery: every GPU of a cluster of at most SMALL_CLUSTER_NODES GPU nodes, else the
    scope's, plus the node count row; `x and <empty>` is answered without evaluating x."""
    import subprocess

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import ROOT, node_binary

    js = ("Promise.all([import('./src/api/promql.js'), import('./src/api/series.js')]).then(ms => Object.assign({}, ...ms)).then(m => process.stdout.write(JSON.stringify("
          "[m.smallClusterQuery(true, 'topology', ['b']), m.SMALL_CLUSTER_NODES])))")
    q, limit = json.loads(subprocess.run([node_binary(), "-e", js], cwd=ROOT, capture_output=True, text=True,
                                         timeout=60).stdout)

    def cluster(nodes):
        d = TSDB()
        for node in nodes:
            for g in range(8):
                d.add(Series({"__name__": "gpu_power_usage", "hostname": node, "gpu_id": str(g)}, fn=lambda t: 500.0))
        return d

    small = _vec(query(cluster("abc"), q, 100.0))
    assert {r["metric"].get("hostname") for r in small if "agg" not in r["metric"]} == {"a", "b", "c"}
    (count,) = [r for r in small if r["metric"].get("agg") == "gpu_nodes"]
    assert float(count["value"][1]) == 3
    many = [chr(ord("a") + i) for i in range(limit + 1)]
    large = _vec(query(cluster(many), q, 100.0))
    assert {r["metric"].get("hostname") for r in large if "agg" not in r["metric"]} == {"b"}

    # The left side is not evaluated when the right is empty (a scalar there would be an error otherwise).
    d = cluster("a")
    assert _vec(query(d, "1 and on() (count(gpu_power_usage) > 1000)", 100.0)) == []
    with pytest.raises(promql.PromQLError):
        promql.Evaluator(d).instant(parse("1 and on() (count(gpu_power_usage) > 1)"), 100.0)


def test_topk_bottomk_and_the_power_ranked_page():
    """topk / bottomk (optionally by), and metrics.js rankedClusterQuery: the page's rows, the rank rows, the count."""
    import subprocess

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import ROOT, node_binary

    d = TSDB()
    watts = {"a": 100.0, "b": 300.0, "c": 200.0, "d": 50.0, "e": 250.0}
    for node, w in watts.items():
        for g in range(2):
            d.add(Series({"__name__": "gpu_power_usage", "hostname": node, "gpu_id": str(g)}, fn=lambda t, w=w: w))
            d.add(Series({"__name__": "gpu_gfx_activity", "hostname": node, "gpu_id": str(g)}, fn=lambda t: 10.0))
    top2 = _vec(query(d, "topk(2, sum by (hostname) (gpu_power_usage))", 100.0))
    assert [(r["metric"]["hostname"], float(r["value"][1])) for r in top2] == [("b", 600.0), ("e", 500.0)]
    page2 = _vec(query(d, "topk(4, sum by (hostname) (gpu_power_usage)) unless on(hostname) "
                          "topk(2, sum by (hostname) (gpu_power_usage))", 100.0))
    assert {r["metric"]["hostname"] for r in page2} == {"c", "a"}
    low = _vec(query(d, "bottomk by (hostname) (1, gpu_power_usage)", 100.0))
    assert len(low) == 5 and all(r["metric"]["__name__"] == "gpu_power_usage" for r in low)

    js = ("Promise.all([import('./src/api/promql.js'), import('./src/api/series.js')]).then(ms => Object.assign({}, ...ms)).then(m => process.stdout.write("
          "m.rankedClusterQuery('gauges', {page: 1, per: 2, filter: ''})))")
    q = subprocess.run([node_binary(), "-e", js], cwd=ROOT, capture_output=True, text=True, timeout=60).stdout
    rows = _vec(query(d, q, 100.0))
    data = {r["metric"]["hostname"] for r in rows if "agg" not in r["metric"]}
    ranks = {r["metric"]["hostname"]: float(r["value"][1]) for r in rows if r["metric"].get("agg") == "rank"}
    (count,) = [float(r["value"][1]) for r in rows if r["metric"].get("agg") == "ranked"]
    assert data == {"c", "a"} and ranks == {"c": 400.0, "a": 200.0} and count == 5


def test_the_pod_power_ranked_page():
    """metrics.js rankedOwnersQuery: the owner series of the page's pods, their rank rows, the count; name filter."""
    import subprocess

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import ROOT, node_binary

    d = TSDB()
    # pod -> (namespace, node, GPUs, watts per GPU)
    pods = {"train-a": ("ml", "n0", 4, 300.0), "train-b": ("ml", "n0", 2, 500.0), "infer-c": ("web", "n1", 1, 200.0),
            "train-d": ("ml", "n1", 2, 50.0)}
    gid = {"n0": 0, "n1": 0}
    for pod, (ns, node, n, w) in pods.items():
        for _ in range(n):
            d.add(Series({"__name__": "gpu_power_usage", "hostname": node, "gpu_id": str(gid[node]), "pod": pod,
                          "namespace": ns}, fn=lambda t, w=w: w))
            gid[node] += 1
    d.add(Series({"__name__": "gpu_power_usage", "hostname": "n1", "gpu_id": "7"}, fn=lambda t: 90.0))  # idle GPU

    def ranked(page, per, flt):
        js = ("Promise.all([import('./src/api/promql.js'), import('./src/api/series.js')]).then(ms => Object.assign({}, ...ms)).then(m => process.stdout.write(m.rankedOwnersQuery("
              "{by: 'power', page: %d, per: %d, filter: %s})))" % (page, per, json.dumps(flt)))
        q = subprocess.run([node_binary(), "-e", js], cwd=ROOT, capture_output=True, text=True, timeout=60).stdout
        rows = _vec(query(d, q, 100.0))
        owners = {(r["metric"]["namespace"], r["metric"]["pod"]) for r in rows if "agg" not in r["metric"]}
        ranks = {r["metric"]["pod"]: float(r["value"][1]) for r in rows if r["metric"].get("agg") == "rank"}
        (count,) = [float(r["value"][1]) for r in rows if r["metric"].get("agg") == "ranked"]
        return owners, ranks, count

    # totals: train-a 1200, train-b 1000, infer-c 200, train-d 100 W
    owners, ranks, count = ranked(0, 2, "")
    assert ranks == {"train-a": 1200.0, "train-b": 1000.0} and count == 4
    assert owners == {("ml", "train-a"), ("ml", "train-b")}
    owners, ranks, count = ranked(1, 2, "")
    assert ranks == {"infer-c": 200.0, "train-d": 100.0} and owners == {("web", "infer-c"), ("ml", "train-d")}
    owners, ranks, count = ranked(0, 2, "TRAIN-")
    assert ranks == {"train-a": 1200.0, "train-b": 1000.0} and count == 3
    # The table's filter also matches the namespace and the node (the page filters "namespace/name node").
    owners, ranks, count = ranked(0, 10, "web")
    assert ranks == {"infer-c": 200.0} and count == 1
    owners, ranks, count = ranked(0, 10, "n1")
    assert set(ranks) == {"infer-c", "train-d"} and count == 2
    owners, ranks, count = ranked(0, 10, "ml/train-")
    assert set(ranks) == {"train-a", "train-b", "train-d"} and count == 3


def _js(expr):
    import subprocess

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import ROOT, node_binary

    js = "Promise.all([import('./src/api/promql.js'), import('./src/api/series.js')]).then(ms => Object.assign({}, ...ms)).then(m => process.stdout.write(JSON.stringify(%s)))" % expr
    r = subprocess.run([node_binary(), "-e", js], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_summary_totals_fold_a_gpu_scraped_twice():
    """summaryQuery folds duplicate scrapes of one GPU (two jobs / instances) before summing and counting."""
    q = _js("m.summaryQuery()")
    d = TSDB()
    for job in ("servicemonitor", "annotations"):
        for g in range(8):
            lab = {"hostname": "a", "gpu_id": str(g), "job": job, "instance": job + ":5000"}
            d.add(Series({"__name__": "gpu_power_usage", **lab}, fn=lambda t: 500.0))
            d.add(Series({"__name__": "gpu_total_vram", **lab}, fn=lambda t: 294896.0))
    got = {(r["metric"]["agg"], r["metric"]["__name__"]): float(r["value"][1]) for r in _vec(query(d, q, 100.0))}
    assert got[("count", "gpu_power_usage")] == 8 and got[("sum", "gpu_power_usage")] == 8 * 500.0
    assert got[("sum", "gpu_total_vram")] == 8 * 294896.0 and got[("nodes", "gpu_power_usage")] == 1


def test_source_probe_decides_the_exporter_in_one_answer():
    """sourceProbe: exporter hostnames, node-exporter's amdgpu chips and, up to SMALL_HWMON_GPUS chips, node-exporter's
    GPU series — so one answer tells exporter / node-exporter / no GPU telemetry apart."""
    q, limit = _js("[m.sourceProbe(true), m.SMALL_HWMON_GPUS]")

    def hwmon(nodes, chips):
        d = TSDB()
        for i, node in enumerate(nodes):
            inst = "10.0.0.%d:9100" % i
            d.add(Series({"__name__": "node_uname_info", "instance": inst, "nodename": node}, fn=lambda t: 1.0))
            d.add(Series({"__name__": "node_hwmon_chip_names", "instance": inst, "chip": "platform_coretemp_0",
                          "chip_name": "coretemp"}, fn=lambda t: 1.0))
            for c in range(chips):
                chip = "0000_%02x_00_0" % (5 + c)
                d.add(Series({"__name__": "node_hwmon_chip_names", "instance": inst, "chip": chip, "chip_name": "amdgpu"},
                             fn=lambda t: 1.0))
                d.add(Series({"__name__": "node_hwmon_power_input_watt", "instance": inst, "chip": chip,
                              "sensor": "power1"}, fn=lambda t: 500.0))
        return d

    def agg(rows, tag):
        vals = [float(r["value"][1]) for r in rows if r["metric"].get("agg") == tag]
        return vals[0] if vals else 0

    small = _vec(query(hwmon(["a", "b"], 8), q, 100.0))
    assert agg(small, "hwmon") == 16 and agg(small, "gpu_nodes") == 0
    data = [r for r in small if "agg" not in r["metric"]]
    assert {r["metric"]["__name__"] for r in data} >= {"node_hwmon_chip_names", "node_hwmon_power_input_watt", "node_uname_info"}
    assert all(set(r["metric"]) <= {"__name__", "instance", "node", "nodename", "chip", "chip_name", "card"} for r in data)
    big = _vec(query(hwmon([str(i) for i in range(limit // 8 + 1)], 8), q, 100.0))
    assert agg(big, "hwmon") == limit + 8 and [r for r in big if "agg" not in r["metric"]] == []
    assert _vec(query(TSDB(), q, 100.0)) == []  # no exporter, no amdgpu hwmon: nothing at all
    # A Prometheus scraping both exporters: node-exporter's series are not sent (the exporter's win).
    both = hwmon(["a"], 8)
    for g in range(8):
        both.add(Series({"__name__": "gpu_power_usage", "hostname": "a", "gpu_id": str(g)}, fn=lambda t: 500.0))
    rows = _vec(query(both, q, 100.0))
    assert agg(rows, "gpu_nodes") == 1 and agg(rows, "hwmon") == 8 and [r for r in rows if "agg" not in r["metric"]] == []


def test_node_exporter_summary_and_scoped_query_against_the_synthetic_cluster():
    """nodeExporterSummaryQuery (server-side totals of a node-exporter-only Prometheus) against an oracle computed
    from the stored series, and nodeExporterScopedQuery returning one node's series through node_uname_info."""
    from headlamp_intel_gpu_plugin_amd.sim.apiserver import make_fake

    summary, scoped = _js("[m.nodeExporterSummaryQuery(), m.nodeExporterScopedQuery(['mi355x-001'])]")
    fc = make_fake(3, source="node-exporter", latency_ms=0)
    d, t = fc.db, 1_000_000.0
    chips = {(s.labels["instance"], s.labels["chip"]) for s in d.by_name["node_hwmon_chip_names"]
             if s.labels.get("chip_name") == "amdgpu"}

    def per(name, key):
        return {key(s.labels): s.at(t)[1] for s in d.by_name.get(name, []) if s.at(t) is not None}

    chip_key = lambda l: (l["instance"], l["chip"])
    card_key = lambda l: (l["instance"], l["card"])
    power = {**per("node_hwmon_power_input_watt", chip_key), **per("node_hwmon_power_average_watt", chip_key)}
    power = {k: v for k, v in power.items() if k in chips}
    insts = {i for i, _ in chips}
    busy = {k: v for k, v in per("node_drm_gpu_busy_percent", card_key).items() if k[0] in insts}
    got = {r["metric"]["agg"]: float(r["value"][1]) for r in _vec(query(d, summary, t))}
    assert got["hw_gpus"] == len(chips) == 24 and got["hw_nodes"] == 3
    assert got["hw_power"] == pytest.approx(sum(power.values())) and got["hw_with_power"] == len(power)
    assert got["hw_cap"] == pytest.approx(sum(v for k, v in per("node_hwmon_power_cap_watt", chip_key).items() if k in chips))
    assert got["hw_vram_used"] == pytest.approx(sum(per("node_drm_memory_vram_used_bytes", card_key).values()))
    assert got["hw_gfx_sum"] == pytest.approx(sum(busy.values())) and got["hw_gfx_n"] == len(busy)
    rows = _vec(query(d, scoped, t))
    node_inst = {s.labels["instance"] for s in d.by_name["node_uname_info"] if s.labels["nodename"] == "mi355x-001"}
    assert len(node_inst) == 1 and rows
    assert {r["metric"]["instance"] for r in rows} == node_inst
    names = {r["metric"]["__name__"] for r in rows}
    assert {"node_uname_info", "node_hwmon_chip_names", "node_hwmon_power_input_watt", "node_drm_gpu_busy_percent"} <= names


def test_node_exporter_series_in_the_exporter_shape():
    """nodeExporterScopedSeriesQuery: per-node power / HBM lines (exporter names, `hostname`, HBM in MiB) of the
    page's nodes through node_uname_info, plus the cluster lines — what seriesFetch.js reads for the exporter."""
    from headlamp_intel_gpu_plugin_amd.sim.apiserver import make_fake

    q, node_q = _js("[m.nodeExporterScopedSeriesQuery(['mi355x-001'], false), m.nodeExporterNodePowerQuery('mi355x-001')]")
    fc = make_fake(3, source="node-exporter", latency_ms=0)
    d, t = fc.db, 1_000_000.0
    body = json.loads(query_range(d, q, t - 60, t, 30.0))
    assert body["status"] == "success", body
    lines = {(r["metric"]["__name__"], r["metric"].get("hostname"), r["metric"].get("scope")): r["values"]
             for r in body["data"]["result"]}
    assert set(lines) == {("gpu_power_usage", "mi355x-001", None), ("gpu_used_vram", "mi355x-001", None),
                          ("gpu_power_usage", None, "cluster"), ("gpu_used_vram", None, "cluster")}
    inst = next(s.labels["instance"] for s in d.by_name["node_uname_info"] if s.labels["nodename"] == "mi355x-001")
    chips = {s.labels["chip"] for s in d.by_name["node_hwmon_chip_names"]
             if s.labels["instance"] == inst and s.labels.get("chip_name") == "amdgpu"}

    def power_at(instances, ts):
        tot = 0.0
        for name in ("node_hwmon_power_input_watt",):
            for s in d.by_name.get(name, []):
                if s.labels["instance"] in instances and (s.labels["instance"] != inst or s.labels["chip"] in chips):
                    tot += s.at(ts)[1]
        return tot

    ts, v = lines[("gpu_power_usage", "mi355x-001", None)][-1]
    assert float(v) == pytest.approx(power_at({inst}, float(ts)))
    all_insts = {s.labels["instance"] for s in d.by_name["node_uname_info"]}
    ts, v = lines[("gpu_power_usage", None, "cluster")][-1]
    assert float(v) == pytest.approx(power_at(all_insts, float(ts)))
    vram = sum(s.at(t)[1] for s in d.by_name["node_drm_memory_vram_used_bytes"] if s.labels["instance"] == inst) / 1048576
    assert float(lines[("gpu_used_vram", "mi355x-001", None)][-1][1]) == pytest.approx(vram)
    node_body = json.loads(query_range(d, node_q, t - 60, t, 30.0))
    (row,) = node_body["data"]["result"]
    assert row["metric"]["__name__"] == "gpu_power_usage"
    assert float(row["values"][-1][1]) == pytest.approx(power_at({inst}, float(row["values"][-1][0])))


def test_node_exporter_ranked_page_against_the_synthetic_cluster():
    """rankedHwQuery: the page of nodes by their amdgpu chips' total power (through node_uname_info), the page's
    series and uname rows, the ranking rows (hostname = nodename) and the count — against an oracle."""
    from headlamp_intel_gpu_plugin_amd.sim.apiserver import make_fake

    q = _js("m.rankedHwQuery({by: 'power', page: 1, per: 2, filter: ''})")
    fc = make_fake(5, source="node-exporter", latency_ms=0)
    d, t = fc.db, 1_000_000.0
    node_of = {s.labels["instance"]: s.labels["nodename"] for s in d.by_name["node_uname_info"]}
    per_node = {}
    for s in d.by_name["node_hwmon_power_input_watt"]:
        n = node_of[s.labels["instance"]]
        per_node[n] = per_node.get(n, 0.0) + s.at(t)[1]
    order = sorted(per_node, key=lambda n: (-per_node[n], n))
    rows = _vec(query(d, q, t))
    rank = {r["metric"]["hostname"]: float(r["value"][1]) for r in rows if r["metric"].get("agg") == "rank"}
    assert sorted(rank, key=lambda n: -rank[n]) == order[2:4]
    assert all(rank[n] == pytest.approx(per_node[n]) for n in rank)
    assert [float(r["value"][1]) for r in rows if r["metric"].get("agg") == "ranked"] == [5.0]
    page_insts = {i for i, n in node_of.items() if n in rank}
    assert {r["metric"]["instance"] for r in rows if "agg" not in r["metric"]} == page_insts


def test_node_exporter_junction_temperature_against_the_synthetic_cluster():
    """nodeExporterTempQuery on the Python fake: the amdgpu sensor labelled "junction" and its crit limit, one pair
    per GPU — not the "mem" sensor of the same chip, not the host CPU's coretemp chip; scoped through
    node_uname_info when asked (nodeExporterScopedQuery carries it)."""
    from headlamp_intel_gpu_plugin_amd.sim.apiserver import make_fake

    fc = make_fake(3, source="node-exporter", latency_ms=0)
    d, t = fc.db, 1_000_000.0
    junction = {(s.labels["instance"], s.labels["chip"]) for s in d.by_name["node_hwmon_sensor_label"]
                if s.labels["label"] == "junction"}
    assert len(junction) == 24
    rows = _vec(query(d, _js("m.nodeExporterTempQuery()"), t))
    assert sorted(r["metric"]["__name__"] for r in rows) == ["node_hwmon_temp_celsius"] * 24 + \
        ["node_hwmon_temp_crit_celsius"] * 24
    assert {(r["metric"]["instance"], r["metric"]["chip"]) for r in rows} == junction
    assert {r["metric"]["sensor"] for r in rows} == {"temp2"}
    by_key = {(s.labels["instance"], s.labels["chip"], s.labels["sensor"]): s for s in d.by_name["node_hwmon_temp_celsius"]}
    for r in rows:
        if r["metric"]["__name__"] == "node_hwmon_temp_celsius":
            k = (r["metric"]["instance"], r["metric"]["chip"], "temp2")
            assert float(r["value"][1]) == pytest.approx(by_key[k].at(t)[1])
    # The page of one node: its 8 GPUs' pairs alone, next to its power rows (`or` keeps them apart by `sensor`).
    node = "mi355x-001"
    inst = [s.labels["instance"] for s in d.by_name["node_uname_info"] if s.labels["nodename"] == node][0]
    page = _vec(query(d, _js(f"m.nodeExporterScopedQuery(['{node}'])"), t))
    temps = [r for r in page if r["metric"]["__name__"] == "node_hwmon_temp_celsius"]
    assert len(temps) == 8 and {r["metric"]["instance"] for r in temps} == {inst}
    assert len([r for r in page if r["metric"]["__name__"] == "node_hwmon_power_input_watt"]) == 8


def test_the_owners_preview_before_the_pod_list():
    """promql.js ownersQuery([], small, preview): every owner on a cluster of at most SMALL_CLUSTER_PODS owners;
    on a larger one the `preview` pods drawing the most power (their owner series and rank rows) and the count."""
    def cluster(n_pods):
        d = TSDB()
        for i in range(n_pods):
            for g in range(2):
                d.add(Series({"__name__": "gpu_power_usage", "hostname": f"n{i // 4}", "gpu_id": str(2 * (i % 4) + g),
                              "pod": f"p{i:03d}", "namespace": "ml"}, fn=lambda t, w=100.0 + i: w))
        return d

    q, limit = _js("[m.ownersQuery([], true, 5), m.SMALL_CLUSTER_PODS]")
    small = _vec(query(cluster(limit), q, 100.0))
    owners = {r["metric"]["pod"] for r in small if "agg" not in r["metric"]}
    assert len(owners) == limit and not [r for r in small if r["metric"].get("agg") == "rank"]
    big = _vec(query(cluster(limit + 36), q, 100.0))
    owners = {r["metric"]["pod"] for r in big if "agg" not in r["metric"]}
    ranks = {r["metric"]["pod"]: float(r["value"][1]) for r in big if r["metric"].get("agg") == "rank"}
    (count,) = [float(r["value"][1]) for r in big if r["metric"].get("agg") == "gpu_pods"]
    top = {f"p{i:03d}" for i in range(limit + 31, limit + 36)}
    assert owners == top and set(ranks) == top and count == limit + 36
    assert ranks[f"p{limit + 35:03d}"] == 2 * (100.0 + limit + 35)
    # Without `preview` (or with a page of pods) the large cluster answers the count alone, as before.
    q0 = _js("m.ownersQuery([], true)")
    assert [r["metric"].get("agg") for r in _vec(query(cluster(limit + 36), q0, 100.0))] == ["gpu_pods"]


def test_count_and_sum_of_the_same_selector_do_not_share_partials():
    """The fake's per-grid aggregation cache keys a count's partials (1.0 per series) apart from the values."""
    d = TSDB()
    for i in range(3):
        d.add(Series({"__name__": "gpu_power_usage", "pod": "p", "gpu_id": str(i)}, fn=lambda t, w=100.0 * (i + 1): w))
    sel = '{__name__="gpu_power_usage", pod!=""}'
    assert [r["value"][1] for r in _vec(query(d, f"count by (pod) ({sel})", 100.0))] == ["3"]
    assert [r["value"][1] for r in _vec(query(d, f"sum by (pod) ({sel})", 100.0))] == ["600"]


def test_sample_timestamps_are_written_as_prometheus_writes_them(db):
    """Prometheus's JSON: seconds, then '.' and 3 millisecond digits unless the milliseconds are 0."""
    assert '"value":[1000.5,' not in query(db, "gpu_power_usage", 1000.5)
    assert '"value":[1000.500,' in query(db, "gpu_power_usage", 1000.5)
    assert '"value":[1000,' in query(db, "gpu_power_usage", 1000.0)
    assert '"value":[1000.042,' in query(db, "gpu_power_usage", 1000.0421)
    body = json.loads(query_range(db, "gpu_power_usage", 1000.0, 1030.0, 15.0))
    assert [p[0] for p in body["data"]["result"][0]["values"]] == [1000, 1015, 1030]
