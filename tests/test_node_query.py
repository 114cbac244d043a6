"""The one-node telemetry query (src/api/promql.js exporterNodeQuery) on the fake Prometheus's real PromQL: what
Prometheus places and sums there equals what the client places from the raw rows (telemetry.js + topology.js)."""
import json

import pytest

from headlamp_intel_gpu_plugin_amd.sim.promql import TSDB, Series, query


def _vec(body):
    if isinstance(body, str):
        body = json.loads(body)
    assert body["status"] == "success", body
    return body["data"]["result"]


def _stock_db(with_links=None):
    """The stock Device Metrics Exporter scrape (tests/fixtures/stock_exporter/node_8x_mi355x.prom) as constant
    series; `with_links`: {(gpu, peer): neighbor} link series as this repo's --sysfs-only exporter writes them."""
    import os

    from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition

    d = TSDB()
    text = open(os.path.join(os.path.dirname(__file__), "fixtures", "stock_exporter", "node_8x_mi355x.prom")).read()
    host = None
    for name, labels, v in parse_exposition(text):
        host = labels.get("hostname", host)
        d.add(Series(dict(labels, __name__=name), fn=lambda t, v=v: v))
    for (a, b), k in (with_links or {}).items():
        d.add(Series({"__name__": "gpu_xgmi_link_hops", "hostname": host, "gpu_id": str(a), "peer_gpu_id": str(b),
                      "neighbor": str(k)}, fn=lambda t: 1.0))
    return d, host


def _jsfn(expr, *args):
    import subprocess

    from headlamp_intel_gpu_plugin_amd.utils.nodebridge import ROOT, node_binary

    js = ("Promise.all([import('./src/api/promql.js'), import('./src/api/telemetry.js'), import('./src/api/topology.js')])"
          ".then(ms => Object.assign({}, ...ms)).then(m => { const a = JSON.parse(process.argv[1]); "
          "process.stdout.write(JSON.stringify((" + expr + ")(m, ...a))); })")
    r = subprocess.run([node_binary(), "-e", js, json.dumps(list(args))], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("pinned", [False, True])
def test_one_node_query_places_xgmi_like_the_client(pinned):
    """exporterNodeQuery has Prometheus place xGMI throughput (a link series' `neighbor` pins neighbour k to a peer)
    and sum what it cannot place per GPU. On the stock exporter's own scrape — with and without this repo's link
    series — the joined one-node answer places exactly what the client places from the raw rows
    (telemetry.js join + topology.js placeThroughput), and the full mesh arrives as per-GPU link counts."""
    links = None
    if pinned:
        # GPU g's neighbours in rotated order (g+1, g+2, ...): not index order
        links = {(g, (g + 1 + k) % 8): k for g in range(8) for k in range(7)}
    db, host = _stock_db(links)
    t = 1000.0
    node_q = _jsfn("(m, h) => m.exporterNodeQuery(h, true)", host)
    node_rows = _vec(query(db, node_q, t))
    names = {r["metric"]["__name__"] for r in node_rows}
    assert ("amdgpu:xgmi_link_tx" in names) == pinned and ("amdgpu:xgmi_gpu_tx" in names) == (not pinned)
    assert not any("hostname" in r["metric"] or "instance" in r["metric"] for r in node_rows)
    raw_q = _jsfn("(m, h) => m.exporterNodeQuery(h, true)", host).split(" or ")[0]  # the gauges alone
    wide_q = _jsfn("(m) => m.exporterQuery(true, false, 'all')")
    wide_rows = _vec(query(db, wide_q, t))
    server = _jsfn("(m, rows, h) => { const j = m.joinExporterResults(m.splitByName(rows), h); const n = j.xgmi[h] || {};"
                 " return { placed: m.placeThroughput(n, j.links[h] || null).map, links: j.links[h] || {}, gpus: j.gpus.length }; }",
                 node_rows, host)
    client = _jsfn("(m, rows, h) => { const j = m.joinExporterResults(m.splitByName(rows)); "
                 " return { placed: m.placeThroughput(j.xgmi[h], j.links[h] || null).map, links: j.links[h] || {} }; }",
                 wide_rows, host)
    assert server["gpus"] == 8
    assert server["placed"].keys() == client["placed"].keys()
    for k, v in client["placed"].items():
        assert server["placed"][k] == pytest.approx(v, rel=1e-9), k
    per_gpu = [k for k in client["placed"] if k.split("-")[0] == k.split("-")[1]]
    assert len(per_gpu) == 8
    assert (len(client["placed"]) == 8 + 56) == pinned
    # the topology: 56 one-hop links either way when pinned (counts expanded vs rows), none without link series
    strip = lambda l: {k: {"type": v["type"], "hops": v["hops"]} for k, v in l.items()}
    assert strip(server["links"]) == strip(client["links"])
    assert len(server["links"]) == (56 if pinned else 0)
    assert raw_q.startswith("max by (__name__, gpu_id, pod, namespace)")


def test_one_node_query_sends_link_rows_only_for_a_gpu_off_the_full_mesh():
    links = {(g, (g + 1 + k) % 8): k for g in range(8) for k in range(7)}
    del links[(3, 4)]  # GPU 3 misses a link
    db, host = _stock_db(links)
    rows = _vec(query(db, _jsfn("(m, h) => m.exporterNodeQuery(h, true)", host), 1000.0))
    hop_rows = [r for r in rows if r["metric"]["__name__"] == "gpu_xgmi_link_hops"]
    assert {r["metric"]["gpu_id"] for r in hop_rows} == {"3"} and len(hop_rows) == 6
    counts = {r["metric"]["gpu_id"]: r["value"][1] for r in rows if r["metric"]["__name__"] == "amdgpu:xgmi_1hop_links"}
    assert counts == {str(g): ("6" if g == 3 else "7") for g in range(8)}
    joined = _jsfn("(m, rows, h) => m.joinExporterResults(m.splitByName(rows), h).links[h]", rows, host)
    assert len(joined) == 55 and "3-4" not in joined and "4-3" in joined
