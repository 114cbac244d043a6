/**
 * A fake Prometheus behind Headlamp's service proxy, shared by the metrics
 * client specs and the provider specs: answers the liveness probe on the
 * services listed as `up`, instant `{__name__=~"a|b"}` queries (optionally
 * hostname-scoped), the pod-owner query and `query_range`, from exporter
 * rows built by `exporterData`.
 */
import { PROMETHEUS_SERVICES, SERIES, servicePath } from '../../src/api/series.js';
import { MI355X } from '../../src/api/k8sCore.js';

export const BASE0 = servicePath(PROMETHEUS_SERVICES[0]);
export const BASE1 = servicePath(PROMETHEUS_SERVICES[1]);

/** Prometheus text exposition → instant-vector rows, as /api/v1/query returns them. */
export function parseExposition(text) {
  const rows = [];
  text.split('\n').forEach((line) => {
    if (!line || line[0] === '#') return;
    const m = /^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{(.*)\})?\s+(\S+)$/.exec(line);
    if (!m) return;
    const metric = { __name__: m[1] };
    const re = /([a-zA-Z_][a-zA-Z0-9_]*)="((?:[^"\\]|\\.)*)"/g;
    let l;
    while ((l = re.exec(m[3] || '')) !== null) metric[l[1]] = l[2];
    rows.push({ metric, value: [1760000000, m[4]] });
  });
  return rows;
}

export function vec(metric, v) {
  return { metric, value: [1760000000, String(v)] };
}
export function ok(result) {
  return { status: 'success', data: { resultType: 'vector', result } };
}

/** Exporter series for `nodes` × 8 GPUs, as a name → rows map (rows carry __name__). */
export function exporterData(nodes) {
  const d = {};
  const E = SERIES.exporter;
  [E.power, E.vramUsed, E.vramTotal, E.gfx, E.umc, E.temp].forEach((k) => (d[k] = []));
  d.__xgmi = [];
  const add = (name, m, v) => d[name].push(vec(Object.assign({ __name__: name }, m), v));
  nodes.forEach((node) => {
    for (let g = 0; g < 8; g++) {
      const m = { hostname: node, gpu_id: String(g), instance: node + ':5000' };
      add(E.power, Object.assign({}, m, g < 2 ? { pod: 'train-' + g, namespace: 'ml' } : {}), 700 + g);
      add(E.vramUsed, m, 1024 * (g + 1));
      add(E.vramTotal, m, 288 * 1000 * 1000 * 1000 / (1024 * 1024));
      add(E.gfx, m, 50);
      add(E.umc, m, 30);
      add(E.temp, m, 60);
      d.__xgmi.push(vec(Object.assign({ __name__: 'xgmi_neighbor_0_tx_throughput' }, m), 50e9));
    }
  });
  return d;
}

export function flatten(d) {
  const out = [];
  if (!d) return out;
  Object.keys(d).forEach((k) => d[k].forEach((r) => out.push(r)));
  return out;
}

/**
 * One instant-query term against `rows`: the selector / projection shapes the
 * client sends (optionally `hostname="…"` or `hostname=~"a|b"` scoped), the
 * pod-owner query, and the summary aggregates (label_replace(sum|count by
 * (__name__) …, "agg", …)). Unknown shapes answer no rows.
 */
/**
 * promql.js exporterNodeQuery's server-shaped xGMI terms, evaluated the way
 * Prometheus would (tests/test_promql.py checks the real PromQL against the
 * fake Prometheus of the Python harness): throughput placed by the link
 * series' `neighbor` or a row's own peer_gpu_id, each GPU's unplaced sum, the
 * one-hop link count per GPU, the link rows of a GPU off the full mesh.
 * Null for any other term.
 */
function nodeShaped(q, rows) {
  const S = SERIES.nodeShaped;
  const host = /hostname="((?:[^"\\]|\\.)*)"/.exec(q);
  if (!host || q.indexOf('gpu_xgmi_link_hops') < 0 && q.indexOf('xgmi_neighbor_') < 0) return null;
  const h = host[1];
  const mine = rows.filter((r) => r.metric.hostname === h);
  const links = mine.filter((r) => r.metric.__name__ === 'gpu_xgmi_link_hops');
  const pin = {};
  links.forEach((r) => { if (r.metric.neighbor !== undefined) pin[r.metric.gpu_id + '>' + r.metric.neighbor] = r.metric.peer_gpu_id; });
  const tx = [];
  mine.forEach((r) => {
    const m = /^xgmi_neighbor_(\d+)_tx_throughput$/.exec(r.metric.__name__ || '');
    if (m) tx.push({ gpu: r.metric.gpu_id, k: m[1], peer: r.metric.peer_gpu_id, v: parseFloat(r.value[1]) });
  });
  if (q.indexOf('"__name__", "' + S.xgmiLink + '"') >= 0) {
    const own = q.indexOf('peer_gpu_id!=""') >= 0;
    return tx.filter((x) => (own ? !!x.peer : !x.peer && pin[x.gpu + '>' + x.k] !== undefined))
      .map((x) => vec({ __name__: S.xgmiLink, gpu_id: x.gpu, peer_gpu_id: own ? x.peer : pin[x.gpu + '>' + x.k] }, x.v));
  }
  if (q.indexOf('"__name__", "' + S.xgmiGpu + '"') >= 0) {
    const sum = {};
    tx.forEach((x) => { if (!x.peer && pin[x.gpu + '>' + x.k] === undefined) sum[x.gpu] = (sum[x.gpu] || 0) + x.v; });
    return Object.keys(sum).map((g) => vec({ __name__: S.xgmiGpu, gpu_id: g, xgmi: 'gpu' }, sum[g]));
  }
  const oneHop = {};
  links.forEach((r) => { if (parseFloat(r.value[1]) === 1) oneHop[r.metric.gpu_id] = (oneHop[r.metric.gpu_id] || 0) + 1; });
  if (q.indexOf('"__name__", "' + S.oneHopLinks + '"') >= 0) {
    return Object.keys(oneHop).map((g) => vec({ __name__: S.oneHopLinks, gpu_id: g, xgmi: '1hop' }, oneHop[g]));
  }
  if (q.indexOf('label_replace(max by (__name__, gpu_id, peer_gpu_id) (gpu_xgmi_link_hops{') === 0) {
    return links.filter((r) => oneHop[r.metric.gpu_id] !== MI355X.xgmiLinksPerGpu)
      .map((r) => vec({ __name__: 'gpu_xgmi_link_hops', gpu_id: r.metric.gpu_id, peer_gpu_id: r.metric.peer_gpu_id, xgmi: 'hops' },
        parseFloat(r.value[1])));
  }
  return null;
}

function term(q, rows) {
  // `a or b` at the top level: every term's rows; `(q)`: q.
  const alts = splitOr(q);
  if (alts.length > 1) return [].concat.apply([], alts.map((t) => term(t, rows)));
  if (q[0] === '(' && closing(q, 0) === q.length - 1) return term(q.slice(1, -1), rows);
  const shaped = nodeShaped(q, rows);
  if (shaped) return shaped;
  // `max by (…) (a or b)`: each alternative under the same projection (the fake does not project).
  const mb = /^max by \([^)]*\) \(/.exec(q);
  if (mb && closing(q, mb[0].length - 1) === q.length - 1) {
    const inner = q.slice(mb[0].length, -1);
    const parts = splitOr(inner);
    if (parts.length > 1) return [].concat.apply([], parts.map((t) => term(mb[0] + t + ')', rows)));
    // `max by (…) ((x) unless on() (count))`: the guard decides (no projection in the fake).
    if (/^\(.*\) unless on\(\) \(count\(count by .*\)\)$/.test(inner) && closing(inner, 0) === inner.indexOf(') unless on() (')) return term(inner, rows);
  }
  // promql.js nodeExporterTempQuery: amdgpu temperatures of the sensor labelled "junction" (of the instances a
  // node_uname_info selection names).
  const bare = mb && closing(q, mb[0].length - 1) === q.length - 1 ? q.slice(mb[0].length, -1) : q;
  const temp = /^\{__name__=~"(node_hwmon_temp_celsius\|node_hwmon_temp_crit_celsius)"\} and on\(instance, chip, sensor\) node_hwmon_sensor_label\{label="junction"\} and on\(instance, chip\) node_hwmon_chip_names\{chip_name="amdgpu"\}(?: and on\(instance\) \((.*)\))?$/.exec(bare);
  if (temp) {
    const key = (r) => r.metric.instance + '/' + r.metric.chip;
    const junction = {};
    const amd = {};
    rows.forEach((r) => {
      if (r.metric.__name__ === 'node_hwmon_sensor_label' && r.metric.label === 'junction') junction[key(r) + '/' + r.metric.sensor] = true;
      if (r.metric.__name__ === 'node_hwmon_chip_names' && r.metric.chip_name === 'amdgpu') amd[key(r)] = true;
    });
    let insts = null;
    if (temp[2] !== undefined) {
      insts = {};
      term('max by (instance) (' + temp[2] + ')', rows).forEach((r) => (insts[r.metric.instance] = true));
    }
    const re = new RegExp('^(?:' + temp[1] + ')$');
    return rows.filter((r) => re.test(r.metric.__name__ || '') && junction[key(r) + '/' + r.metric.sensor] &&
      amd[key(r)] && (!insts || insts[r.metric.instance]));
  }
  // `X unless on() (<count>)`: X only while the count has no sample.
  const unless = /^(.*) unless on\(\) \((count\(count by .*\))\)$/.exec(q);
  if (unless) {
    const n = countOf(unless[2], rows);
    return n ? [] : term(unless[1], rows);
  }
  // sizeGuard: `(Q) and on() (<count> <= N)` keeps Q's rows when the count passes.
  const guard = /^\((.*)\) and on\(\) \((count\(count by .*\)) (<=|>) (\d+)\)$/.exec(q);
  if (guard) {
    const n = countOf(guard[2], rows);
    if (n === null || n === 0) return [];
    const pass = guard[3] === '<=' ? n <= Number(guard[4]) : n > Number(guard[4]);
    return pass ? term(guard[1], rows) : [];
  }
  // rankedClusterQuery: the page's rows, the ranking, the ranked count.
  // (rankedOwnersQuery: the same on (namespace, pod).)
  const onRank = /^\((.*)\) and on\((hostname|namespace, pod)\) \((topk\(.*)\)$/.exec(q);
  if (onRank) {
    const ranked = rankOf(onRank[3], rows) || [];
    const keep = {};
    ranked.forEach((x) => (keep[x[0]] = true));
    const keyOf = onRank[2] === 'hostname' ? (r) => r.metric.hostname : (r) => r.metric.namespace + '/' + r.metric.pod;
    return term(onRank[1], rows).filter((r) => keep[keyOf(r)]);
  }
  const rankRow = /^label_replace\((topk\(.*\)), "agg", "rank", "", ""\)$/.exec(q);
  if (rankRow) return (rankOf(rankRow[1], rows) || []).map((x) => vec(Object.assign({ agg: 'rank' }, x[2]), x[1]));
  const rankedCount = /^label_replace\(count\((sum by \((?:hostname|namespace, pod)\) .*)\), "agg", "ranked", "", ""\)$/.exec(q);
  if (rankedCount) {
    const n = (powerSums(rankedCount[1], rows) || []).length;
    return n ? [vec({ agg: 'ranked' }, n)] : [];
  }
  // promql.js nodeExporterSummaryQuery: node-exporter totals, computed here from the rows.
  const hw = /^label_replace\((?:sum|count)\(.*\), "agg", "(hw_\w+)", "", ""\)$/.exec(q);
  if (hw) {
    const v = hwTotal(hw[1], rows);
    return v === null ? [] : [vec({ agg: hw[1] }, v)];
  }
  const sized = /^label_replace\((count\(count by .*\)), "agg", "(\w+)", "", ""\)$/.exec(q);
  if (sized) {
    const n = countOf(sized[1], rows);
    return n ? [vec({ agg: sized[2] }, n)] : [];
  }
  const own = /^max by \([^)]*\) \(\{__name__="([a-z_]+)", pod!=""\}\)$/.exec(q);
  if (own) return rows.filter((r) => r.metric.__name__ === own[1] && r.metric.pod);
  // summaryQuery: sum / count by __name__ over one series per GPU (max by __name__, hostname, gpu_id).
  const agg = /^label_replace\((sum|count) by \(__name__\) \((?:max by \(__name__, hostname, gpu_id\) \()?\{__name__=~"(.*?)"\}\)?\), "agg", "(\w+)", "", ""\)$/.exec(q);
  if (agg) {
    const re = new RegExp('^(?:' + agg[2] + ')$');
    const perGpu = {};
    rows.filter((r) => re.test(r.metric.__name__ || '')).forEach((r) => {
      const g = r.metric.__name__ + '\u0000' + r.metric.hostname + '\u0000' + r.metric.gpu_id;
      const v = parseFloat(r.value[1]);
      perGpu[g] = g in perGpu ? Math.max(perGpu[g], v) : v;
    });
    const by = {};
    Object.keys(perGpu).forEach((g) => {
      const k = g.split('\u0000')[0];
      by[k] = (by[k] || 0) + (agg[1] === 'sum' ? perGpu[g] : 1);
    });
    return Object.keys(by).map((k) => vec({ __name__: k, agg: agg[3] }, by[k]));
  }
  const nodes = /^label_replace\(count by \(__name__\) \(count by \(__name__, hostname\) \(\{__name__="([a-z_]+)"\}\)\), "agg", "nodes", "", ""\)$/.exec(q);
  if (nodes) {
    const hs = {};
    rows.filter((r) => r.metric.__name__ === nodes[1]).forEach((r) => (hs[r.metric.hostname] = true));
    const n = Object.keys(hs).length;
    return n ? [vec({ __name__: nodes[1], agg: 'nodes' }, n)] : [];
  }
  // promql.js rankedHwQuery: node-exporter's page in power order, its ranking and its count.
  const hwPage = /^max by \([^)]*\) \((?:\{__name__=~"(.*?)"\} and on\(instance\) \()?node_uname_info and on\(nodename\) \((topk\(.*)\)\)?\)$/.exec(q);
  if (hwPage) {
    const keep = {};
    (hwRankOf(hwPage[2], rows) || []).forEach((x) => (keep[x[0]] = true));
    const named = rows.filter((r) => r.metric.__name__ === 'node_uname_info' && keep[r.metric.nodename]);
    if (hwPage[1] === undefined) return named;
    const insts = {};
    named.forEach((r) => (insts[r.metric.instance] = true));
    const re = new RegExp('^(?:' + hwPage[1] + ')$');
    return rows.filter((r) => re.test(r.metric.__name__ || '') && insts[r.metric.instance] === true);
  }
  const hwRankRow = /^label_replace\(label_replace\((topk\(.*\)), "hostname", "\$1", "nodename", "\(\.\*\)"\), "agg", "rank", "", ""\)$/.exec(q);
  if (hwRankRow) return (hwRankOf(hwRankRow[1], rows) || []).map((x) => vec({ nodename: x[0], hostname: x[0], agg: 'rank' }, x[1]));
  const hwRanked = /^label_replace\(count\((sum by \(nodename\) .*)\), "agg", "ranked", "", ""\)$/.exec(q);
  if (hwRanked) {
    const n = hwNodeSums(hwRanked[1], rows).length;
    return n ? [vec({ agg: 'ranked' }, n)] : [];
  }
  // promql.js nodeExporterScopedQuery: node-exporter series of the instances node_uname_info names.
  const byNode = /^max by \([^)]*\) \((?:\{__name__=~"(.*?)"\} and on\(instance\) )?node_uname_info\{nodename(=~?)"((?:[^"\\]|\\.)*)"\}\)$/.exec(q);
  if (byNode) {
    const v = byNode[3].replace(/\\(.)/g, '$1');
    const ok = byNode[2] === '=' ? (n) => n === v : (n) => new RegExp('^(?:' + v + ')$').test(n || '');
    const named = rows.filter((r) => r.metric.__name__ === 'node_uname_info' && ok(r.metric.nodename));
    if (byNode[1] === undefined) return named;
    const insts = {};
    named.forEach((r) => (insts[r.metric.instance] = true));
    const re = new RegExp('^(?:' + byNode[1] + ')$');
    return rows.filter((r) => re.test(r.metric.__name__ || '') && insts[r.metric.instance] === true);
  }
  const m = /^(?:max by \([^)]*\) \()?\{__name__=~"(.*?)"(?:, hostname(=~?)"((?:[^"\\]|\\.)*)")?\}\)?$/.exec(q);
  if (!m) return [];
  const re = new RegExp('^(?:' + m[1] + ')$');
  let hostOk = () => true;
  if (m[3] !== undefined) {
    const v = m[3].replace(/\\(.)/g, '$1');
    if (m[2] === '=') hostOk = (h) => h === v;
    else {
      const hre = new RegExp('^(?:' + v + ')$');
      hostOk = (h) => hre.test(h || '');
    }
  }
  return rows.filter((r) => re.test(r.metric.__name__ || '') && hostOk(r.metric.hostname));
}

/**
 * metrics.js nodePowerSum / podPowerSum over `rows`: [[key, watts, labels], …]
 * (key = hostname, or "namespace/pod"; null for another shape).
 */
function powerSums(expr, rows) {
  const unesc = (v) => new RegExp('^(?:' + v.replace(/\\\\/g, '\\') + ')$');
  const m = /^sum by \(hostname\) \(\{__name__="([a-z_]+)"(?:, hostname=~"(.*)")?\}\)$/.exec(expr);
  // promql.js podFilterMatchers: pod, namespace or node substring (`or` of three selectors), or "ns/name".
  const alt = m ? null : /^sum by \(namespace, pod\) \(\{__name__="([a-z_]+)", pod!="", pod=~"(.*?)"\} or \{__name__="[a-z_]+", pod!="", namespace=~"(.*?)"\} or \{__name__="[a-z_]+", pod!="", hostname=~"(.*?)"\}\)$/.exec(expr);
  const p = m || alt ? null : /^sum by \(namespace, pod\) \(\{__name__="([a-z_]+)", pod!=""(?:, pod=~"([^"]*)")?\}\)$/.exec(expr);
  const nsName = m || p || alt ? null : /^sum by \(namespace, pod\) \(\{__name__="([a-z_]+)", pod!="", namespace=~"(.*?)", pod=~"(.*?)"\}\)$/.exec(expr);
  if (alt || nsName) {
    const un = (v) => new RegExp('^(?:' + v.replace(/\\\\/g, '\\') + ')$');
    const keep = alt
      ? (r) => un(alt[2]).test(r.metric.pod || '') || un(alt[3]).test(r.metric.namespace || '') || un(alt[4]).test(r.metric.hostname || '')
      : (r) => un(nsName[2]).test(r.metric.namespace || '') && un(nsName[3]).test(r.metric.pod || '');
    const name = (alt || nsName)[1];
    const by = {};
    const labels = {};
    rows.forEach((r) => {
      if (r.metric.__name__ !== name || !r.metric.pod || !keep(r)) return;
      const k = r.metric.namespace + '/' + r.metric.pod;
      by[k] = (by[k] || 0) + parseFloat(r.value[1]);
      labels[k] = { namespace: r.metric.namespace, pod: r.metric.pod };
    });
    return Object.keys(by).map((k) => [k, by[k], labels[k]]);
  }
  const x = m || p;
  if (!x) return null;
  const re = x[2] !== undefined ? unesc(x[2]) : null;
  const by = {};
  const labels = {};
  rows.forEach((r) => {
    if (r.metric.__name__ !== x[1]) return;
    if (p && !r.metric.pod) return;
    const k = m ? r.metric.hostname : r.metric.namespace + '/' + r.metric.pod;
    if (re && !re.test((m ? r.metric.hostname : r.metric.pod) || '')) return;
    by[k] = (by[k] || 0) + parseFloat(r.value[1]);
    labels[k] = m ? { hostname: r.metric.hostname } : { namespace: r.metric.namespace, pod: r.metric.pod };
  });
  return Object.keys(by).map((k) => [k, by[k], labels[k]]);
}

/** metrics.js powerRankQuery: the ranked page, [[hostname, watts], …] (null for another shape). */
function rankOf(expr, rows) {
  const m = /^topk\((\d+), (.*?)\)(?: unless on\((?:hostname|namespace, pod)\) topk\((\d+), (.*)\))?$/.exec(expr);
  if (!m) return null;
  const all = powerSums(m[2], rows);
  if (!all) return null;
  all.sort((a, b) => b[1] - a[1] || (a[0] < b[0] ? -1 : 1));
  return all.slice(m[3] ? Number(m[3]) : 0, Number(m[1]));
}

/** metrics.js gpuNodeCount / gpuPodCount over `rows` (null for another shape). */
function countOf(expr, rows) {
  // promql.js hwmonGpuCount: node-exporter's amdgpu chips.
  if (/^count\(count by \(instance, chip\) \(\{__name__="node_hwmon_chip_names", chip_name="amdgpu"\}\)\)$/.test(expr)) {
    const chips = {};
    rows.forEach((r) => {
      if (r.metric.__name__ === 'node_hwmon_chip_names' && r.metric.chip_name === 'amdgpu') chips[r.metric.instance + '/' + r.metric.chip] = true;
    });
    return Object.keys(chips).length;
  }
  const m = /^count\(count by \((hostname|namespace, pod)\) \(\{__name__="([a-z_]+)"(, pod!="")?\}\)\)$/.exec(expr);
  if (!m) return null;
  const seen = {};
  rows.forEach((r) => {
    if (r.metric.__name__ !== m[2] || (m[3] && !r.metric.pod)) return;
    seen[m[1] === 'hostname' ? r.metric.hostname : r.metric.namespace + '/' + r.metric.pod] = true;
  });
  return Object.keys(seen).length;
}

/**
 * promql.js hwNodePowerSum over `rows`: [[nodename, watts]] — each node's
 * amdgpu chips (power average, else input) through node_uname_info, names
 * matching its `nodename=~` filter.
 */
function hwNodeSums(expr, rows) {
  const f = /node_uname_info\{nodename=~"((?:[^"\\]|\\.)*)"\}/.exec(expr);
  const re = f ? new RegExp('^(?:' + f[1].replace(/\\\\/g, '\\') + ')$') : null;
  const nodeOf = {};
  rows.forEach((r) => {
    if (r.metric.__name__ === 'node_uname_info' && (!re || re.test(r.metric.nodename || ''))) nodeOf[r.metric.instance] = r.metric.nodename;
  });
  const chips = {};
  rows.forEach((r) => {
    if (r.metric.__name__ === 'node_hwmon_chip_names' && r.metric.chip_name === 'amdgpu') chips[r.metric.instance + '/' + r.metric.chip] = true;
  });
  const power = {};
  ['node_hwmon_power_input_watt', 'node_hwmon_power_average_watt'].forEach((name) => rows.forEach((r) => {
    const k = r.metric.instance + '/' + r.metric.chip;
    if (r.metric.__name__ === name && chips[k]) power[k] = parseFloat(r.value[1]);
  }));
  const by = {};
  Object.keys(power).forEach((k) => {
    const node = nodeOf[k.split('/')[0]];
    if (node !== undefined) by[node] = (by[node] || 0) + power[k];
  });
  return Object.keys(by).map((n) => [n, by[n]]);
}

/** promql.js hwPowerRankQuery: the ranked page, [[nodename, watts], …] (null for another shape). */
function hwRankOf(expr, rows) {
  if (expr.indexOf('topk(') !== 0) return null;
  const close = closing(expr, 4);
  const inner = expr.slice(5, close);
  const comma = inner.indexOf(', ');
  const n = Number(inner.slice(0, comma));
  const rest = /^ unless on\(nodename\) topk\((\d+), /.exec(expr.slice(close + 1));
  const all = hwNodeSums(inner.slice(comma + 2), rows);
  all.sort((a, b) => b[1] - a[1] || (a[0] < b[0] ? -1 : 1));
  return all.slice(rest ? Number(rest[1]) : 0, n);
}

/** Index of the parenthesis closing the one at `open`. */
function closing(q, open) {
  let depth = 0;
  for (let i = open; i < q.length; i++) {
    if (q[i] === '(') depth++;
    else if (q[i] === ')' && --depth === 0) return i;
  }
  return -1;
}

/**
 * One nodeExporterSummaryQuery figure over `rows` (null: an empty vector):
 * amdgpu chips, their instances, power (average, else input) summed and
 * counted, caps, DRM HBM / busy of the cards of those instances.
 */
function hwTotal(tag, rows) {
  const chips = {};
  const insts = {};
  rows.forEach((r) => {
    if (r.metric.__name__ !== 'node_hwmon_chip_names' || r.metric.chip_name !== 'amdgpu') return;
    chips[r.metric.instance + '/' + r.metric.chip] = true;
    insts[r.metric.instance] = true;
  });
  const per = (name, keyOf, keep) => {
    const out = {};
    rows.forEach((r) => {
      if (r.metric.__name__ !== name || !keep(r)) return;
      const k = keyOf(r);
      const v = parseFloat(r.value[1]);
      out[k] = k in out ? Math.max(out[k], v) : v;
    });
    return out;
  };
  const chipKey = (r) => r.metric.instance + '/' + r.metric.chip;
  const cardKey = (r) => r.metric.instance + '/' + r.metric.card;
  const onChip = (r) => chips[chipKey(r)] === true;
  const onInst = (r) => insts[r.metric.instance] === true;
  const power = Object.assign(per('node_hwmon_power_input_watt', chipKey, onChip), per('node_hwmon_power_average_watt', chipKey, onChip));
  const vals = (o) => Object.keys(o).map((k) => o[k]);
  const sum = (a) => (a.length ? a.reduce((x, y) => x + y, 0) : null);
  const count = (a) => (a.length ? a.length : null);
  switch (tag) {
    case 'hw_gpus': return count(Object.keys(chips));
    case 'hw_nodes': return count(Object.keys(insts));
    case 'hw_power': return sum(vals(power));
    case 'hw_with_power': return count(vals(power));
    case 'hw_cap': return sum(vals(per('node_hwmon_power_cap_watt', chipKey, onChip)));
    case 'hw_vram_used': return sum(vals(per('node_drm_memory_vram_used_bytes', cardKey, onInst)));
    case 'hw_vram_total': return sum(vals(per('node_drm_memory_vram_size_bytes', cardKey, onInst)));
    case 'hw_gfx_sum': return sum(vals(per('node_drm_gpu_busy_percent', cardKey, onInst)));
    case 'hw_gfx_n': return count(vals(per('node_drm_gpu_busy_percent', cardKey, onInst)));
    default: return null;
  }
}

/** `q` split at its top-level ` or ` (not inside parentheses). */
export function splitOr(q) {
  const out = [];
  let depth = 0;
  let start = 0;
  for (let i = 0; i < q.length; i++) {
    const c = q[i];
    if (c === '(') depth++;
    else if (c === ')') depth--;
    else if (depth === 0 && q.substr(i, 4) === ' or ') {
      out.push(q.slice(start, i));
      start = i + 4;
      i += 3;
    }
  }
  out.push(q.slice(start));
  return out;
}

/** A fake proxy: answers probes on `up` services and the client's queries from `data` / `ne`. */
export function prom(opts) {
  const o = Object.assign({ up: [BASE0], data: exporterData(['n0']), ne: null }, opts || {});
  const rows = flatten(o.data).concat(flatten(o.ne));
  return vi.fn((path) => {
    const base = o.up.find((b) => path.indexOf(b) === 0);
    if (!base) return Promise.reject(new Error('503'));
    const q = decodeURIComponent((path.split('query=')[1] || '').split('&')[0]);
    if (q === '1') return Promise.resolve(ok([{ metric: {}, value: [0, '1'] }]));
    if (path.indexOf('/query_range') >= 0) {
      const end = Number(/end=(\d+)/.exec(path)[1]);
      const values = [[end - 30, '100'], [end, '200']];
      const result = [
        { metric: { __name__: 'gpu_power_usage', hostname: 'n0' }, values },
        { metric: { __name__: 'gpu_used_vram', hostname: 'n0' }, values },
      ];
      // the scoped series query also asks for the cluster-wide line
      if (q.indexOf('"scope", "cluster"') >= 0) {
        result.push({ metric: { __name__: 'gpu_power_usage', scope: 'cluster' }, values });
        result.push({ metric: { __name__: 'gpu_used_vram', scope: 'cluster' }, values });
      }
      return Promise.resolve({ status: 'success', data: { resultType: 'matrix', result } });
    }
    // `a or b`: every term's rows (the client keeps their label sets apart).
    const out = [];
    splitOr(q).forEach((t) => term(t, rows).forEach((r) => out.push(r)));
    return Promise.resolve(ok(out));
  });
}
