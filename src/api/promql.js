/**
 * PromQL the telemetry client sends: pure string builders, no I/O.
 *
 * Reference analog: the four instant queries of src/api/metrics.ts:101-116
 * (i915 chip names, energy rate, power max, uname), sent on every fetch.
 * Here each page asks ONE query shaped for what it draws (ADR 006, 008, 009):
 * a `__name__=~` selector projected onto the labels the join reads, scoped to
 * the page's nodes (`hostname=~`) or pods, with server-side aggregates for
 * cluster totals and size guards Prometheus evaluates in the same request.
 */

import { MI355X } from './k8sCore.js';
import {
  EXPORTER_JOIN_LABELS,
  EXPORTER_LEAN_LABELS,
  NODE_EXPORTER_JOIN_LABELS,
  SERIES,
  SMALL_CLUSTER_NODES,
  SMALL_CLUSTER_PODS,
  SMALL_HWMON_GPUS,
} from './series.js';

/**
 * Per-GPU exporter gauges. The static ones (HBM capacity, power cap, throttle
 * threshold, link topology) change only with a reconfiguration of the node,
 * so callers ask for them once per DISCOVERY_TTL_MS and keep a copy; every
 * refresh asks for the live ones (those of `view`, METRIC_VIEWS).
 */
export function exporterNames(withStatic, view) {
  const E = SERIES.exporter;
  const gauges = [E.power, E.vramUsed, E.gfx, E.umc, E.temp, E.eccCorrect, E.eccUncorrect];
  const names = view === 'gauges' ? gauges : view === 'topology' ? [E.power, E.temp, E.xgmiRe] : gauges.concat([E.xgmiRe]);
  if (withStatic !== false) names.push(E.powerCap, E.vramTotal, E.tempSlowdown, E.linkHops);
  return names;
}

export function isExporterName(name) {
  const E = SERIES.exporter;
  for (const k in E) if (E[k] === name) return true;
  return false;
}

/**
 * ONE instant query per source: a `__name__=~` selector returns every series
 * the page needs in a single response (split client-side by `__name__`).
 * A browser allows 6 concurrent HTTP/1.1 connections per origin, so a
 * refresh that stays within 6 requests completes in one round-trip.
 * @param {boolean} [withStatic]  include the static series (default true)
 * @param {boolean} [lean]        project onto EXPORTER_LEAN_LABELS (live-only queries of a hostname-keyed exporter)
 * @param {string} [view]         METRIC_VIEWS entry (default 'all')
 * @param {string[]} [scope]      node names (`hostname=~`)
 */
export function exporterQuery(withStatic, lean, view, scope) {
  const names = exporterNames(withStatic, view);
  if (scope) {
    // Every row matches the hostname matcher: the live-only query needs no fallback keys.
    const scopedLabels = withStatic === false ? EXPORTER_LEAN_LABELS : EXPORTER_JOIN_LABELS;
    return 'max by (' + scopedLabels.join(', ') + ') ({__name__=~"' + names.join('|') + '", ' + hostnameMatcher(scope) + '})';
  }
  const labels = lean && withStatic === false ? EXPORTER_LEAN_LABELS : EXPORTER_JOIN_LABELS;
  return 'max by (' + labels.join(', ') + ') ({__name__=~"' + names.join('|') + '"})';
}

/** A regex matching exactly `s` (RE2 metacharacters escaped). */
export function regexLiteral(s) {
  return String(s).replace(/[\\.+*?()|[\]{}^$]/g, '\\$&');
}

/** A PromQL double-quoted string literal body. */
export function promString(s) {
  return String(s).replace(/\\/g, '\\\\').replace(/"/g, '\\"');
}

/**
 * `hostname=~"a|b|…"` for the nodes a paged view shows — the label the joins
 * key GPUs by (Kubernetes node name). An empty scope matches nothing.
 */
export function hostnameMatcher(names) {
  // "." is no valid node name: an empty scope matches nothing (callers skip it anyway).
  if (!names.length) return 'hostname="."';
  return 'hostname=~"' + promString(names.map(regexLiteral).join('|')) + '"';
}

/** Exporter hostnames reporting a power gauge: the GPU nodes Prometheus sees. */
export function gpuNodeCount() {
  return 'count(count by (hostname) ({__name__="' + SERIES.exporter.power + '"}))';
}

/** Pods the exporter attributes a GPU to. */
export function gpuPodCount() {
  return 'count(count by (namespace, pod) ({__name__="' + SERIES.exporter.power + '", pod!=""}))';
}

/** amdgpu hwmon chips node-exporter reports: its GPUs (any cluster size, one sample). */
export function hwmonGpuCount() {
  return 'count(count by (instance, chip) ({__name__="node_hwmon_chip_names", chip_name="amdgpu"}))';
}

/**
 * `q` when `count` (a one-sample count, gpuNodeCount / gpuPodCount) is at
 * most `limit` (`small`), or above it (`!small`): `and on()` keeps all of `q`
 * or none of it, decided by Prometheus in the same evaluation.
 */
export function sizeGuard(q, small, count, limit) {
  return '(' + q + ') and on() (' + count + ' ' + (small ? '<=' : '>') + ' ' + limit + ')';
}

/** The count itself as a row tagged `agg="<tag>"` (telemetry.js sizeFromRows reads it back). */
export function sizeRow(count, tag) {
  return 'label_replace(' + count + ', "agg", "' + tag + '", "", "")';
}

/**
 * A paged view's telemetry while its page may be the whole cluster (the node
 * list is loading, or every GPU node fits on one page): every GPU when the
 * cluster is small, else the nodes of `scope` — one request either way, and
 * none waits for the node list on a small cluster.
 */
export function smallClusterQuery(withStatic, view, scope) {
  const n = gpuNodeCount();
  const all = sizeGuard(exporterQuery(withStatic, false, view), true, n, SMALL_CLUSTER_NODES);
  const page = scope.length ? ' or ' + sizeGuard(exporterQuery(withStatic, true, view, scope), false, n, SMALL_CLUSTER_NODES) : '';
  // The count itself: which branch answered, and a large cluster (nothing
  // asked for yet) told apart from one without exporter series.
  return all + page + ' or ' + sizeRow(n, 'gpu_nodes');
}

/**
 * What the first query of a session appends while it is not known which
 * exporter feeds this Prometheus, so that ONE answer decides it:
 *   * `agg="gpu_nodes"`: exporter hostnames (also when the page's own query
 *     is hostname-scoped and matched nothing);
 *   * `agg="hwmon"`: node-exporter's amdgpu chips;
 *   * node-exporter's GPU series themselves while there are at most
 *     SMALL_HWMON_GPUS chips (a size guard, as smallClusterQuery) and no
 *     exporter reports.
 * A cluster without GPU telemetry (no exporter, no amdgpu hwmon) is then told
 * apart in the first wave; the reference probed and queried serially
 * (src/api/metrics.ts:77-116), and round 3 paid a second, cluster-wide
 * query for it.
 */
export function sourceProbe(withGpuNodes) {
  const hw = hwmonGpuCount();
  // node-exporter's series only where no exporter reports (`unless on()`):
  // a cluster running both sends the exporter's alone.
  return (withGpuNodes ? sizeRow(gpuNodeCount(), 'gpu_nodes') + ' or ' : '') +
    sizeRow(hw, 'hwmon') + ' or ' + sizeGuard(nodeExporterProjected(), true, hw, SMALL_HWMON_GPUS) +
    ' unless on() (' + gpuNodeCount() + ')';
}

/** Node names are lowercase (RFC 1123): a name filter becomes a lowercase substring regex. */
function hostnameFilter(filter) {
  const f = String(filter || '').trim().toLowerCase();
  return f ? ', hostname=~".*' + promString(regexLiteral(f)) + '.*"' : '';
}

/** Each GPU node's total GPU power (the ranking key), names matching `filter`. */
export function nodePowerSum(filter) {
  return 'sum by (hostname) ({__name__="' + SERIES.exporter.power + '"' + hostnameFilter(filter) + '})';
}

/**
 * The GPU nodes of page `page` (0-based, `per` a page) ranked by total GPU
 * power, highest first: `topk` of the pages so far minus `topk` of the pages
 * before — Prometheus ranks, so the answer is one page whatever the cluster.
 */
export function powerRankQuery(page, per, filter) {
  const r = nodePowerSum(filter);
  const top = function (n) { return 'topk(' + n + ', ' + r + ')'; };
  return page > 0 ? top(per * (page + 1)) + ' unless on(hostname) ' + top(per * page) : top(per);
}

/**
 * A page of GPU nodes in power order, in ONE request: the view's series of
 * the nodes the ranking picks (`and on(hostname)`), the ranking itself as
 * `agg="rank"` rows (their order) and how many nodes are ranked
 * (`agg="ranked"`, the pager's count).
 */
export function rankedClusterQuery(view, rank, withStatic) {
  const s = powerRankQuery(rank.page, rank.per, rank.filter);
  const st = withStatic !== false;
  return '(' + exporterQuery(st, !st, view) + ') and on(hostname) (' + s + ')' +
    ' or ' + sizeRow(s, 'rank') +
    ' or ' + sizeRow('count(' + nodePowerSum(rank.filter) + ')', 'ranked');
}

/** Exporter series the cluster totals of the Metrics page summary sum or count. */
function summaryNames() {
  const E = SERIES.exporter;
  return {
    sum: [E.power, E.powerCap, E.vramUsed, E.vramTotal, E.gfx, E.eccCorrect, E.eccUncorrect],
    count: [E.power, E.powerCap, E.vramUsed, E.gfx, E.temp, E.tempSlowdown, E.eccUncorrect],
  };
}

/** One series per GPU of `names`: duplicate scrapes of a GPU (two jobs, two instances) fold into one. */
function perGpu(names) {
  return 'max by (__name__, hostname, gpu_id) ({__name__=~"' + names.join('|') + '"})';
}

/**
 * Cluster totals for the Metrics page summary as server-side aggregates: a
 * handful of rows whatever the cluster size, instead of every gauge of every
 * GPU. Each aggregation is tagged with an `agg` label (sum / count / nodes)
 * so the rows survive `or` next to each other and next to a per-GPU query.
 * Series are first folded to one per (hostname, gpu_id), as the per-GPU join
 * keys them, so an exporter scraped twice (a ServiceMonitor plus annotation
 * scraping: different `job` / `instance`) is not counted twice.
 */
export function summaryQuery() {
  const s = summaryNames();
  const E = SERIES.exporter;
  return 'label_replace(sum by (__name__) (' + perGpu(s.sum) + '), "agg", "sum", "", "")' +
    ' or label_replace(count by (__name__) (' + perGpu(s.count) + '), "agg", "count", "", "")' +
    ' or label_replace(count by (__name__) (count by (__name__, hostname) ({__name__="' + E.power + '"})), "agg", "nodes", "", "")';
}

/** Labels of the one-node query's per-GPU rows: `hostname` is its matcher (the client puts it back), `instance` unread. */
export const NODE_GAUGE_LABELS = ['__name__', 'gpu_id', 'pod', 'namespace'];

/**
 * The exporter query scoped to ONE node (`hostname` label = Kubernetes node
 * name, the same key the joins and views use): what the native Node / Pod
 * detail pages ask for, O(GPUs per node) series whatever the cluster size,
 * shaped so each row carries only what the page reads (ADR 006):
 *   * per-GPU gauges projected onto NODE_GAUGE_LABELS;
 *   * xGMI throughput placed on its peer by Prometheus — the stock
 *     exporter's xgmi_neighbor_<k>_tx_throughput joined on the link series'
 *     `neighbor` (this repo's amdgpu-exporter), or a row's own peer_gpu_id —
 *     and, per GPU, the sum of what no series places (the client's
 *     topology.js placeThroughput rules, evaluated where the rows are);
 *   * with `withStatic`, the link topology as a count of one-hop links per
 *     GPU, plus the link rows of any GPU that does not have the full MI355X
 *     mesh of MI355X.xgmiLinksPerGpu (telemetry.js expands the count).
 */
export function exporterNodeQuery(nodeName, withStatic) {
  const E = SERIES.exporter;
  const S = SERIES.nodeShaped;
  const host = 'hostname="' + promString(nodeName) + '"';
  const names = exporterNames(withStatic, 'gauges').filter(function (n) { return n !== E.linkHops; });
  const hops = E.linkHops + '{' + host + '}';
  const xgmi = '{__name__=~"' + E.xgmiRe + '", ' + host;
  const byNeighbor = 'label_replace(' + xgmi + ', peer_gpu_id=""}, "neighbor", "$1", "__name__", "xgmi_neighbor_([0-9]+)_tx_throughput")';
  // one link row per (gpu_id, neighbor): a bad duplicate cannot turn the join many-to-many
  const pins = 'topk by (gpu_id, neighbor) (1, max by (gpu_id, neighbor, peer_gpu_id) (' + hops + '))';
  // `or` keeps a right-hand row only when no left-hand row has its labels
  // other than __name__: a GPU's total and link count would collide with its
  // gauges ({gpu_id}), a non-mesh link row with its placed throughput
  // ({gpu_id, peer_gpu_id}) — an `xgmi` label tells them apart.
  function named(expr, name, tag) {
    const e = 'label_replace(' + expr + ', "__name__", "' + name + '", "", "")';
    return tag ? 'label_replace(' + e + ', "xgmi", "' + tag + '", "", "")' : e;
  }
  const parts = [
    'max by (' + NODE_GAUGE_LABELS.join(', ') + ') ({__name__=~"' + names.join('|') + '", ' + host + '})',
    named('max by (gpu_id, peer_gpu_id) (' + byNeighbor + ' * on (gpu_id, neighbor) group_left (peer_gpu_id) (0 * ' + pins + ' + 1))',
      S.xgmiLink),
    named('max by (gpu_id, peer_gpu_id) (' + xgmi + ', peer_gpu_id!=""})', S.xgmiLink),
    named('sum by (gpu_id) (max by (gpu_id, neighbor) (' + byNeighbor + ' unless on (gpu_id, neighbor) ' + pins + '))', S.xgmiGpu, 'gpu'),
  ];
  if (withStatic !== false) {
    const oneHop = 'count by (gpu_id) (max by (gpu_id, peer_gpu_id) (' + hops + ') == 1)';
    parts.push(named(oneHop, S.oneHopLinks, '1hop'));
    parts.push('label_replace(max by (__name__, gpu_id, peer_gpu_id) (' + hops + '), "xgmi", "hops", "", "") unless on (gpu_id) (' + oneHop +
      ' == ' + MI355X.xgmiLinksPerGpu + ')');
  }
  return parts.join(' or ');
}

/**
 * Pod → GPU attribution only (the Pods page): the power gauge of GPUs whose
 * `pod` label is set — one series per allocated GPU, instead of every live
 * gauge and xGMI link of every GPU.
 */
export function ownersQuery(pods, small, preview) {
  const sel = '{__name__="' + SERIES.exporter.power + '", ';
  if (small) {
    // Every owner when they fit on one page of the Pods table, else the page's pods (smallClusterQuery).
    const n = gpuPodCount();
    const all = sizeGuard(ownersQuery(null), true, n, SMALL_CLUSTER_PODS);
    const page = pods && pods.length ? ' or ' + sizeGuard(ownersQuery(pods), false, n, SMALL_CLUSTER_PODS) : '';
    // No page yet (the pod list is on its way) on a larger cluster: the
    // `preview` pods drawing the most power, ranked, so the page has rows to
    // show before the list is in (pods.js podsPreview).
    const pre = preview > 0 && !(pods && pods.length) ? ' or ' + sizeGuard(previewOwners(preview), false, n, SMALL_CLUSTER_PODS) : '';
    return all + page + pre + ' or ' + sizeRow(n, 'gpu_pods');
  }
  if (!pods) return 'max by (' + EXPORTER_JOIN_LABELS.join(', ') + ') (' + sel + 'pod!=""})';
  // The pods of one page of the Pods table ("namespace/name" keys): O(page).
  const names = {};
  const nss = {};
  for (let i = 0; i < pods.length; i++) {
    const k = String(pods[i]);
    const slash = k.indexOf('/');
    nss[k.slice(0, slash)] = true;
    names[k.slice(slash + 1)] = true;
  }
  const alt = function (o) { return promString(Object.keys(o).map(regexLiteral).join('|')); };
  return 'max by (' + EXPORTER_JOIN_LABELS.join(', ') + ') (' + sel + 'pod=~"' + alt(names) + '", namespace=~"' + alt(nss) + '"})';
}

/**
 * The owner series of the `per` pods drawing the most GPU power and their
 * ranking as `agg="rank"` rows: page 0 of rankedOwnersQuery without its
 * count (the size row of the small query counts the owners).
 */
function previewOwners(per) {
  const s = podPowerRankQuery(0, per, '');
  return '(' + ownersQuery(null) + ') and on(namespace, pod) (' + s + ') or ' + sizeRow(s, 'rank');
}

/**
 * The GPU Pods filter as exporter label matchers: the table matches a
 * case-insensitive substring of "namespace/name node" (pages.js podPage), so
 * in power order a filter matches the pod name, the namespace or the node
 * (`hostname`); "ns/name" matches a namespace ending in "ns" and a pod name
 * starting with "name". Returns alternative matcher lists (any may match).
 */
export function podFilterMatchers(filter) {
  const f = typeof filter === 'string' ? filter.trim().toLowerCase() : '';
  if (!f) return [''];
  const sub = function (s) { return '.*' + promString(regexLiteral(s)) + '.*'; };
  const slash = f.indexOf('/');
  if (slash >= 0 && f.indexOf(' ') < 0) {
    const ns = f.slice(0, slash);
    const name = f.slice(slash + 1);
    return [', namespace=~".*' + promString(regexLiteral(ns)) + '", pod=~"' + promString(regexLiteral(name)) + '.*"'];
  }
  return [', pod=~"' + sub(f) + '"', ', namespace=~"' + sub(f) + '"', ', hostname=~"' + sub(f) + '"'];
}

/** Total GPU power per pod from the exporter's pod labels; `filter` as podFilterMatchers. */
export function podPowerSum(filter) {
  const sel = function (m) { return '{__name__="' + SERIES.exporter.power + '", pod!=""' + m + '}'; };
  return 'sum by (namespace, pod) (' + podFilterMatchers(filter).map(sel).join(' or ') + ')';
}

/**
 * The GPU pods of page `page` (0-based, `per` a page) ranked by the power
 * of the GPUs they hold, highest first — as powerRankQuery for nodes:
 * Prometheus ranks, the answer is one page whatever the cluster.
 */
export function podPowerRankQuery(page, per, filter) {
  const r = podPowerSum(filter);
  const top = function (n) { return 'topk(' + n + ', ' + r + ')'; };
  return page > 0 ? top(per * (page + 1)) + ' unless on(namespace, pod) ' + top(per * page) : top(per);
}

/**
 * A page of GPU pods in power order, in ONE request: the owner series of the
 * pods the ranking picks, the ranking as `agg="rank"` rows and how many pods
 * draw GPU power (`agg="ranked"`, the pager's count).
 */
export function rankedOwnersQuery(rank) {
  const s = podPowerRankQuery(rank.page, rank.per, rank.filter);
  return '(' + ownersQuery(null) + ') and on(namespace, pod) (' + s + ')' +
    ' or ' + sizeRow(s, 'rank') +
    ' or ' + sizeRow('count(' + podPowerSum(rank.filter) + ')', 'ranked');
}

function nodeExporterNames() {
  const N = SERIES.nodeExporter;
  return [N.chips.split('{')[0], N.power, N.powerInput, N.powerCap, N.busy, N.vramUsed, N.vramTotal, N.uname];
}

/**
 * amdgpu junction temperature and its crit (throttle) limit through
 * node-exporter: the hwmon temperatures whose sensor node_hwmon_sensor_label
 * names "junction", on amdgpu chips only — two series per GPU, not every
 * sensor of every chip of the node. `uname` (a node_uname_info selector):
 * only the instances it names. The rows keep `sensor`, so `or`-ed next to
 * the power rows of the same chip (which `or` would match, ignoring the
 * name) they stay apart.
 */
export function nodeExporterTempQuery(uname) {
  const N = SERIES.nodeExporter;
  return '{__name__=~"' + N.temp + '|' + N.tempCrit + '"} and on(instance, chip, sensor) ' + N.sensorLabel +
    '{label="junction"} and on(instance, chip) ' + N.chips + (uname ? ' and on(instance) (' + uname + ')' : '');
}

export function nodeExporterQuery() {
  return '{__name__=~"' + nodeExporterNames().join('|') + '"} or ' + nodeExporterTempQuery();
}

/** nodeExporterQuery projected onto the labels its join reads. */
export function nodeExporterProjected() {
  return 'max by (' + NODE_EXPORTER_JOIN_LABELS.join(', ') + ') (' + nodeExporterQuery() + ')';
}

/**
 * `nodename=~"a|b|…"` on node_uname_info: node-exporter's GPU series carry
 * `instance`, not the Kubernetes node name; node_uname_info names the node
 * (telemetry.js joinNodeExporterResults maps instance → nodename). An empty
 * scope matches nothing.
 */
function nodenameMatcher(names) {
  if (!names.length) return 'nodename="."';
  return 'nodename=~"' + promString(names.map(regexLiteral).join('|')) + '"';
}

/**
 * node-exporter's series of the nodes a paged view shows, in ONE request:
 * the GPU series of the instances whose node_uname_info names one of them
 * (`and on(instance)`), plus those node_uname_info rows for the join —
 * O(page) on a cluster that feeds Prometheus through node-exporter only
 * (the reference's one source: src/api/metrics.ts:101-116, every chip of
 * the cluster on every fetch).
 */
export function nodeExporterScopedQuery(names) {
  const N = SERIES.nodeExporter;
  const labels = NODE_EXPORTER_JOIN_LABELS.join(', ');
  const gpuNames = nodeExporterNames().filter(function (n) { return n !== N.uname; });
  const uname = N.uname + '{' + nodenameMatcher(names) + '}';
  return 'max by (' + labels + ') ({__name__=~"' + gpuNames.join('|') + '"} and on(instance) ' + uname +
    ' or ' + nodeExporterTempQuery(uname) + ')' +
    ' or max by (' + labels + ') (' + uname + ')';
}

/** Each amdgpu chip's power: the average where node-exporter reports one, else the instantaneous input. */
function hwChipPower() {
  const N = SERIES.nodeExporter;
  return '(max by (instance, chip) (' + N.power + ') or max by (instance, chip) (' + N.powerInput + '))' +
    ' and on(instance, chip) count by (instance, chip) (' + N.chips + ')';
}

/** `q` renamed to `name` and tagged `series="<tag>"` (keeps `or`-ed lines apart: `or` ignores the name). */
function asSeries(q, name, tag) {
  return 'label_replace(label_replace(' + q + ', "__name__", "' + name + '", "", ""), "series", "' + tag + '", "", "")';
}

/**
 * Power + HBM-used history of a node-exporter source in the exporter's
 * shape (series.js names, per `hostname`, HBM in the exporter's MiB), so
 * seriesFetch.js reads it unchanged: `nodes` — per node through
 * node_uname_info, the nodes of `scope` or every node (`scope` null) — and
 * `cluster` — the cluster-wide lines (`scope="cluster"`).
 */
function hwSeriesParts(scope) {
  const N = SERIES.nodeExporter;
  const E = SERIES.exporter;
  const uname = 'max by (instance, nodename) (' + N.uname + (scope ? '{' + nodenameMatcher(scope) + '}' : '') + ')';
  const perNode = function (q) {
    return 'label_replace(sum by (nodename) ((' + q + ') * on(instance) group_left(nodename) ' + uname + '), "hostname", "$1", "nodename", "(.*)")';
  };
  const vram = 'max by (instance, card) (' + N.vramUsed + ') / ' + SERIES.exporterVramUnitBytes;
  const cluster = function (q) { return 'label_replace(' + q + ', "scope", "cluster", "", "")'; };
  return {
    nodes: asSeries(perNode(hwChipPower()), E.power, 'power') + ' or ' + asSeries(perNode(vram), E.vramUsed, 'vram'),
    cluster: cluster(asSeries('sum(' + hwChipPower() + ')', E.power, 'power')) + ' or ' +
      cluster(asSeries('sum(' + vram + ' and on(instance) count by (instance) (' + N.chips + '))', E.vramUsed, 'vram')),
  };
}

/** Every node's power + HBM lines of a node-exporter source (seriesQuery's counterpart). */
export function nodeExporterSeriesQuery() {
  return hwSeriesParts(null).nodes;
}

/**
 * A paged view's lines of a node-exporter source, as scopedSeriesQuery: the
 * page's nodes and the cluster line; `small` keeps every node's line while
 * at most SMALL_HWMON_GPUS amdgpu chips report (the page may be asked before
 * the node list names it), else the page's.
 */
export function nodeExporterScopedSeriesQuery(scope, small) {
  const page = hwSeriesParts(scope).nodes;
  const total = hwSeriesParts(null).cluster;
  if (!small) return page + ' or ' + total;
  const hw = hwmonGpuCount();
  const all = sizeGuard(nodeExporterSeriesQuery(), true, hw, SMALL_HWMON_GPUS);
  return (scope.length ? all + ' or ' + sizeGuard(page, false, hw, SMALL_HWMON_GPUS) : all) + ' or ' + total;
}

/** Each node's total GPU power on a node-exporter source (the ranking key), per `nodename`; names matching `filter`. */
export function hwNodePowerSum(filter) {
  const N = SERIES.nodeExporter;
  const f = String(filter || '').trim().toLowerCase();
  const sel = f ? '{nodename=~".*' + promString(regexLiteral(f)) + '.*"}' : '';
  return 'sum by (nodename) ((' + hwChipPower() + ') * on(instance) group_left(nodename) max by (instance, nodename) (' +
    N.uname + sel + '))';
}

/** powerRankQuery on a node-exporter source: the page of nodes by total GPU power, ranked by Prometheus. */
export function hwPowerRankQuery(page, per, filter) {
  const r = hwNodePowerSum(filter);
  const top = function (n) { return 'topk(' + n + ', ' + r + ')'; };
  return page > 0 ? top(per * (page + 1)) + ' unless on(nodename) ' + top(per * page) : top(per);
}

/**
 * rankedClusterQuery on a node-exporter source, in ONE request: the GPU
 * series of the instances whose node_uname_info names a ranked node, those
 * node_uname_info rows, the ranking as `agg="rank"` rows (with `hostname` =
 * nodename, as the exporter's) and how many nodes are ranked.
 */
export function rankedHwQuery(rank) {
  const N = SERIES.nodeExporter;
  const s = hwPowerRankQuery(rank.page, rank.per, rank.filter);
  const labels = NODE_EXPORTER_JOIN_LABELS.join(', ');
  const gpuNames = nodeExporterNames().filter(function (n) { return n !== N.uname; });
  const uname = N.uname + ' and on(nodename) (' + s + ')';
  return 'max by (' + labels + ') ({__name__=~"' + gpuNames.join('|') + '"} and on(instance) (' + uname + ')' +
    ' or ' + nodeExporterTempQuery(uname) + ')' +
    ' or max by (' + labels + ') (' + uname + ')' +
    ' or ' + sizeRow('label_replace(' + s + ', "hostname", "$1", "nodename", "(.*)")', 'rank') +
    ' or ' + sizeRow('count(' + hwNodePowerSum(rank.filter) + ')', 'ranked');
}

/** One node's total GPU power over time on a node-exporter source (Node detail history). */
export function nodeExporterNodePowerQuery(nodeName) {
  const uname = SERIES.nodeExporter.uname + '{nodename="' + promString(nodeName) + '"}';
  return 'label_replace(sum(' + hwChipPower() + ' and on(instance) ' + uname + '), "__name__", "' + SERIES.exporter.power + '", "", "")';
}

/**
 * Cluster totals of a node-exporter source as server-side aggregates, the
 * figures summarizeMetrics takes from the per-GPU join (telemetry.js
 * hwTotalsFromRows reads them back): amdgpu chips (GPUs) and the nodes
 * reporting them; power per chip — the average where reported, else the
 * instantaneous input (`or` keeps the first) — summed and counted; power
 * caps; HBM used / total and GFX busy of the DRM cards of those nodes.
 * A few rows whatever the cluster size.
 */
export function nodeExporterSummaryQuery() {
  const N = SERIES.nodeExporter;
  const chips = 'count by (instance, chip) (' + N.chips + ')';
  const insts = 'count by (instance) (' + N.chips + ')';
  const power = '(max by (instance, chip) (' + N.power + ') or max by (instance, chip) (' + N.powerInput + '))' +
    ' and on(instance, chip) ' + chips;
  const cap = 'max by (instance, chip) (' + N.powerCap + ') and on(instance, chip) ' + chips;
  const card = function (n) { return 'max by (instance, card) (' + n + ') and on(instance) ' + insts; };
  return [
    sizeRow('count(' + chips + ')', 'hw_gpus'),
    sizeRow('count(' + insts + ')', 'hw_nodes'),
    sizeRow('sum(' + power + ')', 'hw_power'),
    sizeRow('count(' + power + ')', 'hw_with_power'),
    sizeRow('sum(' + cap + ')', 'hw_cap'),
    sizeRow('sum(' + card(N.vramUsed) + ')', 'hw_vram_used'),
    sizeRow('sum(' + card(N.vramTotal) + ')', 'hw_vram_total'),
    sizeRow('sum(' + card(N.busy) + ')', 'hw_gfx_sum'),
    sizeRow('count(' + card(N.busy) + ')', 'hw_gfx_n'),
  ].join(' or ');
}

/**
 * First query of a session, while it is not yet known which exporter feeds
 * this Prometheus: both exporters' series in ONE request, projected onto the
 * union of the labels the two joins read. Later refreshes ask only the
 * exporter that answered.
 */
export function mergedQuery(withStatic, view) {
  const names = exporterNames(withStatic, view).concat(nodeExporterNames());
  const labels = EXPORTER_JOIN_LABELS.slice();
  for (let i = 0; i < NODE_EXPORTER_JOIN_LABELS.length; i++) {
    if (labels.indexOf(NODE_EXPORTER_JOIN_LABELS[i]) < 0) labels.push(NODE_EXPORTER_JOIN_LABELS[i]);
  }
  // node-exporter's temperatures only where no exporter reports (its join would be read for nothing).
  return 'max by (' + labels.join(', ') + ') ({__name__=~"' + names.join('|') + '"} or (' + nodeExporterTempQuery() +
    ') unless on() (' + gpuNodeCount() + '))';
}

/**
 * One pod's total GPU power over time (Pod detail history): the power gauge
 * of the GPUs the exporter attributes to the pod (`pod` / `namespace`
 * labels), summed per step. O(points), whatever the cluster size.
 */
export function podPowerQuery(namespace, pod) {
  return 'sum by (__name__) ({__name__="' + SERIES.exporter.power + '", namespace="' + promString(namespace) +
    '", pod="' + promString(pod) + '"})';
}

/** One node's total GPU power over time (Node detail history), summed per step. */
export function nodePowerQuery(nodeName) {
  return 'sum by (__name__) ({__name__="' + SERIES.exporter.power + '", hostname="' + promString(nodeName) + '"})';
}

/** Per-node power + HBM-used history in one range query (split by `__name__`). */
export function seriesQuery() {
  const E = SERIES.exporter;
  return 'sum by (__name__, hostname) ({__name__=~"' + E.power + '|' + E.vramUsed + '"})';
}

/**
 * Power + HBM-used history of the nodes a paged view shows (`hostname=~`)
 * plus the cluster-wide total (tagged `scope="cluster"`): O(visible nodes ×
 * points) whatever the cluster size.
 */
export function scopedSeriesQuery(scope, small) {
  const E = SERIES.exporter;
  const names = '__name__=~"' + E.power + '|' + E.vramUsed + '"';
  const page = 'sum by (__name__, hostname) ({' + names + ', ' + hostnameMatcher(scope) + '})';
  const total = 'label_replace(sum by (__name__) ({' + names + '}), "scope", "cluster", "", "")';
  if (small) {
    // Every node's line on a cluster of one page, else the page's (smallClusterQuery).
    const n = gpuNodeCount();
    const all = sizeGuard(seriesQuery(), true, n, SMALL_CLUSTER_NODES);
    return (scope.length ? all + ' or ' + sizeGuard(page, false, n, SMALL_CLUSTER_NODES) : all) + ' or ' + total;
  }
  return page + ' or ' + total;
}
