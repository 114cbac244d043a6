/**
 * MI355X telemetry from Prometheus, reached through the Kubernetes service proxy.
 *
 * Reference analog: src/api/metrics.ts (SURVEY.md C4), which finds
 * Prometheus by probing three services serially with no timeout (:77-90),
 * then runs four instant queries on i915 hwmon series and joins power by
 * PCI `chip` only (:127-138, quirk Q1).
 *
 * This client (ADR 002, 003, 006):
 *   * sends the first query straight to the preferred service (its answer
 *     is the discovery); only if that fails are all candidates probed IN
 *     PARALLEL with a timeout (reference: serial, no timeout,
 *     src/api/metrics.ts:77-90). The winner is cached for 5 min;
 *   * reads AMD series — the AMD Device Metrics Exporter (`gpu_*`, per-GPU,
 *     optionally pod-labelled), this repo's amdgpu-exporter extensions
 *     (power cap, link hops, throttle thresholds) and, as a fallback,
 *     node-exporter's amdgpu hwmon + DRM collectors — with ONE merged first
 *     query, then only the exporter that answered, projected onto the labels
 *     the join reads (reference: four queries per fetch, :101-116);
 *   * keys every GPU by (node, gpu index), never by PCI address alone
 *     (reference quirk Q1, :127-138);
 *   * exposes power, HBM used/total, GFX and memory-controller activity,
 *     temperature vs throttle threshold, xGMI per-link throughput and measured
 *     link topology, and incremental `query_range` series (power / HBM per
 *     node; the reference has instant queries only, :67-75);
 *   * shares structure between snapshots and serves the last snapshot marked
 *     `stale` through transient failures.
 *
 * Metric and label names are all in `SERIES`; the device-level ones are
 * pinned by captures from a real MI355X (tests/fixtures/mi355x).
 */

import { MI355X, isObject } from './amdgpu.js';
import { withTimeout, DEFAULT_REQUEST_TIMEOUT_MS } from './clusterStore.js';

/** Candidate Prometheus services, highest priority first (reference metrics.ts:61-65). */
export const PROMETHEUS_SERVICES = [
  { namespace: 'monitoring', service: 'kube-prometheus-stack-prometheus', port: '9090' },
  { namespace: 'monitoring', service: 'prometheus-operated', port: '9090' },
  { namespace: 'monitoring', service: 'prometheus', port: '9090' },
];

export function servicePath(svc) {
  return '/api/v1/namespaces/' + svc.namespace + '/services/' + svc.service + ':' + svc.port + '/proxy';
}

/**
 * Series names. Exporter names follow the AMD Device Metrics Exporter field
 * list (lower-cased); node-exporter names follow its hwmon/drm collectors.
 * (verify both against the deployed versions)
 */
export const SERIES = {
  exporter: {
    power: 'gpu_power_usage', // W
    powerCap: 'gpu_power_cap', // W (board power cap; 1400 on MI355X)
    vramUsed: 'gpu_used_vram', // MiB
    vramTotal: 'gpu_total_vram', // MiB: an MI355X reads 294896 = 288 GiB (tests/fixtures/mi355x)
    gfx: 'gpu_gfx_activity', // %
    umc: 'gpu_umc_activity', // % — HBM controller busy
    temp: 'gpu_junction_temperature', // °C
    tempSlowdown: 'gpu_junction_temperature_slowdown', // °C throttle threshold (this repo's amdgpu-exporter)
    eccCorrect: 'gpu_ecc_correct_total', // corrected RAS errors, all IP blocks
    eccUncorrect: 'gpu_ecc_uncorrect_total', // uncorrected RAS errors, all IP blocks
    xgmiRe: 'xgmi_neighbor_[0-6]_tx_throughput', // bytes/s per neighbour
    linkHops: 'gpu_xgmi_link_hops', // measured link topology (this repo's native amdgpu-exporter)
  },
  exporterVramUnitBytes: 1024 * 1024,
  nodeExporter: {
    chips: 'node_hwmon_chip_names{chip_name="amdgpu"}',
    power: 'node_hwmon_power_average_watt',
    // hwmon power1_input. An MI355X exposes power1_input and no power1_average
    // (tests/fixtures/mi355x/sysfs_amdgpu_files.txt), so this is its only power
    // series through node-exporter; the average wins where both exist.
    powerInput: 'node_hwmon_power_input_watt',
    powerCap: 'node_hwmon_power_cap_watt',
    busy: 'node_drm_gpu_busy_percent',
    vramUsed: 'node_drm_memory_vram_used_bytes',
    vramTotal: 'node_drm_memory_vram_size_bytes',
    uname: 'node_uname_info',
  },
};

/** Discovery cache lifetime. Prometheus services move rarely. */
export const DISCOVERY_TTL_MS = 5 * 60 * 1000;
/** Consecutive failed metrics fetches before the page switches to "Prometheus Unreachable". */
export const STALE_FAILURES = 3;
/**
 * GPU nodes (exporter hostnames) up to which a paged view asks for the whole
 * cluster instead of its page: one page of nodes (pages.js NODES_PER_PAGE).
 * Prometheus evaluates the guard inside the same request
 * (smallClusterQuery), so a page opened while the node list is still loading
 * needs no second wave on a small cluster, and a large one gets nothing it
 * did not ask for.
 */
export const SMALL_CLUSTER_NODES = 8;
/**
 * GPU pods (exporter `pod` labels) up to which the Pods page asks for every
 * owner: as many as a cluster of one page of nodes can run (8 × 8 GPUs, one
 * each). Their owner series are at most a few KB; the table still shows one
 * page of PODS_PER_PAGE, and paging through it needs no request.
 */
export const SMALL_CLUSTER_PODS = 64;

/**
 * @typedef {Object} GpuTelemetry
 * @property {string} nodeName
 * @property {string} gpu            device index on the node ("0".."7")
 * @property {string} instance
 * @property {number|null} powerWatts
 * @property {number|null} powerCapWatts
 * @property {number|null} vramUsedBytes
 * @property {number|null} vramTotalBytes
 * @property {number|null} gfxActivityPct
 * @property {number|null} memActivityPct
 * @property {number|null} tempC
 * @property {number|null} tempSlowdownC  junction throttle threshold (exporter), if reported
 * @property {number|null} eccCorrectable    corrected RAS errors since driver load (exporter only)
 * @property {number|null} eccUncorrectable  uncorrected RAS errors since driver load (exporter only)
 * @property {string|null} pod
 * @property {string|null} namespace
 *
 * @typedef {Object} GpuMetrics
 * @property {'amd-exporter'|'node-exporter'|null} source
 * @property {GpuTelemetry[]} gpus
 * @property {Record<string, Record<string, number>>} xgmi  node → "src-dst" → GB/s
 * @property {Record<string, Record<string, {type: string, hops: number}>>} links  node → "src-dst" →
 *           measured link (gpu_xgmi_link_hops); empty when the exporter does not report topology
 * @property {string} fetchedAt
 * @property {boolean} [stale]  the latest fetch failed; this is the previous snapshot
 * @property {string} prometheusPath
 */

function num(v) {
  const f = parseFloat(v);
  return isFinite(f) ? f : null;
}

/** A label value, or '' when it is missing or not a string. */
function labelStr(v) {
  return typeof v === 'string' ? v : '';
}

/** A well-formed instant-vector row: `{metric: {...}, value: [ts, "v"]}`. */
function isRow(row) {
  return !!row && isObject(row.metric) && Array.isArray(row.value);
}

function emptyGpu(nodeName, gpu, instance) {
  return {
    nodeName: nodeName, gpu: gpu, instance: instance,
    powerWatts: null, powerCapWatts: null, vramUsedBytes: null, vramTotalBytes: null,
    gfxActivityPct: null, memActivityPct: null, tempC: null, tempSlowdownC: null,
    eccCorrectable: null, eccUncorrectable: null, pod: null, namespace: null,
    // The cap is the MI355X board limit because the source reported none.
    powerCapAssumed: false,
  };
}

/** Sort GPUs by node then numeric device index. */
function byNodeGpu(a, b) {
  if (a.nodeName !== b.nodeName) return a.nodeName < b.nodeName ? -1 : 1;
  return parseInt(a.gpu, 10) - parseInt(b.gpu, 10);
}

/**
 * Join AMD Device Metrics Exporter instant vectors into per-GPU telemetry.
 * Keyed by (hostname, gpu_id). Exported for direct unit tests.
 */
export function joinExporterResults(r) {
  const E = SERIES.exporter;
  const map = {};
  function slot(m) {
    // Label values are strings; anything else in a malformed answer is ignored.
    const node = labelStr(m.hostname) || labelStr(m.node) || labelStr(m.instance);
    const gpu = m.gpu_id !== undefined ? String(m.gpu_id) : '0';
    const k = node + '\u0000' + gpu;
    if (!map[k]) map[k] = emptyGpu(node, gpu, m.instance || '');
    return map[k];
  }
  function each(list, fn) {
    if (!Array.isArray(list)) return;
    for (let i = 0; i < list.length; i++) {
      const row = list[i];
      if (!isRow(row)) continue;
      fn(slot(row.metric), num(row.value[1]), row.metric);
    }
  }
  each(r[E.power], function (g, v, m) {
    g.powerWatts = v;
    if (m.pod) {
      g.pod = m.pod;
      g.namespace = m.namespace || null;
    }
  });
  each(r[E.powerCap], function (g, v) { if (v !== null && v > 0) g.powerCapWatts = v; });
  each(r[E.vramUsed], function (g, v) { g.vramUsedBytes = v === null ? null : v * SERIES.exporterVramUnitBytes; });
  each(r[E.vramTotal], function (g, v) { g.vramTotalBytes = v === null ? null : v * SERIES.exporterVramUnitBytes; });
  each(r[E.gfx], function (g, v) { g.gfxActivityPct = v; });
  each(r[E.umc], function (g, v) { g.memActivityPct = v; });
  each(r[E.temp], function (g, v) { g.tempC = v; });
  each(r[E.tempSlowdown], function (g, v) { g.tempSlowdownC = v; });
  each(r[E.eccCorrect], function (g, v) { g.eccCorrectable = v; });
  each(r[E.eccUncorrect], function (g, v) { g.eccUncorrectable = v; });
  const gpus = [];
  for (const k in map) {
    const g = map[k];
    if (g.powerCapWatts === null) {
      // The stock Device Metrics Exporter has no cap series: every GPU is an
      // MI355X, so bars use its board limit, flagged as assumed.
      g.powerCapWatts = MI355X.tdpWatts;
      g.powerCapAssumed = true;
    }
    gpus.push(g);
  }
  gpus.sort(byNodeGpu);

  // xGMI: neighbour k of GPU i is the k-th peer in index order, skipping i (verify).
  const xgmi = {};
  const xr = r.__xgmi;
  if (Array.isArray(xr)) {
    for (let i = 0; i < xr.length; i++) {
      if (!isRow(xr[i])) continue;
      const m = xr[i].metric;
      const name = typeof m.__name__ === 'string' ? m.__name__ : '';
      const mm = /^xgmi_neighbor_(\d)_tx_throughput$/.exec(name);
      if (!mm) continue;
      const src = parseInt(m.gpu_id, 10);
      if (!isFinite(src)) continue;
      const k = parseInt(mm[1], 10);
      const dst = k < src ? k : k + 1;
      const node = labelStr(m.hostname) || labelStr(m.instance);
      if (!xgmi[node]) xgmi[node] = {};
      const v = num(xr[i].value[1]);
      if (v !== null) xgmi[node][src + '-' + dst] = v / 1e9;
    }
  }
  // Measured topology: gpu_xgmi_link_hops{gpu_id, peer_gpu_id} per xGMI-connected pair.
  const links = {};
  const lr = r[E.linkHops];
  if (Array.isArray(lr)) {
    for (let i = 0; i < lr.length; i++) {
      if (!isRow(lr[i])) continue;
      const m = lr[i].metric;
      const node = labelStr(m.hostname) || labelStr(m.instance);
      const v = num(lr[i].value[1]);
      if (v === null || m.gpu_id === undefined || m.peer_gpu_id === undefined) continue;
      if (!links[node]) links[node] = {};
      links[node][m.gpu_id + '-' + m.peer_gpu_id] = { type: 'XGMI', hops: v };
    }
  }
  return { gpus: gpus, xgmi: xgmi, links: links };
}

/**
 * Join node-exporter hwmon (power, keyed by PCI chip) and DRM (busy %, VRAM,
 * keyed by card) series. Within one instance the k-th amdgpu chip in PCI
 * order is card k — DRM cards enumerate in PCI order on amdgpu (verify).
 */
export function joinNodeExporterResults(r) {
  const N = SERIES.nodeExporter;
  const instToNode = {};
  const un = Array.isArray(r[N.uname]) ? r[N.uname] : [];
  for (let i = 0; i < un.length; i++) {
    if (!isRow(un[i])) continue;
    const m = un[i].metric;
    if (m.instance) instToNode[m.instance] = m.nodename || m.node || m.instance;
  }
  const chipsByInst = {};
  const chips = Array.isArray(r[N.chips]) ? r[N.chips] : [];
  for (let i = 0; i < chips.length; i++) {
    if (!isRow(chips[i])) continue;
    const m = chips[i].metric;
    if (!m.instance || !m.chip) continue;
    if (!chipsByInst[m.instance]) chipsByInst[m.instance] = [];
    if (chipsByInst[m.instance].indexOf(m.chip) < 0) chipsByInst[m.instance].push(m.chip);
  }
  const map = {};
  const gpus = [];
  for (const inst in chipsByInst) {
    const list = chipsByInst[inst].sort();
    for (let k = 0; k < list.length; k++) {
      const g = emptyGpu(instToNode[inst] || inst, String(k), inst);
      map[inst + '\u0000chip:' + list[k]] = g;
      map[inst + '\u0000card:card' + k] = g;
      gpus.push(g);
    }
  }
  function each(list, keyFn, fn) {
    if (!Array.isArray(list)) return;
    for (let i = 0; i < list.length; i++) {
      if (!isRow(list[i])) continue;
      const m = list[i].metric;
      const g = map[(m.instance || '') + '\u0000' + keyFn(m)];
      if (g) fn(g, num(list[i].value[1]));
    }
  }
  function chipKey(m) { return 'chip:' + (m.chip || ''); }
  function cardKey(m) { return 'card:' + (m.card || ''); }
  each(r[N.powerInput], chipKey, function (g, v) { g.powerWatts = v; });
  each(r[N.power], chipKey, function (g, v) { if (v !== null) g.powerWatts = v; });
  each(r[N.powerCap], chipKey, function (g, v) { g.powerCapWatts = v; });
  each(r[N.busy], cardKey, function (g, v) { g.gfxActivityPct = v; });
  each(r[N.vramUsed], cardKey, function (g, v) { g.vramUsedBytes = v; });
  each(r[N.vramTotal], cardKey, function (g, v) { g.vramTotalBytes = v; });
  gpus.sort(byNodeGpu);
  return { gpus: gpus, xgmi: {}, links: {} };
}

/**
 * ONE instant query per source: a `__name__=~` selector returns every series
 * the page needs in a single response (split client-side by `__name__`).
 * A browser allows 6 concurrent HTTP/1.1 connections per origin, so a
 * refresh that stays within 6 requests completes in one round-trip.
 */
/**
 * Labels the exporter join reads. The combined query projects every series
 * onto them (`max by (...)`), so the response carries no per-series
 * card/driver/serial/job labels: the Device Metrics Exporter attaches a
 * dozen of those to every gauge, which would otherwise dominate the bytes
 * moved through the Headlamp proxy on each refresh. `max` also folds
 * duplicate scrapes of one GPU (two jobs scraping one exporter).
 */
export const EXPORTER_JOIN_LABELS = ['__name__', 'hostname', 'node', 'instance', 'gpu_id', 'peer_gpu_id', 'pod', 'namespace'];

/**
 * The projection of the per-refresh (live-only) query once the static query
 * has shown that every exporter series carries `hostname` (the Device Metrics
 * Exporter labels all its gauges with it): `node` / `instance` are then only
 * fallback keys, and `instance` ("10.0.0.17:5000") is ~18 % of the response
 * bytes. The GPU's `instance` is kept from the static query (STATIC_GPU_FIELDS).
 */
export const EXPORTER_LEAN_LABELS = ['__name__', 'hostname', 'gpu_id', 'peer_gpu_id', 'pod', 'namespace'];

/**
 * What a cluster-wide fetch is for — each page asks only for the live series
 * it draws (the same idea as the Pods page's ownersQuery):
 *   all       every live gauge and every xGMI link (terminal client, detail fallback);
 *   gauges    the Metrics page: per-GPU power / HBM / activity / temperature /
 *             RAS, no xGMI links (7 of the 14 live series of a GPU);
 *   topology  the GPU Nodes page: per-GPU pod owners (from the power gauge)
 *             and the per-link xGMI throughput of the neighbour matrix.
 */
export const METRIC_VIEWS = ['all', 'gauges', 'topology'];

/**
 * Per-GPU exporter gauges. The static ones (HBM capacity, power cap, throttle
 * threshold, link topology) change only with a reconfiguration of the node,
 * so callers ask for them once per DISCOVERY_TTL_MS and keep a copy; every
 * refresh asks for the live ones (those of `view`, METRIC_VIEWS).
 */
function exporterNames(withStatic, view) {
  const E = SERIES.exporter;
  const gauges = [E.power, E.vramUsed, E.gfx, E.umc, E.temp, E.eccCorrect, E.eccUncorrect];
  const names = view === 'gauges' ? gauges : view === 'topology' ? [E.power, E.xgmiRe] : gauges.concat([E.xgmiRe]);
  if (withStatic !== false) names.push(E.powerCap, E.vramTotal, E.tempSlowdown, E.linkHops);
  return names;
}

function isExporterName(name) {
  const E = SERIES.exporter;
  for (const k in E) if (E[k] === name) return true;
  return false;
}

/** Fields of GpuTelemetry that come from the static series (see exporterNames). */
export const STATIC_GPU_FIELDS = ['powerCapWatts', 'powerCapAssumed', 'vramTotalBytes', 'tempSlowdownC', 'instance'];

/**
 * @param {boolean} [withStatic]  include the static series (default true)
 * @param {boolean} [lean]        project onto EXPORTER_LEAN_LABELS (live-only queries of a hostname-keyed exporter)
 * @param {string} [view]         METRIC_VIEWS entry (default 'all')
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

/**
 * `q` when `count` (a one-sample count, gpuNodeCount / gpuPodCount) is at
 * most `limit` (`small`), or above it (`!small`): `and on()` keeps all of `q`
 * or none of it, decided by Prometheus in the same evaluation.
 */
export function sizeGuard(q, small, count, limit) {
  return '(' + q + ') and on() (' + count + ' ' + (small ? '<=' : '>') + ' ' + limit + ')';
}

/** The count itself as a row tagged `agg="<tag>"` (sizeFromRows reads it back). */
function sizeRow(count, tag) {
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

/** The `agg="<tag>"` count row of a size-guarded answer (0 when absent: nothing reports). */
export function sizeFromRows(rows, tag) {
  for (let i = 0; i < rows.length; i++) {
    if (isRow(rows[i]) && rows[i].metric.agg === tag) return num(rows[i].value[1]) || 0;
  }
  return 0;
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

/**
 * Cluster totals for the Metrics page summary as server-side aggregates: a
 * handful of rows whatever the cluster size, instead of every gauge of every
 * GPU. Each aggregation is tagged with an `agg` label (sum / count / nodes)
 * so the rows survive `or` next to each other and next to a per-GPU query.
 */
export function summaryQuery() {
  const s = summaryNames();
  const E = SERIES.exporter;
  return 'label_replace(sum by (__name__) ({__name__=~"' + s.sum.join('|') + '"}), "agg", "sum", "", "")' +
    ' or label_replace(count by (__name__) ({__name__=~"' + s.count.join('|') + '"}), "agg", "count", "", "")' +
    ' or label_replace(count by (__name__) (count by (__name__, hostname) ({__name__="' + E.power + '"})), "agg", "nodes", "", "")';
}

/**
 * Rows of a summaryQuery answer (those with an `agg` label) → the shape of
 * summarizeMetrics plus `nodes` (nodes reporting); null when there are none.
 */
export function totalsFromRows(rows) {
  const E = SERIES.exporter;
  const sum = {};
  const cnt = {};
  let nodes = 0;
  let any = false;
  for (let i = 0; i < rows.length; i++) {
    const row = rows[i];
    if (!isRow(row) || typeof row.metric.agg !== 'string') continue;
    const v = num(row.value[1]);
    if (v === null) continue;
    const name = row.metric.__name__;
    any = true;
    if (row.metric.agg === 'sum') sum[name] = v;
    else if (row.metric.agg === 'count') cnt[name] = v;
    else if (row.metric.agg === 'nodes' && name === E.power) nodes = v;
  }
  if (!any) return null;
  const c = function (n) { return cnt[n] || 0; };
  const s = function (n) { return sum[n] || 0; };
  const gpus = c(E.power);
  const capAssumed = Math.max(0, gpus - c(E.powerCap));
  const eccGpus = c(E.eccUncorrect);
  return {
    gpus: gpus,
    withPower: gpus,
    nodes: nodes,
    powerWatts: s(E.power),
    // GPUs without a cap series get the MI355X board limit, as in the per-GPU join.
    powerCapWatts: s(E.powerCap) + capAssumed * MI355X.tdpWatts,
    vramUsedBytes: s(E.vramUsed) * SERIES.exporterVramUnitBytes,
    vramTotalBytes: s(E.vramTotal) * SERIES.exporterVramUnitBytes,
    avgGfxActivityPct: c(E.gfx) ? s(E.gfx) / c(E.gfx) : null,
    eccCorrectable: eccGpus ? s(E.eccCorrect) : null,
    eccUncorrectable: eccGpus ? s(E.eccUncorrect) : null,
    powerCapAssumed: capAssumed,
    tempLimitAssumed: Math.max(0, c(E.temp) - c(E.tempSlowdown)),
  };
}

/**
 * True when every exporter row of a combined result (splitByName output)
 * carries a `hostname` label; node-exporter rows in a merged result are not
 * looked at.
 */
export function keyedByHostname(rows) {
  let n = 0;
  for (const k in rows) {
    const list = rows[k];
    if (!Array.isArray(list) || (k !== '__xgmi' && !isExporterName(k))) continue;
    for (let i = 0; i < list.length; i++) {
      const m = list[i] && list[i].metric;
      if (!m || !m.hostname) return false;
      n++;
    }
  }
  return n > 0;
}

/** A PromQL double-quoted string literal body. */
export function promString(s) {
  return String(s).replace(/\\/g, '\\\\').replace(/"/g, '\\"');
}

/**
 * The exporter query scoped to ONE node (`hostname` label = Kubernetes node
 * name, the same key the joins and views use): what the native Node / Pod
 * detail pages ask for, O(GPUs per node) series whatever the cluster size.
 */
export function exporterNodeQuery(nodeName, withStatic) {
  const names = exporterNames(withStatic);
  // Every row matches the hostname matcher: the live-only query needs no fallback keys.
  const labels = withStatic === false ? EXPORTER_LEAN_LABELS : EXPORTER_JOIN_LABELS;
  return 'max by (' + labels.join(', ') + ') ({__name__=~"' + names.join('|') + '", hostname="' +
    promString(nodeName) + '"})';
}

/**
 * Pod → GPU attribution only (the Pods page): the power gauge of GPUs whose
 * `pod` label is set — one series per allocated GPU, instead of every live
 * gauge and xGMI link of every GPU.
 */
export function ownersQuery(pods, small) {
  const sel = '{__name__="' + SERIES.exporter.power + '", ';
  if (small) {
    // Every owner when they fit on one page of the Pods table, else the page's pods (smallClusterQuery).
    const n = gpuPodCount();
    const all = sizeGuard(ownersQuery(null), true, n, SMALL_CLUSTER_PODS);
    const page = pods && pods.length ? ' or ' + sizeGuard(ownersQuery(pods), false, n, SMALL_CLUSTER_PODS) : '';
    return all + page + ' or ' + sizeRow(n, 'gpu_pods');
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

/** Total GPU power per pod from the exporter's pod labels; `filter` is a substring of the pod name. */
export function podPowerSum(filter) {
  const f = typeof filter === 'string' ? filter.trim().toLowerCase() : '';
  return 'sum by (namespace, pod) ({__name__="' + SERIES.exporter.power + '", pod!=""' +
    (f ? ', pod=~".*' + promString(regexLiteral(f)) + '.*"' : '') + '})';
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

/** The part of a snapshot that belongs to one node (GPU objects shared, not copied). */
export function nodeSlice(m, nodeName) {
  if (!m) return m;
  const out = {};
  for (const k in m) out[k] = m[k];
  out.gpus = m.gpus.filter(function (g) { return g.nodeName === nodeName; });
  out.xgmi = {};
  out.links = {};
  if (m.xgmi && m.xgmi[nodeName]) out.xgmi[nodeName] = m.xgmi[nodeName];
  if (m.links && m.links[nodeName]) out.links[nodeName] = m.links[nodeName];
  out.scope = nodeName;
  return out;
}

export function nodeExporterQuery() {
  const N = SERIES.nodeExporter;
  const names = [N.chips.split('{')[0], N.power, N.powerInput, N.powerCap, N.busy, N.vramUsed, N.vramTotal, N.uname];
  return '{__name__=~"' + names.join('|') + '"}';
}

/** Labels the node-exporter join reads (hwmon chip, DRM card, uname). */
export const NODE_EXPORTER_JOIN_LABELS = ['__name__', 'instance', 'node', 'nodename', 'chip', 'chip_name', 'card'];

/**
 * First query of a session, while it is not yet known which exporter feeds
 * this Prometheus: both exporters' series in ONE request, projected onto the
 * union of the labels the two joins read. Later refreshes ask only the
 * exporter that answered.
 */
export function mergedQuery(withStatic, view) {
  const N = SERIES.nodeExporter;
  const names = exporterNames(withStatic, view);
  names.push(N.chips.split('{')[0], N.power, N.powerInput, N.powerCap, N.busy, N.vramUsed, N.vramTotal, N.uname);
  const labels = EXPORTER_JOIN_LABELS.slice();
  for (let i = 0; i < NODE_EXPORTER_JOIN_LABELS.length; i++) {
    if (labels.indexOf(NODE_EXPORTER_JOIN_LABELS[i]) < 0) labels.push(NODE_EXPORTER_JOIN_LABELS[i]);
  }
  return 'max by (' + labels.join(', ') + ') ({__name__=~"' + names.join('|') + '"})';
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

/** Key of the cluster-wide line in a scoped series answer (no node name can be this). */
export const TOTAL_SERIES = '\u0000cluster';

/**
 * A result row whose label values are all strings, as Prometheus promises: a
 * label of any other type (a broken proxy, a hand-written exporter) is
 * dropped, so no join, total or view ever takes an object or a number for a
 * node, pod or card name. The row itself is returned when it is clean.
 */
export function stringLabels(row) {
  const m = row && row.metric;
  if (!isObject(m)) return row;
  for (const k in m) {
    if (typeof m[k] !== 'string') {
      const clean = {};
      for (const k2 in m) if (typeof m[k2] === 'string') clean[k2] = m[k2];
      return { metric: clean, value: row.value };
    }
  }
  return row;
}

/** Split a combined result into `name → rows` (xGMI rows under `__xgmi`). */
export function splitByName(result) {
  // No prototype: a series named e.g. "__proto__" is a plain key here.
  const out = Object.create(null);
  out.__xgmi = [];
  // Cluster aggregates (summaryQuery) carry an `agg` label and share metric
  // names with the per-GPU rows: kept apart so no join mistakes one for a GPU.
  out.__agg = [];
  const N = SERIES.nodeExporter;
  const xre = new RegExp('^' + SERIES.exporter.xgmiRe + '$');
  for (let i = 0; i < result.length; i++) {
    const row = result[i];
    const m = row && row.metric;
    if (!isObject(m)) continue;
    if (typeof m.agg === 'string') {
      out.__agg.push(row);
      continue;
    }
    const name = typeof m.__name__ === 'string' ? m.__name__ : '';
    if (xre.test(name)) {
      out.__xgmi.push(row);
      continue;
    }
    // The chip-name series is keyed by its full selector in SERIES.
    const key = name === 'node_hwmon_chip_names' ? (m.chip_name === 'amdgpu' ? N.chips : null) : name;
    if (!key) continue;
    if (!out[key]) out[key] = [];
    out[key].push(row);
  }
  return out;
}

// ---------------------------------------------------------------------------
// Structural sharing between consecutive snapshots
// ---------------------------------------------------------------------------

/** Deep equality for the plain JSON-like values a snapshot holds. */
function sameValue(a, b) {
  if (a === b) return true;
  if (!a || !b || typeof a !== 'object' || typeof b !== 'object') return false;
  const ka = Object.keys(a);
  if (ka.length !== Object.keys(b).length) return false;
  for (let i = 0; i < ka.length; i++) {
    if (!sameValue(a[ka[i]], b[ka[i]])) return false;
  }
  return true;
}

/**
 * Reuse objects of `prev` wherever `next` holds equal content, so that
 * identity-keyed memos downstream (view sections, renderers) hit when a
 * refresh returns what the last one did — the common case, since exporters
 * are scraped every 15-30 s and a dashboard refreshes more often than that.
 * GPU lists are matched by (node, gpu); maps by key. Returns `prev` itself
 * when nothing changed.
 */
export function shareGpus(prev, next) {
  if (!prev) return next;
  const byKey = {};
  for (let i = 0; i < prev.length; i++) byKey[prev[i].nodeName + '\u0000' + prev[i].gpu] = prev[i];
  let all = prev.length === next.length;
  const out = new Array(next.length);
  for (let i = 0; i < next.length; i++) {
    const p = byKey[next[i].nodeName + '\u0000' + next[i].gpu];
    if (p && sameValue(p, next[i])) {
      out[i] = p;
      if (prev[i] !== p) all = false;
    } else {
      out[i] = next[i];
      all = false;
    }
  }
  return all ? prev : out;
}

export function shareMap(prev, next) {
  if (!prev) return next;
  const out = {};
  let all = Object.keys(prev).length === Object.keys(next).length;
  for (const k in next) {
    if (prev[k] !== undefined && sameValue(prev[k], next[k])) {
      out[k] = prev[k];
    } else {
      out[k] = next[k];
      all = false;
    }
  }
  return all ? prev : out;
}

/**
 * @param {{ request: (path: string) => Promise<any>, timeoutMs?: number,
 *           clock?: {setTimeout: Function, clearTimeout: Function, now: Function},
 *           services?: Array<{namespace: string, service: string, port: string}>,
 *           discoveryTtlMs?: number,
 *           onTrace?: (span: {name: string, path: string, start: number, end: number, ok: boolean}) => void }} opts
 */
export function createMetricsSource(opts) {
  const request = opts.request;
  const timeoutMs = opts.timeoutMs || DEFAULT_REQUEST_TIMEOUT_MS;
  const clock = opts.clock || { setTimeout: setTimeout, clearTimeout: clearTimeout, now: Date.now };
  const services = opts.services || PROMETHEUS_SERVICES;
  const ttl = opts.discoveryTtlMs === undefined ? DISCOVERY_TTL_MS : opts.discoveryTtlMs;
  const onTrace = opts.onTrace || null;

  let cachedPath = null;
  let cachedAt = 0;
  let discovering = null;
  let source = null; // which exporter answered last time
  let links = null; // measured xGMI link topology per node (static), refreshed every `ttl` with `statics`
  let statics = null; // static per-GPU fields (STATIC_GPU_FIELDS), fetched with the topology
  let linksAt = 0;
  let lean = false; // the last static query showed every exporter series keyed by hostname
  let lastBy = {}; // view → previous snapshot, for structural sharing and stale fallbacks
  const failuresBy = {}; // view → consecutive failed fetches against the cached service

  // HTTP status of the most recent failed request (401 / 403: the user may not
  // proxy to the Prometheus service — RBAC, not an outage); 0 after a success.
  let lastFailureStatus = 0;

  function get(name, path) {
    const start = clock.now();
    const p = withTimeout(request(path), timeoutMs, clock).then(
      function (v) { lastFailureStatus = 0; return v; },
      function (e) {
        const st = e && (e.status || (e.response && e.response.status));
        lastFailureStatus = typeof st === 'number' ? st : -1;
        throw e;
      }
    );
    if (!onTrace) return p;
    return p.then(
      function (v) { onTrace({ name: name, path: path, start: start, end: clock.now(), ok: true }); return v; },
      function (e) { onTrace({ name: name, path: path, start: start, end: clock.now(), ok: false }); throw e; }
    );
  }

  function probe(svc) {
    const base = servicePath(svc);
    return get('probe', base + '/api/v1/query?query=1').then(
      function (raw) { return raw && raw.status === 'success' ? base : null; },
      function () { return null; }
    );
  }

  /** Base proxy path of a reachable Prometheus, or null. Parallel probes, cached. */
  function discover() {
    if (cachedPath && clock.now() - cachedAt < ttl) return Promise.resolve(cachedPath);
    if (discovering) return discovering;
    discovering = Promise.all(services.map(probe)).then(function (paths) {
      discovering = null;
      for (let i = 0; i < paths.length; i++) {
        if (paths[i]) {
          cachedPath = paths[i];
          cachedAt = clock.now();
          return cachedPath;
        }
      }
      cachedPath = null;
      return null;
    });
    return discovering;
  }

  function invalidate() {
    cachedPath = null;
    source = null;
    lean = false;
    seriesCache = null;
    links = null;
    statics = null;
    lastBy = {};
    scopeStatic = {};
    scopedState = new Map();
    noGpusUntil = 0;
    for (const k in nodeStates) delete nodeStates[k];
  }

  /** Marker for "the request did not reach a Prometheus". */
  const UNREACHABLE = {};

  // Fetches in flight, by what they fetch: a second caller while one is
  // pending (two views on one page, React StrictMode re-running a mount
  // effect, a poller tick during a click) shares its answer instead of
  // sending the same query again.
  const inflight = {};
  function shared(key, make) {
    if (inflight[key]) return inflight[key];
    const p = make();
    inflight[key] = p;
    const done = function () { if (inflight[key] === p) delete inflight[key]; };
    p.then(done, done);
    return p;
  }

  /**
   * Run `fn(base)` against Prometheus. With no cached service the preferred
   * candidate is queried directly — its answer doubles as discovery, so the
   * first fetch costs one round trip instead of probe + query; only when it
   * does not answer are all candidates probed in parallel. `fn` resolves to
   * UNREACHABLE when its request failed.
   */
  function withPrometheus(fn, onCachedFailure) {
    if (cachedPath && clock.now() - cachedAt < ttl) {
      const base = cachedPath;
      return fn(base).then(function (r) { return r === UNREACHABLE ? onCachedFailure() : r; });
    }
    const first = servicePath(services[0]);
    return fn(first).then(function (r) {
      if (r !== UNREACHABLE) {
        cachedPath = first;
        cachedAt = clock.now();
        return r;
      }
      return discover().then(function (base) {
        if (!base) return null;
        return fn(base).then(function (r2) { return r2 === UNREACHABLE ? onCachedFailure() : r2; });
      });
    });
  }

  function instant(base, q) {
    return get('query', base + '/api/v1/query?query=' + encodeURIComponent(q)).then(function (raw) {
      if (!raw || raw.status !== 'success' || !raw.data || !Array.isArray(raw.data.result)) return [];
      return raw.data.result.map(stringLabels);
    });
  }

  /** Run one combined query; resolves {rows: name → results, ok}. */
  function combined(base, q) {
    return instant(base, q).then(
      function (res) { return { rows: splitByName(res), ok: true }; },
      function () { return { rows: {}, ok: false }; }
    );
  }

  /**
   * One metrics snapshot of the series `view` needs (METRIC_VIEWS; default
   * 'all'). Resolves to null when no Prometheus is reachable (the page's
   * "Prometheus Unreachable" state).
   * @param {string} [view]
   * @returns {Promise<GpuMetrics|null>}
   */
  function fetchGpuMetrics(view, opts) {
    const v = view === undefined ? 'all' : view;
    if (METRIC_VIEWS.indexOf(v) < 0) return Promise.reject(new Error('fetchGpuMetrics: unknown view ' + JSON.stringify(view)));
    if (opts && opts.rank) {
      // A page of GPU nodes in power order (rankedClusterQuery).
      const rank = {
        by: 'power',
        page: Math.max(0, Math.floor(opts.rank.page) || 0),
        per: opts.rank.per > 0 ? Math.min(200, Math.floor(opts.rank.per)) : 8,
        filter: String(opts.rank.filter || '').trim().toLowerCase(),
      };
      const rkey = 'rank|' + v + '|' + rank.page + '|' + rank.per + '|' + rank.filter + (opts.summary ? '|sum' : '');
      return shared(rkey, function () { return rankedSnapshot(v, rank, !!opts.summary, rkey); });
    }
    const scope = opts && Array.isArray(opts.scope) ? opts.scope.map(String) : null;
    if (!scope) return shared('gpus|' + v, function () { return gpuSnapshot(v); });
    const summary = !!opts.summary;
    const small = !!opts.small;
    const key = v + '|' + (summary ? 'sum' : '') + '|' + (small ? 'small|' : '') + scope.join(',');
    return shared('scoped|' + key, function () { return scopedSnapshot(v, scope, summary, key, small); });
  }

  // ---- Scoped snapshots (paged views: the GPU nodes on screen) -------------

  // node → {at, statics: gpuKey → static fields, links}: static series of the
  // nodes a paged view has shown, re-read per node every `ttl`.
  let scopeStatic = {};
  // scoped key → {last, failures}; the most recent SCOPED_KEYS kept.
  let scopedState = new Map();
  const SCOPED_KEYS = 16;

  function scopedEntry(key) {
    let e = scopedState.get(key);
    if (e) {
      scopedState.delete(key); // most recently used last
    } else {
      e = { last: null, failures: 0 };
    }
    scopedState.set(key, e);
    if (scopedState.size > SCOPED_KEYS) scopedState.delete(scopedState.keys().next().value);
    return e;
  }

  /**
   * Static series of a scoped answer: kept per node when the answer carried
   * them (`withStatic`), else filled in from that per-node copy. A GPU the
   * copy does not know yet marks its node to be re-read next time.
   */
  function scopeStatics(j, scope, withStatic) {
    const now = clock.now();
    if (withStatic) {
      const per = {};
      for (let i = 0; i < scope.length; i++) per[scope[i]] = {};
      const sts = staticsOf(j.gpus);
      for (let i = 0; i < j.gpus.length; i++) {
        const g = j.gpus[i];
        if (!per[g.nodeName]) per[g.nodeName] = {};
        per[g.nodeName][gpuKey(g)] = sts[gpuKey(g)];
      }
      for (const n in per) scopeStatic[n] = { at: now, statics: per[n], links: (j.links && j.links[n]) || {} };
      return;
    }
    const merged = {};
    const links = {};
    for (let i = 0; i < scope.length; i++) {
      const e = scopeStatic[scope[i]];
      if (!e) continue;
      for (const k in e.statics) merged[k] = e.statics[k];
      if (Object.keys(e.links).length) links[scope[i]] = e.links;
    }
    for (let i = 0; i < j.gpus.length; i++) {
      const g = j.gpus[i];
      if (merged[gpuKey(g)]) continue;
      // Not known yet: re-read this node's statics next time.
      if (scopeStatic[g.nodeName]) scopeStatic[g.nodeName].at = -Infinity;
      else scopeStatic[g.nodeName] = { at: -Infinity, statics: {}, links: {} };
    }
    applyStatics(j.gpus, merged);
    j.links = links;
  }

  function scopeNeedsStatic(scope) {
    const now = clock.now();
    for (let i = 0; i < scope.length; i++) {
      const e = scopeStatic[scope[i]];
      if (!e || now - e.at >= ttl) return true;
    }
    return false;
  }

  /**
   * Telemetry of the GPU nodes a paged view shows (`scope`: Kubernetes node
   * names = exporter `hostname`), plus the cluster totals when `summary`: one
   * request whose size follows the page, not the cluster — `hostname=~` on
   * the per-GPU series, server-side aggregates for the totals (summaryQuery),
   * joined with `or`. A node-exporter source (no `hostname` label) or a
   * first query that finds no exporter series falls back to the cluster-wide
   * snapshot cut to the scope. Stale / null handling as in the cluster-wide
   * path, per scope.
   *
   * `small`: the page may be the whole cluster (smallClusterQuery) — every
   * GPU when at most SMALL_CLUSTER_NODES nodes report, else `scope`'s. The
   * answer says which (`small.exceeded`).
   */
  function scopedSnapshot(v, scope, summary, key, small) {
    const st = scopedEntry(key);
    if (source === 'node-exporter') return clusterCut(v, scope, summary, key);
    return withPrometheus(function (base) {
      // Nothing cached yet for a small-cluster fetch before the node list: statics too.
      const withStatic = small && scope.length === 0 ? true : scope.length > 0 && scopeNeedsStatic(scope);
      const parts = [];
      if (small) parts.push(smallClusterQuery(withStatic, v, scope));
      else if (scope.length) parts.push(exporterQuery(withStatic, true, v, scope));
      if (summary) parts.push(summaryQuery());
      if (!parts.length) return Promise.resolve(scopedResult(st, base, null, { gpus: [], xgmi: {}, links: {} }, scope, undefined, v));
      const q = parts.join(' or ');
      return combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const rows = res.rows;
        const j = joinExporterResults(rows);
        const totals = summary ? totalsFromRows(rows.__agg.filter(function (r) { return r.metric.agg !== 'gpu_nodes'; })) : undefined;
        const reporting = small ? sizeFromRows(rows.__agg, 'gpu_nodes') : 0;
        const found = j.gpus.length > 0 || (!!totals && totals.gpus > 0) || reporting > 0;
        // Nothing from the exporter yet: maybe node-exporter feeds this
        // Prometheus (no hostname label) — ask cluster-wide to find out, at
        // most once per discovery TTL when that finds no GPU either (a
        // cluster without GPU telemetry would otherwise pay two round trips
        // on every refresh).
        if (!found && source !== 'amd-exporter' && clock.now() >= noGpusUntil) return NOT_SCOPED;
        if (found) source = 'amd-exporter';
        scopeStatics(j, scope, withStatic);
        const sized = small ? { count: reporting, limit: SMALL_CLUSTER_NODES, exceeded: reporting > SMALL_CLUSTER_NODES } : undefined;
        return scopedResult(st, base, q, j, scope, totals, v, sized);
      });
    }, function () {
      st.failures++;
      if (st.last && st.failures < STALE_FAILURES) return Object.assign({}, st.last, { stale: true });
      st.last = null;
      invalidate(); // as the cluster-wide path: Prometheus is re-discovered next time
      return null;
    }).then(function (r) { return r === NOT_SCOPED ? clusterCut(v, scope, summary, key) : r; });
  }

  function scopedResult(st, base, q, j, scope, totals, v, sized) {
    const prev = st.last;
    st.last = {
      source: source,
      view: v,
      gpus: prev ? shareGpus(prev.gpus, j.gpus) : j.gpus,
      xgmi: prev ? shareMap(prev.xgmi, j.xgmi) : j.xgmi,
      links: prev ? shareMap(prev.links, j.links || {}) : j.links || {},
      fetchedAt: new Date(clock.now()).toISOString(),
      prometheusPath: base,
      query: q,
      scope: scope,
      totals: totals && prev && prev.totals && sameValue(prev.totals, totals) ? prev.totals : totals,
      // A small-cluster query: how many GPU nodes report, and whether that was more than one page.
      small: sized,
    };
    return st.last;
  }

  /**
   * One page of GPU nodes ranked by total GPU power (rankedClusterQuery):
   * `scope` is the page's nodes in rank order, `rank` the page, the ranked
   * count and each node's watts. Static series ride along (the page's names
   * are not known before the answer). Stale / null handling as scoped.
   */
  function rankedSnapshot(v, rank, summary, key) {
    const st = scopedEntry(key);
    return withPrometheus(function (base) {
      // The page's names come with the answer: ask for the static series
      // while the nodes last shown (most likely shown again) lack a copy.
      const prev = st.last && st.last.scope;
      const withStatic = !prev || prev.length === 0 || scopeNeedsStatic(prev);
      const q = rankedClusterQuery(v, rank, withStatic) + (summary ? ' or ' + summaryQuery() : '');
      return combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const rows = res.rows;
        const j = joinExporterResults(rows);
        const ranked = [];
        const watts = {};
        for (let i = 0; i < rows.__agg.length; i++) {
          const r = rows.__agg[i];
          if (!isRow(r) || r.metric.agg !== 'rank' || typeof r.metric.hostname !== 'string') continue;
          const w = num(r.value[1]);
          ranked.push([r.metric.hostname, w === null ? -Infinity : w]);
          watts[r.metric.hostname] = w;
        }
        ranked.sort(function (a, b) { return b[1] - a[1] || (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0); });
        const names = ranked.map(function (x) { return x[0]; });
        scopeStatics(j, names, withStatic);
        const count = sizeFromRows(rows.__agg, 'ranked');
        const totals = summary
          ? totalsFromRows(rows.__agg.filter(function (r) { return r.metric.agg !== 'rank' && r.metric.agg !== 'ranked'; }))
          : undefined;
        if (j.gpus.length > 0 || count > 0) source = 'amd-exporter';
        // Nothing ranked and no exporter seen: maybe node-exporter feeds this
        // Prometheus (no hostname label to rank by) — the cluster-wide
        // snapshot instead, in name order.
        else if (source !== 'amd-exporter') return NOT_SCOPED;
        const out = scopedResult(st, base, q, j, names, totals, v, undefined);
        out.rank = { by: rank.by, page: rank.page, per: rank.per, filter: rank.filter, count: count, watts: watts };
        return out;
      });
    }, function () {
      st.failures++;
      if (st.last && st.failures < STALE_FAILURES) return Object.assign({}, st.last, { stale: true });
      st.last = null;
      invalidate();
      return null;
    }).then(function (r) { return r === NOT_SCOPED ? fetchGpuMetrics(v) : r; });
  }

  // Until then a scoped fetch that finds nothing does not ask cluster-wide
  // again: the last cluster-wide look found no GPU telemetry at all.
  let noGpusUntil = 0;

  /** The cluster-wide snapshot cut to `scope` (node-exporter source; exporter not found by a scoped query). */
  function clusterCut(v, scope, summary, key) {
    return fetchGpuMetrics(v).then(function (m) {
      if (!m) return null;
      if (m.gpus.length === 0) noGpusUntil = clock.now() + ttl;
      const st = scopedEntry(key);
      if (st.cutOf === m && st.last) return st.last;
      const inScope = {};
      for (let i = 0; i < scope.length; i++) inScope[scope[i]] = true;
      const xgmi = {};
      const links = {};
      for (let i = 0; i < scope.length; i++) {
        if (m.xgmi && m.xgmi[scope[i]]) xgmi[scope[i]] = m.xgmi[scope[i]];
        if (m.links && m.links[scope[i]]) links[scope[i]] = m.links[scope[i]];
      }
      let totals;
      if (summary) {
        const seen = {};
        let nodes = 0;
        for (let i = 0; i < m.gpus.length; i++) {
          if (!seen[m.gpus[i].nodeName]) {
            seen[m.gpus[i].nodeName] = true;
            nodes++;
          }
        }
        totals = Object.assign(summarizeMetrics(m), { nodes: nodes });
      }
      const out = Object.assign({}, m, {
        gpus: m.gpus.filter(function (g) { return inScope[g.nodeName] === true; }),
        xgmi: xgmi,
        links: links,
        scope: scope,
        totals: totals,
      });
      st.cutOf = m;
      st.last = out;
      return out;
    });
  }

  function gpuSnapshot(v) {
    return withPrometheus(function (base) { return snapshotFrom(base, v); }, function () {
      // A transient failure (timeout, 5xx) serves the last snapshot marked
      // stale; only repeated failures mean Prometheus went away.
      failuresBy[v] = (failuresBy[v] || 0) + 1;
      const last = lastBy[v];
      if (last && failuresBy[v] < STALE_FAILURES) {
        return Object.assign({}, last, { stale: true });
      }
      invalidate();
      return null;
    });
  }

  function snapshotFrom(base, view) {
    const withStatic = links === null || clock.now() - linksAt >= ttl;
    const q = source === 'amd-exporter' ? exporterQuery(withStatic, lean, view)
      : source === 'node-exporter' ? nodeExporterQuery() : mergedQuery(withStatic, view);
    return combined(base, q).then(function (res) {
      if (!res.ok) return UNREACHABLE;
      failuresBy[view] = 0;
      const rows = res.rows;
      let joined = { gpus: [], xgmi: {}, links: {} };
      let src = null;
      if (source !== 'node-exporter') {
        const j = joinExporterResults(rows);
        if (j.gpus.length) {
          joined = j;
          src = 'amd-exporter';
          if (withStatic) {
            links = j.links;
            statics = staticsOf(j.gpus);
            linksAt = clock.now();
            lean = keyedByHostname(rows);
          } else {
            joined.links = links;
            // A GPU the static copy does not know yet (node added since):
            // fetch the static series again on the next refresh.
            if (!applyStatics(j.gpus, statics)) linksAt = -Infinity;
          }
        }
      }
      if (!src && source !== 'amd-exporter') {
        const j = joinNodeExporterResults(rows);
        if (j.gpus.length) {
          joined = j;
          src = 'node-exporter';
        }
      }
      const last = lastBy[view];
      const same = last && last.source === src;
      source = src;
      lastBy[view] = {
        source: src,
        view: view,
        gpus: same ? shareGpus(last.gpus, joined.gpus) : joined.gpus,
        xgmi: same ? shareMap(last.xgmi, joined.xgmi) : joined.xgmi,
        links: same ? shareMap(last.links, joined.links || {}) : joined.links || {},
        fetchedAt: new Date(clock.now()).toISOString(),
        prometheusPath: base,
        // The PromQL this snapshot came from (Metrics page "Query" row).
        query: q,
      };
      return lastBy[view];
    });
  }

  // Per-node snapshots for the detail pages: node → {last, links, statics, staticAt, failures}.
  const nodeStates = {};
  /** Marker: the scoped query found no exporter GPU on this node. */
  const NOT_SCOPED = {};

  /**
   * Telemetry of ONE node's GPUs — what the native Node and Pod detail pages
   * show. The exporter query carries a `hostname` matcher, so opening a
   * detail page moves O(GPUs per node) bytes (a few KB) instead of the whole
   * cluster's telemetry (O(GPUs in the cluster): MBs on a few hundred
   * nodes). Static series (power cap, HBM size, throttle threshold, link
   * topology) are re-read per node every discovery TTL, as in the
   * cluster-wide path.
   *
   * Falls back to the cluster-wide snapshot, cut to the node, when the
   * scoped query finds no GPU: node-exporter as the source (its series carry
   * `instance`, not `hostname`) or an exporter whose hostname label is not
   * the node name. Transient failures serve the node's last snapshot marked
   * stale, like fetchGpuMetrics. Resolves to null when Prometheus is
   * unreachable.
   * @param {string} nodeName
   * @returns {Promise<GpuMetrics|null>}
   */
  function fetchNodeMetrics(nodeName) {
    return shared('node|' + String(nodeName), function () { return nodeSnapshot(String(nodeName)); });
  }

  function nodeSnapshot(key) {
    if (!nodeStates[key]) nodeStates[key] = { last: null, links: null, statics: null, staticAt: 0, failures: 0 };
    const st = nodeStates[key];
    function clusterWide() {
      return fetchGpuMetrics().then(function (m) { return m ? nodeSlice(m, key) : null; });
    }
    if (source === 'node-exporter') return clusterWide();
    return withPrometheus(function (base) {
      const withStatic = st.links === null || clock.now() - st.staticAt >= ttl;
      return combined(base, exporterNodeQuery(key, withStatic)).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const j = joinExporterResults(res.rows);
        if (!j.gpus.length) return NOT_SCOPED;
        if (withStatic) {
          st.links = j.links;
          st.statics = staticsOf(j.gpus);
          st.staticAt = clock.now();
        } else {
          j.links = st.links;
          if (!applyStatics(j.gpus, st.statics)) st.staticAt = -Infinity;
        }
        const prev = st.last;
        st.last = {
          source: 'amd-exporter',
          gpus: prev ? shareGpus(prev.gpus, j.gpus) : j.gpus,
          xgmi: prev ? shareMap(prev.xgmi, j.xgmi) : j.xgmi,
          links: prev ? shareMap(prev.links, j.links || {}) : j.links || {},
          fetchedAt: new Date(clock.now()).toISOString(),
          prometheusPath: base,
          scope: key,
        };
        return st.last;
      });
    }, function () {
      st.failures++;
      if (st.last && st.failures < STALE_FAILURES) return Object.assign({}, st.last, { stale: true });
      st.last = null;
      invalidate(); // as the cluster-wide path: Prometheus is re-discovered next time
      return null;
    }).then(function (r) { return r === NOT_SCOPED ? clusterWide() : r; });
  }

  let ownersLast = null;
  let ownersFailures = 0;

  /**
   * Which GPUs each pod holds (exporter `pod`/`namespace` labels) and their
   * power — all the Pods page reads from Prometheus — in one query whose
   * size follows the number of allocated GPUs, not every gauge of every GPU.
   * `gpus` lists the attributed GPUs only; an empty list means no
   * attribution (no pod on a GPU, or a source without pod labels, e.g.
   * node-exporter). Stale / null handling as in fetchGpuMetrics.
   * @returns {Promise<GpuMetrics|null>}
   */
  function fetchGpuOwners(opts) {
    const rank = opts && opts.rank;
    if (rank) {
      return shared('owners|rank|' + rank.page + '|' + rank.per + '|' + rank.filter, function () { return ownersRanked(rank); });
    }
    const pods = opts && Array.isArray(opts.pods) ? opts.pods.map(String) : null;
    const small = !!(opts && opts.small);
    if (small) return shared('owners|small|' + (pods || []).join(','), function () { return ownersSnapshot(pods || [], true); });
    if (pods && pods.length === 0) {
      return Promise.resolve({ source: source, gpus: [], xgmi: {}, links: {}, fetchedAt: new Date(clock.now()).toISOString(),
        prometheusPath: cachedPath, scope: 'owners' });
    }
    return shared('owners|' + (pods ? pods.join(',') : '*'), function () { return ownersSnapshot(pods); });
  }

  function ownersSnapshot(pods, small) {
    return withPrometheus(function (base) {
      return combined(base, ownersQuery(pods, small)).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        ownersFailures = 0;
        const j = joinExporterResults(res.rows);
        const owning = small ? sizeFromRows(res.rows.__agg, 'gpu_pods') : 0;
        ownersLast = {
          small: small ? { count: owning, limit: SMALL_CLUSTER_PODS, exceeded: owning > SMALL_CLUSTER_PODS } : undefined,
          source: j.gpus.length ? 'amd-exporter' : source,
          gpus: ownersLast ? shareGpus(ownersLast.gpus, j.gpus) : j.gpus,
          xgmi: {},
          links: {},
          fetchedAt: new Date(clock.now()).toISOString(),
          prometheusPath: base,
          scope: 'owners',
        };
        return ownersLast;
      });
    }, function () {
      ownersFailures++;
      if (ownersLast && ownersFailures < STALE_FAILURES) return Object.assign({}, ownersLast, { stale: true });
      ownersLast = null;
      invalidate();
      return null;
    });
  }

  /**
   * GPU pods in power order (rankedOwnersQuery): the page's owners plus
   * `rank` = {by, page, per, filter, count, order: "namespace/pod" keys
   * highest first, watts per key}.
   */
  function ownersRanked(rank) {
    return withPrometheus(function (base) {
      return combined(base, rankedOwnersQuery(rank)).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        ownersFailures = 0;
        const rows = res.rows;
        const j = joinExporterResults(rows);
        const ranked = [];
        const watts = {};
        for (let i = 0; i < rows.__agg.length; i++) {
          const r = rows.__agg[i];
          if (!isRow(r) || r.metric.agg !== 'rank' || typeof r.metric.pod !== 'string') continue;
          const key = (typeof r.metric.namespace === 'string' ? r.metric.namespace : '') + '/' + r.metric.pod;
          const w = num(r.value[1]);
          ranked.push([key, w === null ? -Infinity : w]);
          watts[key] = w;
        }
        ranked.sort(function (a, b) { return b[1] - a[1] || (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0); });
        ownersLast = {
          source: j.gpus.length ? 'amd-exporter' : source,
          gpus: ownersLast ? shareGpus(ownersLast.gpus, j.gpus) : j.gpus,
          xgmi: {},
          links: {},
          fetchedAt: new Date(clock.now()).toISOString(),
          prometheusPath: base,
          scope: 'owners',
          rank: { by: rank.by, page: rank.page, per: rank.per, filter: rank.filter, count: sizeFromRows(rows.__agg, 'ranked'),
            order: ranked.map(function (x) { return x[0]; }), watts: watts },
        };
        return ownersLast;
      });
    }, function () {
      ownersFailures++;
      if (ownersLast && ownersFailures < STALE_FAILURES) return Object.assign({}, ownersLast, { stale: true });
      ownersLast = null;
      invalidate();
      return null;
    });
  }

  // Incremental range cache: step-aligned samples per series key.
  let seriesCache = null; // { range, step, end, data: { power: {node: [[t,v]]}, vram: {...} } }

  /** One range query; resolves {name → {node → [[t, v]]}} or UNREACHABLE. */
  function rangeQuery(base, q, start, end, step) {
    const path = base + '/api/v1/query_range?query=' + encodeURIComponent(q) +
      '&start=' + start + '&end=' + end + '&step=' + step;
    return get('query_range', path).then(
      function (raw) {
        const out = Object.create(null);
        const res = raw && raw.status === 'success' && raw.data && Array.isArray(raw.data.result) ? raw.data.result : [];
        for (let i = 0; i < res.length; i++) {
          if (!res[i] || !isObject(res[i].metric) || !Array.isArray(res[i].values)) continue;
          const m = res[i].metric;
          const name = typeof m.__name__ === 'string' ? m.__name__ : '';
          const node = m.scope === 'cluster' ? TOTAL_SERIES
            : typeof m.hostname === 'string' && m.hostname ? m.hostname : typeof m.instance === 'string' && m.instance ? m.instance : 'cluster';
          // Only [t, v] pairs; a malformed point is dropped, not propagated.
          const vals = res[i].values.filter(function (p) { return Array.isArray(p) && p.length >= 2; });
          if (!out[name]) out[name] = Object.create(null);
          out[name][node] = vals;
        }
        return out;
      },
      function () { return UNREACHABLE; }
    );
  }

  /**
   * Per-node power and HBM-used time series over the last `rangeSec`.
   * Server-side `sum by (__name__, hostname)` keeps the payload
   * O(nodes × points) and both series in one request.
   *
   * Incremental: samples are aligned to `step`, and Prometheus never rewrites
   * a past step, so after the first call only the steps newer than the cache
   * are requested — and none at all until the next step boundary.
   * @returns {Promise<{ rangeSec: number, power: Record<string, Array<[number, number]>>, vram: Record<string, Array<[number, number]>> } | null>}
   */
  function fetchSeries(rangeSec, stepSec, scope, small) {
    const range = rangeSec || 1800;
    const step = stepSec || 30;
    const E = SERIES.exporter;
    const parts = [['power', E.power, 1], ['vram', E.vramUsed, SERIES.exporterVramUnitBytes]];
    const scoped = Array.isArray(scope);
    const sk = scoped ? (small ? 'small:' : '') + scope.map(String).join(',') : null;
    const q = scoped ? scopedSeriesQuery(scope.map(String), !!small) : seriesQuery();
    function from(base) {
      const end = Math.floor(clock.now() / 1000 / step) * step;
      const fresh = !seriesCache || seriesCache.range !== range || seriesCache.step !== step ||
        seriesCache.base !== base || seriesCache.scope !== sk || end - seriesCache.end >= range;
      const start = fresh ? end - range : seriesCache.end + step;
      if (!fresh && start > end) return Promise.resolve(seriesCache.data);
      return rangeQuery(base, q, start, end, step).then(function (got) {
        if (got === UNREACHABLE) return UNREACHABLE;
        const data = { rangeSec: range, stepSec: step };
        if (scoped) {
          data.scope = scope.map(String);
          data.total = {};
        }
        const cutoff = end - range;
        for (let i = 0; i < parts.length; i++) {
          const key = parts[i][0];
          const scale = parts[i][2];
          const rows = got[parts[i][1]] || {};
          const prev = fresh ? {} : seriesCache.data[key] || {};
          const merged = {};
          const nodes = Object.keys(Object.assign({}, prev, rows));
          for (let n = 0; n < nodes.length; n++) {
            if (nodes[n] === TOTAL_SERIES) continue;
            const add = (rows[nodes[n]] || []).map(function (v) { return [Number(v[0]), (num(v[1]) || 0) * scale]; });
            const pts = (prev[nodes[n]] || []).concat(add).filter(function (p) { return p[0] >= cutoff; });
            if (pts.length) merged[nodes[n]] = pts;
          }
          data[key] = merged;
          if (scoped) {
            // The cluster-wide line (peak / average over the whole cluster).
            const add = (rows[TOTAL_SERIES] || []).map(function (v) { return [Number(v[0]), (num(v[1]) || 0) * scale]; });
            const prevTotal = fresh ? [] : (seriesCache.data.total && seriesCache.data.total[key]) || [];
            data.total[key] = prevTotal.concat(add).filter(function (p) { return p[0] >= cutoff; });
          }
        }
        seriesCache = { range: range, step: step, end: end, base: base, scope: sk, data: data };
        return data;
      });
    }
    // A failed range request keeps the last window of the same scope (retried next time).
    return shared('series|' + range + '|' + step + '|' + sk, function () {
      return withPrometheus(from, function () { return seriesCache && seriesCache.scope === sk ? seriesCache.data : null; });
    });
  }

  /**
   * A pod's GPU power over the last `rangeSec` (podPowerQuery), step-aligned
   * like fetchSeries: `{rangeSec, power: [[t, W]]}`; `power` is empty when
   * the exporter attributes no GPU to the pod (no pod association, or the pod
   * holds none). Resolves to null when Prometheus is unreachable.
   * @returns {Promise<{rangeSec: number, power: Array<[number, number]>} | null>}
   */
  function fetchPodSeries(namespace, pod, rangeSec, stepSec) {
    return powerSeries('pod|' + namespace + '/' + pod, podPowerQuery(namespace, pod), rangeSec, stepSec);
  }

  /** A node's GPU power over the last `rangeSec` (nodePowerQuery); shape and nulls as fetchPodSeries. */
  function fetchNodeSeries(nodeName, rangeSec, stepSec) {
    return powerSeries('node|' + nodeName, nodePowerQuery(nodeName), rangeSec, stepSec);
  }

  function powerSeries(scope, q, rangeSec, stepSec) {
    const range = rangeSec || 1800;
    const step = stepSec || 30;
    const key = 'power|' + scope + '|' + range + '|' + step;
    return shared(key, function () {
      return withPrometheus(function (base) {
        const end = Math.floor(clock.now() / 1000 / step) * step;
        return rangeQuery(base, q, end - range, end, step).then(function (got) {
          if (got === UNREACHABLE) return UNREACHABLE;
          // Sum whatever rows came back per step (one row after `sum by (__name__)`).
          const total = {};
          const rows = got[SERIES.exporter.power] || {};
          for (const k in rows) {
            for (let i = 0; i < rows[k].length; i++) {
              const t = Number(rows[k][i][0]);
              const v = num(rows[k][i][1]);
              if (v !== null) total[t] = (total[t] || 0) + v;
            }
          }
          const power = Object.keys(total).map(Number).sort(function (a, b) { return a - b; })
            .map(function (t) { return [t, total[t]]; });
          return { rangeSec: range, stepSec: step, power: power };
        });
      }, function () { return null; });
    });
  }

  return {
    discover: discover,
    invalidate: invalidate,
    /**
     * Why the last fetch found no Prometheus: 'forbidden' when the proxy
     * answered 401 / 403 (the user lacks `services/proxy` get on the
     * Prometheus service), else 'unreachable'.
     */
    failureReason: function () { return lastFailureStatus === 401 || lastFailureStatus === 403 ? 'forbidden' : 'unreachable'; },
    fetchGpuMetrics: fetchGpuMetrics,
    fetchPodSeries: fetchPodSeries,
    fetchNodeSeries: fetchNodeSeries,
    fetchNodeMetrics: fetchNodeMetrics,
    fetchGpuOwners: fetchGpuOwners,
    fetchSeries: fetchSeries,
    source: function () { return source; },
  };
}

function gpuKey(g) {
  return g.nodeName + '\u0000' + g.gpu;
}

/** The static fields of each GPU, keyed by (node, gpu). */
export function staticsOf(gpus) {
  const out = {};
  for (let i = 0; i < gpus.length; i++) {
    const g = gpus[i];
    const v = {};
    for (let f = 0; f < STATIC_GPU_FIELDS.length; f++) v[STATIC_GPU_FIELDS[f]] = g[STATIC_GPU_FIELDS[f]];
    out[gpuKey(g)] = v;
  }
  return out;
}

/** Copy cached static fields onto freshly joined GPUs; false if some GPU has none cached. */
export function applyStatics(gpus, statics) {
  let complete = true;
  for (let i = 0; i < gpus.length; i++) {
    const c = statics && statics[gpuKey(gpus[i])];
    if (!c) {
      complete = false;
      continue;
    }
    for (let f = 0; f < STATIC_GPU_FIELDS.length; f++) gpus[i][STATIC_GPU_FIELDS[f]] = c[STATIC_GPU_FIELDS[f]];
  }
  return complete;
}

/**
 * Cluster power over a series window: the per-step sum over nodes
 * (fetchSeries aligns every node's samples to the same steps), then its peak
 * and mean — the "peak / average" figures the reference's Metrics mock-up
 * advertises but its code never computed (reference docs/screenshots/03-metrics.svg,
 * SURVEY.md Q12). Null when the window holds no sample.
 * @param {Record<string, Array<[number, number]>>} powerByNode
 * @returns {{peakWatts: number, peakAt: number, avgWatts: number, steps: number} | null}
 */
export function clusterPowerStats(powerByNode) {
  const total = {};
  for (const node in powerByNode || {}) {
    const pts = powerByNode[node] || [];
    for (let i = 0; i < pts.length; i++) {
      const t = pts[i][0];
      const v = pts[i][1];
      if (typeof v !== 'number' || !isFinite(v)) continue;
      total[t] = (total[t] || 0) + v;
    }
  }
  const ts = Object.keys(total);
  if (!ts.length) return null;
  let peak = -Infinity;
  let peakAt = 0;
  let sum = 0;
  for (let i = 0; i < ts.length; i++) {
    const v = total[ts[i]];
    sum += v;
    if (v > peak) {
      peak = v;
      peakAt = Number(ts[i]);
    }
  }
  return { peakWatts: peak, peakAt: peakAt, avgWatts: sum / ts.length, steps: ts.length };
}

/** Cluster totals for the summary box. */
export function summarizeMetrics(m) {
  let power = 0;
  let cap = 0;
  let vramUsed = 0;
  let vramTotal = 0;
  let gfx = 0;
  let gfxN = 0;
  let withPower = 0;
  let eccGpus = 0;
  let eccUncorrectable = 0;
  let eccCorrectable = 0;
  let capAssumed = 0;
  let tempLimitAssumed = 0;
  for (let i = 0; i < m.gpus.length; i++) {
    const g = m.gpus[i];
    if (g.powerCapAssumed) capAssumed++;
    if (g.tempC !== null && g.tempC !== undefined && !(g.tempSlowdownC > 0)) tempLimitAssumed++;
    if (g.eccUncorrectable !== null && g.eccUncorrectable !== undefined) {
      eccGpus++;
      eccUncorrectable += g.eccUncorrectable;
      eccCorrectable += g.eccCorrectable || 0;
    }
    if (g.powerWatts !== null) {
      power += g.powerWatts;
      withPower++;
    }
    if (g.powerCapWatts !== null) cap += g.powerCapWatts;
    if (g.vramUsedBytes !== null) vramUsed += g.vramUsedBytes;
    if (g.vramTotalBytes !== null) vramTotal += g.vramTotalBytes;
    if (g.gfxActivityPct !== null) {
      gfx += g.gfxActivityPct;
      gfxN++;
    }
  }
  return {
    gpus: m.gpus.length,
    withPower: withPower,
    powerWatts: power,
    powerCapWatts: cap,
    vramUsedBytes: vramUsed,
    vramTotalBytes: vramTotal,
    avgGfxActivityPct: gfxN ? gfx / gfxN : null,
    // RAS totals over the GPUs that report them (null: no GPU does, e.g. node-exporter)
    eccCorrectable: eccGpus ? eccCorrectable : null,
    eccUncorrectable: eccGpus ? eccUncorrectable : null,
    // GPUs whose power cap / throttle threshold is the MI355X platform value
    // because the source reports none (stock exporter, node-exporter).
    powerCapAssumed: capAssumed,
    tempLimitAssumed: tempLimitAssumed,
  };
}
