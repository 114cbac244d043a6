/**
 * Prometheus answers → per-GPU telemetry: the joins, the server-side totals,
 * the size rows of guarded queries, and structural sharing between
 * consecutive snapshots. Pure functions, no I/O.
 *
 * Reference analog: the join of src/api/metrics.ts:119-149, which keyed
 * power and TDP by PCI `chip` only (quirk Q1: on a homogeneous multi-node
 * cluster every node showed the last node's power). Here every GPU is keyed
 * by (node, gpu index).
 */

import { isObject, MI355X } from './k8sCore.js';
import { SERIES, STATIC_GPU_FIELDS } from './series.js';
import { isExporterName } from './promql.js';

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
 * @property {Record<string, Record<string, number>>} xgmi  node → GB/s sent over xGMI, keyed "src-dst" when
 *           the series named the peer, "src>k" for neighbour k (placed by topology.js placeThroughput)
 * @property {Record<string, Record<string, {type: string, hops: number, neighbor?: number}>>} links  node →
 *           "src-dst" → measured link (gpu_xgmi_link_hops; `neighbor` when the exporter publishes its neighbour
 *           order); empty when the exporter does not report topology
 * @property {string} fetchedAt
 * @property {boolean} [stale]  the latest fetch failed; this is the previous snapshot
 * @property {string} prometheusPath
 */

/** A number from a Prometheus sample value ("NaN", "+Inf" and junk → null). */
export function num(v) {
  const f = parseFloat(v);
  return isFinite(f) ? f : null;
}

/** A label value, or '' when it is missing or not a string. */
function labelStr(v) {
  return typeof v === 'string' ? v : '';
}

/** A well-formed instant-vector row: `{metric: {...}, value: [ts, "v"]}`. */
export function isRow(row) {
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
 * Keyed by (hostname, gpu_id). `nodeName`: the node a one-node answer
 * (promql.js exporterNodeQuery) is about — its rows leave out `hostname`, the
 * query's matcher. Exported for direct unit tests.
 */
export function joinExporterResults(r, nodeName) {
  const E = SERIES.exporter;
  const S = SERIES.nodeShaped;
  const fallback = typeof nodeName === 'string' ? nodeName : '';
  const map = {};
  function nodeOf(m) {
    return labelStr(m.hostname) || labelStr(m.node) || labelStr(m.instance) || fallback;
  }
  function slot(m) {
    // Label values are strings; anything else in a malformed answer is ignored.
    const node = nodeOf(m);
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

  // xGMI throughput as the series state it, placed on no peer yet:
  // `src-dst` when the row names its peer (a `peer_gpu_id` label), else
  // `src>k` for neighbour k of the stock exporter's
  // xgmi_neighbor_<k>_tx_throughput, whose neighbour numbering no series
  // documents. topology.js placeThroughput puts `src>k` on a peer only when a
  // link series pins neighbour k (this repo's amdgpu-exporter: the `neighbor`
  // label, from the KFD io_link order); otherwise it counts towards GPU src's
  // xGMI total alone.
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
      const peer = typeof m.peer_gpu_id === 'string' && m.peer_gpu_id !== '' ? parseInt(m.peer_gpu_id, 10) : NaN;
      if (peer === src) continue;
      const node = labelStr(m.hostname) || labelStr(m.instance) || fallback;
      if (!xgmi[node]) xgmi[node] = {};
      const v = num(xr[i].value[1]);
      if (v !== null) xgmi[node][isFinite(peer) ? src + '-' + peer : src + '>' + mm[1]] = v / 1e9;
    }
  }
  // The one-node answer's rows placed by Prometheus: on a link ("src-dst"),
  // or a GPU's total over the links nothing places ("src>*": counted towards
  // the GPU alone, topology.js placeThroughput).
  function shaped(list, keyOf) {
    if (!Array.isArray(list)) return;
    for (let i = 0; i < list.length; i++) {
      if (!isRow(list[i])) continue;
      const m = list[i].metric;
      const k = keyOf(m);
      const v = num(list[i].value[1]);
      if (k === null || v === null) continue;
      const node = nodeOf(m);
      (xgmi[node] || (xgmi[node] = {}))[k] = v / 1e9;
    }
  }
  shaped(r[S.xgmiLink], function (m) {
    const a = parseInt(m.gpu_id, 10);
    const b = parseInt(m.peer_gpu_id, 10);
    return isFinite(a) && isFinite(b) && a !== b ? a + '-' + b : null;
  });
  shaped(r[S.xgmiGpu], function (m) {
    const a = parseInt(m.gpu_id, 10);
    return isFinite(a) ? a + '>*' : null;
  });
  // Measured topology: gpu_xgmi_link_hops{gpu_id, peer_gpu_id[, neighbor]} per
  // xGMI-connected pair; `neighbor`: the link's place in gpu_id's neighbour order.
  const links = {};
  const lr = r[E.linkHops];
  if (Array.isArray(lr)) {
    for (let i = 0; i < lr.length; i++) {
      if (!isRow(lr[i])) continue;
      const m = lr[i].metric;
      const node = labelStr(m.hostname) || labelStr(m.instance) || fallback;
      const v = num(lr[i].value[1]);
      if (v === null || m.gpu_id === undefined || m.peer_gpu_id === undefined) continue;
      if (!links[node]) links[node] = {};
      const nb = typeof m.neighbor === 'string' && /^\d+$/.test(m.neighbor) ? parseInt(m.neighbor, 10) : -1;
      links[node][m.gpu_id + '-' + m.peer_gpu_id] = nb >= 0 ? { type: 'XGMI', hops: v, neighbor: nb } : { type: 'XGMI', hops: v };
    }
  }
  // A GPU with the full MI355X mesh arrives as its one-hop link count alone
  // (exporterNodeQuery): every other GPU of the node at one hop.
  const oh = r[S.oneHopLinks];
  if (Array.isArray(oh)) {
    const per = MI355X.xgmiLinksPerGpu;
    for (let i = 0; i < oh.length; i++) {
      if (!isRow(oh[i])) continue;
      const m = oh[i].metric;
      const a = parseInt(m.gpu_id, 10);
      if (num(oh[i].value[1]) !== per || !(a >= 0 && a <= per)) continue;
      const node = nodeOf(m);
      const l = links[node] || (links[node] = {});
      for (let b = 0; b <= per; b++) if (b !== a && !l[a + '-' + b]) l[a + '-' + b] = { type: 'XGMI', hops: 1 };
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
  // The query keeps the amdgpu "junction" sensor only (promql.js nodeExporterTempQuery).
  each(r[N.temp], chipKey, function (g, v) { g.tempC = v; });
  each(r[N.tempCrit], chipKey, function (g, v) { if (v !== null && v > 0) g.tempSlowdownC = v; });
  gpus.sort(byNodeGpu);
  return { gpus: gpus, xgmi: {}, links: {} };
}

/** The `agg="<tag>"` count row of a size-guarded answer (0 when absent: nothing reports). */
export function sizeFromRows(rows, tag) {
  for (let i = 0; i < rows.length; i++) {
    if (isRow(rows[i]) && rows[i].metric.agg === tag) return num(rows[i].value[1]) || 0;
  }
  return 0;
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

/** `agg` tags of nodeExporterSummaryQuery rows (promql.js). */
export const HW_TOTAL_TAGS = ['hw_gpus', 'hw_nodes', 'hw_power', 'hw_with_power', 'hw_cap', 'hw_vram_used',
  'hw_vram_total', 'hw_gfx_sum', 'hw_gfx_n'];

/**
 * Rows of a nodeExporterSummaryQuery answer → the totals summarizeMetrics
 * computes from the per-GPU node-exporter join (plus `nodes`); null when
 * there are none. node-exporter reports no RAS counters and no throttle
 * threshold, and a missing cap is not replaced (as in the join).
 */
export function hwTotalsFromRows(rows) {
  const v = {};
  let any = false;
  for (let i = 0; i < rows.length; i++) {
    const row = rows[i];
    if (!isRow(row) || HW_TOTAL_TAGS.indexOf(row.metric.agg) < 0) continue;
    const x = num(row.value[1]);
    if (x === null) continue;
    v[row.metric.agg] = x;
    any = true;
  }
  if (!any) return null;
  const g = function (k) { return v[k] || 0; };
  return {
    gpus: g('hw_gpus'),
    withPower: g('hw_with_power'),
    nodes: g('hw_nodes'),
    powerWatts: g('hw_power'),
    powerCapWatts: g('hw_cap'),
    vramUsedBytes: g('hw_vram_used'),
    vramTotalBytes: g('hw_vram_total'),
    avgGfxActivityPct: g('hw_gfx_n') ? g('hw_gfx_sum') / g('hw_gfx_n') : null,
    eccCorrectable: null,
    eccUncorrectable: null,
    powerCapAssumed: 0,
    tempLimitAssumed: 0,
  };
}

/**
 * The totals of a cluster where nothing reports: what a summary answer with
 * no aggregate rows means (summary asked, no exporter GPU anywhere), so the
 * Metrics page keeps saying that no GPU telemetry was found on every
 * refresh, not only on the first.
 */
export function zeroTotals() {
  return {
    gpus: 0, withPower: 0, nodes: 0, powerWatts: 0, powerCapWatts: 0, vramUsedBytes: 0, vramTotalBytes: 0,
    avgGfxActivityPct: null, eccCorrectable: null, eccUncorrectable: null, powerCapAssumed: 0, tempLimitAssumed: 0,
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
export function sameValue(a, b) {
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

/** Key of a GPU in maps: (node, device index). */
export function gpuKey(g) {
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
  const names = Object.keys(powerByNode || {});
  // One series (the cluster line the Metrics page passes) is its own sum.
  if (names.length === 1) return windowStats(powerByNode[names[0]] || []);
  const total = new Map();
  for (let n = 0; n < names.length; n++) {
    const pts = powerByNode[names[n]] || [];
    for (let i = 0; i < pts.length; i++) {
      const v = pts[i][1];
      if (typeof v !== 'number' || !isFinite(v)) continue;
      total.set(pts[i][0], (total.get(pts[i][0]) || 0) + v);
    }
  }
  const steps = [];
  total.forEach(function (v, t) { steps.push([t, v]); });
  steps.sort(function (a, b) { return a[0] - b[0]; });
  return windowStats(steps);
}

/** Peak (the earliest step holding it) and mean of one time-ordered series; null without a finite sample. */
function windowStats(pts) {
  let peak = -Infinity;
  let peakAt = 0;
  let sum = 0;
  let steps = 0;
  for (let i = 0; i < pts.length; i++) {
    const v = pts[i][1];
    if (typeof v !== 'number' || !isFinite(v)) continue;
    sum += v;
    steps++;
    if (v > peak) {
      peak = v;
      peakAt = Number(pts[i][0]);
    }
  }
  return steps ? { peakWatts: peak, peakAt: peakAt, avgWatts: sum / steps, steps: steps } : null;
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
