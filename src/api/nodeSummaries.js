/**
 * Per-node summaries of a telemetry snapshot, derived when the snapshot
 * arrives — metrics.js primes every snapshot it hands out — and kept with the
 * snapshot's objects (the client keeps them by identity while unchanged):
 *
 *   * nodePowerKeys: each node's GPU power against its summed caps,
 *     "watts|cap" in whole watts, and the bar the GPU Nodes summary draws;
 *   * nodeTempKeys: each node's hottest junction temperature, its throttle
 *     limit and the level of the unrounded reading, "temp|limit|level", and
 *     the cell's text;
 *   * ownersByNode: node → [{gpu, pod, namespace}] from exporter pod labels;
 *   * podGpuAssignments: "namespace/pod" → the GPUs attributed to the pod,
 *     and assignmentTexts, the GPU Pods row's "Assigned GPUs" and "GPU Power";
 *   * nonEmptyMap / topology.js linkFacts of every node's link maps.
 *
 * They are data-layer facts, like clusterIndex.js nodeFacts at list arrival:
 * the GPU Nodes page, its cards and the Node detail section read them. A
 * snapshot made elsewhere (a test) derives them on first read.
 */

import { BAR_COLORS, formatPercent, formatWatts, MI355X, pct, pctToColor } from './k8sCore.js';
import { linkFacts } from './topology.js';

const powerKeyCache = new WeakMap();
const tempKeyCache = new WeakMap();
const ownersCache = new WeakMap();
const nonEmpty = new WeakMap();
const assignCache = new WeakMap();
const textCache = new WeakMap();

/** `compute(gs)` once per GPU list of a telemetry snapshot. */
function perGpuList(cache, metrics, compute) {
  const gs = metrics && Array.isArray(metrics.gpus) ? metrics.gpus : null;
  if (!gs) return compute([]);
  if (cache.has(gs)) return cache.get(gs);
  const v = compute(gs);
  cache.set(gs, v);
  return v;
}

/**
 * Per-node GPU power from a telemetry snapshot: {byNode: {node: "watts|cap"}, sig, bars: {node: {watts, cap, pct,
 * color, text}}} in whole watts; `cap` null without a cap (pages/common.js powerBar's text and colours).
 */
export function nodePowerKeys(metrics) {
  return perGpuList(powerKeyCache, metrics, powerKeys);
}

function powerKeys(gs) {
  const sum = {};
  for (let i = 0; i < gs.length; i++) {
    const g = gs[i];
    if (typeof g.powerWatts !== 'number' || !isFinite(g.powerWatts)) continue;
    const e = sum[g.nodeName] || (sum[g.nodeName] = [0, 0]);
    e[0] += g.powerWatts;
    e[1] += typeof g.powerCapWatts === 'number' && isFinite(g.powerCapWatts) ? g.powerCapWatts : 0;
  }
  const byNode = {};
  const bars = {};
  const names = Object.keys(sum).sort();
  for (let i = 0; i < names.length; i++) {
    const w = Math.round(sum[names[i]][0]);
    const c = Math.round(sum[names[i]][1]);
    byNode[names[i]] = w + '|' + c;
    bars[names[i]] = powerBarFacts(w, c > 0 ? c : null);
  }
  return { byNode: byNode, sig: names.map(function (n) { return n + '=' + byNode[n]; }).join(','), bars: bars };
}

/** The power bar's numbers and text: "X W / Y W (Z%)", coloured at 70 / 90 % (reference PowerBar, MetricsPage.tsx:50-89). */
export function powerBarFacts(watts, capWatts) {
  const hasCap = capWatts !== null && capWatts > 0;
  const p = hasCap ? Math.min(100, pct(watts, capWatts)) : null;
  return {
    watts: watts,
    cap: hasCap ? capWatts : null,
    pct: p,
    color: p === null ? BAR_COLORS.ok : pctToColor(p),
    text: formatWatts(watts) + (hasCap ? ' / ' + formatWatts(capWatts) + ' (' + formatPercent(watts, capWatts) + ')' : ''),
  };
}

/**
 * The hottest GPU of each node (junction °C, whole degrees), its throttle
 * limit (the source's, else the MI355X's) and the status level its UNROUNDED
 * reading has against that limit (pages/common.js tempCell): "temp|limit|level"
 * per node, so the GPU Nodes summary rebuilds only when a shown value
 * changes, and a GPU at 99.6 °C under a 100 °C limit is a warning there as on
 * the Metrics page, not an error after rounding.
 */
export function nodeTempKeys(metrics) {
  return perGpuList(tempKeyCache, metrics, tempKeys);
}

function tempKeys(gs) {
  const hot = {};
  for (let i = 0; i < gs.length; i++) {
    const g = gs[i];
    if (typeof g.tempC !== 'number' || !isFinite(g.tempC)) continue;
    const lim = typeof g.tempSlowdownC === 'number' && g.tempSlowdownC > 0 ? g.tempSlowdownC : MI355X.junctionSlowdownC;
    const e = hot[g.nodeName];
    if (!e || g.tempC > e[0]) hot[g.nodeName] = [g.tempC, lim];
  }
  const byNode = {};
  const cells = {};
  const names = Object.keys(hot).sort();
  for (let i = 0; i < names.length; i++) {
    const t = hot[names[i]][0];
    const lim = hot[names[i]][1];
    const level = t >= lim ? 'error' : t >= lim - 10 ? 'warning' : 'ok';
    byNode[names[i]] = Math.round(t) + '|' + Math.round(lim) + '|' + level;
    const text = Math.round(t) + ' °C';
    cells[names[i]] = { level: level, text: level === 'error' ? text + ' (throttling at ' + Math.round(lim) + ' °C)' : text };
  }
  return { byNode: byNode, sig: names.map(function (n) { return n + '=' + byNode[n]; }).join(','), cells: cells };
}

let lastOwners = {};

function sameOwners(a, b) {
  if (!a || !b || a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) {
    if (a[i].gpu !== b[i].gpu || a[i].pod !== b[i].pod || a[i].namespace !== b[i].namespace) return false;
  }
  return true;
}

const NO_OWNERS = Object.freeze({});

/**
 * node → [{gpu, pod, namespace}] from exporter pod labels, once per GPU list;
 * a node's array keeps its identity while its owners are unchanged
 * (telemetry values change every scrape, GPU ownership rarely).
 */
export function ownersByNode(metrics) {
  if (!metrics || !metrics.gpus) return NO_OWNERS;
  if (ownersCache.has(metrics.gpus)) return ownersCache.get(metrics.gpus);
  const out = {};
  for (let i = 0; i < metrics.gpus.length; i++) {
    const g = metrics.gpus[i];
    if (!g.pod) continue;
    if (!out[g.nodeName]) out[g.nodeName] = [];
    out[g.nodeName].push({ gpu: g.gpu, pod: g.pod, namespace: g.namespace });
  }
  for (const k in out) {
    if (sameOwners(lastOwners[k], out[k])) out[k] = lastOwners[k];
  }
  lastOwners = out;
  ownersCache.set(metrics.gpus, out);
  return out;
}

let lastAssign = {};

function sameAssign(a, b) {
  if (!a || !b || a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) if (a[i] !== b[i]) return false;
  return true;
}

/**
 * "namespace/pod" → the GPUs the exporter attributes to that pod (its
 * pod/namespace labels), as GPU objects of the snapshot. Kubernetes itself
 * does not say which device a pod got; this is the exporter's view. A pod's
 * array keeps its identity while its GPUs are the same objects (the metrics
 * client's structural sharing), and the whole map keeps its identity while
 * no pod's list changed.
 */
export function podGpuAssignments(metrics) {
  if (!metrics || !metrics.gpus) return {};
  if (assignCache.has(metrics.gpus)) return assignCache.get(metrics.gpus);
  const out = {};
  for (let i = 0; i < metrics.gpus.length; i++) {
    const g = metrics.gpus[i];
    if (!g.pod) continue;
    const k = (g.namespace || '') + '/' + g.pod;
    if (!out[k]) out[k] = [];
    out[k].push(g);
  }
  let same = Object.keys(out).length === Object.keys(lastAssign).length;
  for (const k in out) {
    if (sameAssign(lastAssign[k], out[k])) out[k] = lastAssign[k];
    else same = false;
  }
  const res = same ? lastAssign : out;
  lastAssign = res;
  assignCache.set(metrics.gpus, res);
  return res;
}

/** A pod's summed GPU power ("2393.4 W"), or "—" without a reading. */
export function podPowerText(gs) {
  if (!gs || !gs.length) return '—';
  let w = 0;
  let any = false;
  for (let i = 0; i < gs.length; i++) {
    if (typeof gs[i].powerWatts === 'number' && isFinite(gs[i].powerWatts)) {
      w += gs[i].powerWatts;
      any = true;
    }
  }
  return any ? formatWatts(w) : '—';
}

function assignedText(gs) {
  const byNode = {};
  const order = [];
  for (let i = 0; i < gs.length; i++) {
    if (!byNode[gs[i].nodeName]) {
      byNode[gs[i].nodeName] = [];
      order.push(gs[i].nodeName);
    }
    byNode[gs[i].nodeName].push(gs[i].gpu);
  }
  return order.map(function (n) { return n + ': GPU ' + byNode[n].join(', '); }).join('; ');
}

const NO_ASSIGNMENT = Object.freeze({ assigned: '—', power: '—' });

/**
 * A pod's GPUs as its GPU Pods row says them: {assigned: "n1: GPU 2, 3",
 * power: "2393.4 W"}, once per assignment array (podGpuAssignments keeps an
 * unchanged pod's array).
 */
export function assignmentTexts(gs) {
  if (!gs || !gs.length) return NO_ASSIGNMENT;
  let t = textCache.get(gs);
  if (!t) {
    t = { assigned: assignedText(gs), power: podPowerText(gs) };
    textCache.set(gs, t);
  }
  return t;
}

/** `o` is an object with an own key (answered once per map: a link map is a 56-key dictionary, slow to enumerate). */
export function nonEmptyMap(o) {
  if (!o || typeof o !== 'object') return false;
  if (nonEmpty.has(o)) return nonEmpty.get(o);
  let any = false;
  for (const k in o) {
    if (Object.prototype.hasOwnProperty.call(o, k)) {
      any = true;
      break;
    }
  }
  nonEmpty.set(o, any);
  return any;
}

/**
 * Derive a snapshot's per-node summaries now (metrics.js, when the snapshot
 * arrives): power, temperature and owner keys, and the link facts of every
 * node's maps for as many GPUs as the snapshot reports on that node.
 * Returns the snapshot.
 */
export function primeSnapshot(m) {
  if (!m || typeof m !== 'object' || !Array.isArray(m.gpus)) return m;
  nodePowerKeys(m);
  nodeTempKeys(m);
  ownersByNode(m);
  const assign = podGpuAssignments(m);
  for (const k in assign) assignmentTexts(assign[k]);
  const xgmi = m.xgmi || {};
  const links = m.links || {};
  const nodes = {};
  for (const k in xgmi) nodes[k] = true;
  for (const k in links) nodes[k] = true;
  let gpusOf = null;
  for (const name in nodes) {
    if (!gpusOf) {
      gpusOf = {};
      for (let i = 0; i < m.gpus.length; i++) {
        const g = m.gpus[i];
        const s = gpusOf[g.nodeName] || (gpusOf[g.nodeName] = {});
        s[g.gpu] = true;
      }
    }
    const n = gpusOf[name] ? Object.keys(gpusOf[name]).length : 0;
    const measured = xgmi[name] && typeof xgmi[name] === 'object' ? xgmi[name] : null;
    const probed = nonEmptyMap(links[name]) ? links[name] : null;
    if (n > 1 && (measured || probed)) linkFacts(n, measured, probed);
  }
  return m;
}
