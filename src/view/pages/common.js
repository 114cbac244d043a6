/**
 * What every page view-model shares: the section memo and per-object row
 * caches (identity-keyed, age-aware: ./ir.js createMemo), chunked table rows,
 * the refresh button and error box, and the bars and cells several pages
 * draw (allocation, power, HBM, temperature, RAS).
 */

import { getPodRestarts, isPodReady } from '../../api/amdPods.js';
import {
  formatAge,
  formatBytes,
  get,
  MI355X,
  nextAgeChange,
  pct,
  pctToColor,
} from '../../api/k8sCore.js';
import { derivedCache, resetDerivedCaches } from '../../api/derivedCache.js';
import { powerBarFacts } from '../../api/nodeSummaries.js';
import { bar, createMemo, createObjectCache, kv, noteExpiry, row, section, status } from '../ir.js';

export const BRAND = 'AMD GPU';

/**
 * Section-level memo shared by all views. Deps are the snapshot fields a
 * section reads plus the age clock (ages are shown with 1 s resolution), so a
 * refresh that returns unchanged Kubernetes objects reuses the section IR.
 */
// One slot per section: node cards, node details, metrics nodes and pod details
// of a few hundred nodes / thousands of pods fit without LRU churn.
export const memo = createMemo(8192);

// Table rows per Kubernetes object, one cache per table (pods, nodes): an
// event rebuilds the changed object's row only.
export const ovPluginRows = createObjectCache();
export const dpPluginRows = createObjectCache();
export const nodeSummaryRows = createObjectCache();
export const podRows = createObjectCache();
export const pendingRows = createObjectCache();
const ROW_CACHES = [ovPluginRows, dpPluginRows, nodeSummaryRows, podRows, pendingRows];

export const podDetailCache = derivedCache();

/**
 * Progressive loading: what has settled. A page waits only for the lists it
 * draws — Metrics for the node list and its own query, GPU Nodes for the
 * node list (its pod-derived cells fill in when the pods arrive), Overview
 * for the nodes and the DeviceConfigs (a loader where the pods go), Device
 * Plugins for the DeviceConfigs — instead of the reference's single
 * `loading` that holds every page until the all-namespaces pod list is in
 * (IntelGpuDataContext.tsx:214). Contexts without the per-list fields (hand
 * made in tests, older snapshots) fall back to `loading`.
 */
export function nodesPending(ctx) {
  return ctx.nodesLoading !== undefined ? !!ctx.nodesLoading : !!ctx.loading;
}
export function podsPending(ctx) {
  return ctx.podsLoading !== undefined ? !!ctx.podsLoading : !!ctx.loading;
}
export function crdPending(ctx) {
  return ctx.crdLoading !== undefined ? !!ctx.crdLoading : !!ctx.loading;
}
/** The operator pods: from the watched pod list, or from the plugin-pod requests where no pod list is mounted. */
export function pluginPodsPending(ctx) {
  return ctx.pluginPodsLoading !== undefined ? !!ctx.pluginPodsLoading : podsPending(ctx);
}

/** Text of a cell whose value needs the pod list while it is still loading. */
export const PODS_LOADING = 'Loading…';

/** Rows per memo slot in the large tables (see chunkedRows). */
const ROW_CHUNK = 64;

/**
 * `objs.map(build)` for a large table, memoised in chunks of ROW_CHUNK
 * objects keyed on their identities: after a watch event that replaced one
 * pod in a 5000-row table, 78 chunks are identity-compared and one is
 * rebuilt (its other rows come from `rowCacheOf`'s per-object cache).
 */
export function chunkedRows(name, objs, deps, build, now, depsOf) {
  const out = [];
  for (let c = 0; c < objs.length; c += ROW_CHUNK) {
    const part = objs.slice(c, c + ROW_CHUNK);
    const key = part.concat(deps);
    // Per-object inputs besides the object itself (its stats, its pods).
    if (depsOf) {
      for (let i = 0; i < part.length; i++) {
        const d = depsOf(part[i]);
        for (let k = 0; k < d.length; k++) key.push(d[k]);
      }
    }
    const rows = memo(name + ':' + c / ROW_CHUNK, key, function () { return part.map(build); }, now);
    for (let i = 0; i < rows.length; i++) out.push(rows[i]);
  }
  return out;
}

/** `objs.filter(pred)` memoised in chunks the same way (pred depends on the object only). */
export function chunkedFilter(name, objs, pred) {
  const out = [];
  for (let c = 0; c < objs.length; c += ROW_CHUNK) {
    const part = objs.slice(c, c + ROW_CHUNK);
    const kept = memo(name + ':' + c / ROW_CHUNK, part, function () { return part.filter(pred); });
    for (let i = 0; i < kept.length; i++) out.push(kept[i]);
  }
  return out;
}

/** formatAge, noting when the label changes (the enclosing memo holds until then). */
export function ageText(timestamp, now) {
  noteExpiry(nextAgeChange(timestamp, now));
  return formatAge(timestamp, now);
}

/** Seconds → "30 min" / "1 h" / "6 h" / "90 s" for section titles. */
export function formatWindow(sec) {
  if (sec >= 3600 && sec % 3600 === 0) return sec / 3600 + ' h';
  if (sec >= 60 && sec % 60 === 0) return sec / 60 + ' min';
  return sec + ' s';
}

/** Drop memoised sections and the first-use derived caches (derivedCache.js): tests, a cluster switch, a cold mount. */
export function clearViewMemo() {
  memo.clear();
  for (let i = 0; i < ROW_CACHES.length; i++) ROW_CACHES[i].clear();
  resetDerivedCaches();
}

let timeFormat = null;

/**
 * `new Date(t).toLocaleTimeString()` (the reference's "Last Fetched",
 * MetricsPage.tsx:336-338) through one cached formatter with the same
 * options: the method builds a formatter per call, ≈30 µs on Node.
 */
export function localTimeText(t) {
  if (!timeFormat) {
    timeFormat = typeof Intl === 'object' && Intl.DateTimeFormat
      ? new Intl.DateTimeFormat(undefined, { hour: 'numeric', minute: 'numeric', second: 'numeric' })
      : { format: function (d) { return d.toLocaleTimeString(); } };
  }
  return timeFormat.format(new Date(t));
}

export function nowOf(opts) {
  return opts && typeof opts.now === 'number' ? opts.now : Date.now();
}

export function refreshButton(ariaLabel, busy) {
  return { label: busy ? 'Refreshing…' : 'Refresh', ariaLabel: ariaLabel, disabled: !!busy };
}

export function errorSection(err) {
  return section('Error', [kv([row('Status', status('error', err))])]);
}

/** Inline allocation bar (reference NodesPage.tsx:35-63; 70/90 thresholds). */
export function allocationBar(used, allocatable) {
  if (!(allocatable > 0)) return '—';
  const p = Math.min(100, pct(used, allocatable));
  return bar(used, allocatable, p, pctToColor(p), used + '/' + allocatable + ' (' + p + '%)');
}

export function podName(p) {
  return p.metadata.name;
}

export function podNs(p) {
  return p.metadata.namespace || '—';
}

export function podNode(p) {
  return get(p, ['spec', 'nodeName'], '—');
}

export function readyLabel(p) {
  const r = isPodReady(p);
  return status(r ? 'success' : 'warning', r ? 'Ready' : get(p, ['status', 'phase'], 'Unknown'));
}

export function restartsCell(p) {
  const n = getPodRestarts(p);
  return n > 0 ? status('warning', n) : String(n);
}

export const NO_PODS = Object.freeze([]);

/** Mean value per node of a series map (node → [[t, v]]); nodes without samples are left out. */
export function seriesMeans(byNode) {
  const out = {};
  for (const n in byNode || {}) {
    const pts = byNode[n] || [];
    let sum = 0;
    let k = 0;
    for (let i = 0; i < pts.length; i++) {
      if (typeof pts[i][1] === 'number' && isFinite(pts[i][1])) {
        sum += pts[i][1];
        k++;
      }
    }
    if (k) out[n] = sum / k;
  }
  return out;
}

/** Power bar: "X W / Y W (Z%)" with 70/90 colouring (reference PowerBar, MetricsPage.tsx:50-89). */
export function powerBar(watts, capWatts) {
  const f = powerBarFacts(watts, capWatts);
  return bar(f.watts, f.cap, f.pct, f.color, f.text);
}

export function hbmBar(used, total) {
  if (used === null) return '—';
  if (total === null || !(total > 0)) return formatBytes(used);
  const p = Math.min(100, pct(used, total));
  return bar(used, total, p, pctToColor(p), formatBytes(used) + ' / ' + formatBytes(total) + ' (' + p + '%)');
}

export function pctText(v) {
  return v === null ? '—' : Math.round(v) + '%';
}

/**
 * Junction temperature, coloured against the GPU's throttle threshold
 * (exporter-reported, else the MI355X's 100 °C): warning within 10 °C of
 * it, error at or above it.
 */
export function tempCell(g) {
  if (g.tempC === null || g.tempC === undefined) return '—';
  const limit = g.tempSlowdownC > 0 ? g.tempSlowdownC : MI355X.junctionSlowdownC;
  const text = Math.round(g.tempC) + ' °C';
  if (g.tempC >= limit) return status('error', text + ' (throttling at ' + Math.round(limit) + ' °C)');
  if (g.tempC >= limit - 10) return status('warning', text);
  return text;
}

/**
 * RAS error counts of one GPU (or cluster totals): uncorrected errors are an
 * error (the driver may already have retired HBM pages or poisoned data),
 * corrected ones a warning, none "OK". '—' when the source reports no RAS
 * counters (node-exporter).
 */
export function eccCell(g) {
  if (g.eccUncorrectable === null || g.eccUncorrectable === undefined) return '—';
  const ce = g.eccCorrectable || 0;
  if (g.eccUncorrectable > 0) {
    return status('error', g.eccUncorrectable + ' uncorrected' + (ce > 0 ? ', ' + ce + ' corrected' : ''));
  }
  if (ce > 0) return status('warning', ce + ' corrected');
  return 'OK';
}
