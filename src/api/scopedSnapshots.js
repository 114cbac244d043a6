/**
 * Telemetry of the GPU nodes a paged view shows (ADR 009): GPU Nodes and
 * Metrics ask for ONE page of nodes — by name (`hostname=~`), by the
 * size-guarded "whole cluster if it is one page" query while the node list
 * loads, or ranked by power (Prometheus picks the page) — plus, for the
 * Metrics summary, the cluster totals as server-side aggregates. The bytes
 * moved follow the page, not the cluster.
 *
 * While the session does not know which exporter feeds this Prometheus, the
 * same request carries the source probe (promql.js sourceProbe): its answer
 * says exporter, node-exporter (whose GPU series come along on a small
 * cluster) or no GPU telemetry at all, so a cluster without exporter series
 * costs one wave, not a second cluster-wide query.
 *
 * Reference analog: the Metrics page fetched every chip of the cluster on
 * every refresh (src/api/metrics.ts:96-155, MetricsPage.tsx:348-350).
 */

import { SERIES, SMALL_CLUSTER_NODES, SMALL_HWMON_GPUS, STALE_FAILURES } from './series.js';
import {
  exporterQuery,
  gpuNodeCount,
  hwmonGpuCount,
  nodeExporterProjected,
  nodeExporterScopedQuery,
  nodeExporterSummaryQuery,
  rankedClusterQuery,
  rankedHwQuery,
  sizeGuard,
  sizeRow,
  smallClusterQuery,
  sourceProbe,
  summaryQuery,
} from './promql.js';
import {
  applyStatics,
  gpuKey,
  isRow,
  joinExporterResults,
  joinNodeExporterResults,
  num,
  sameValue,
  shareGpus,
  hwTotalsFromRows,
  HW_TOTAL_TAGS,
  shareMap,
  sizeFromRows,
  staticsOf,
  summarizeMetrics,
  totalsFromRows,
  zeroTotals,
} from './telemetry.js';
import { UNREACHABLE, staleOrNull } from './promClient.js';
import { NOT_SCOPED } from './clusterSnapshots.js';

/** `agg` tags of size / probe rows and of node-exporter totals (not exporter cluster totals). */
const SIZE_TAGS = { gpu_nodes: true, hwmon: true, rank: true, ranked: true };
for (let i = 0; i < HW_TOTAL_TAGS.length; i++) SIZE_TAGS[HW_TOTAL_TAGS[i]] = true;

function totalsOf(rows) {
  return totalsFromRows(rows.__agg.filter(function (r) { return !SIZE_TAGS[r.metric.agg]; }));
}

/** Scoped answers kept (stale fallbacks, structural sharing), most recent first. */
const SCOPED_KEYS = 16;

/**
 * @param {PromClient} client
 * @param {{source: ('amd-exporter'|'node-exporter'|null), lean: boolean}} state
 * @param {ClusterSnapshots} snaps
 */
export function createScopedSnapshots(client, state, snaps) {
  // node → {at, statics: gpuKey → static fields, links}: static series of the
  // nodes a paged view has shown, re-read per node every ttl.
  let scopeStatic = {};
  // scoped key → {last, failures, cutOf}; the most recent SCOPED_KEYS kept.
  let scopedState = new Map();

  client.onInvalidate(function () {
    scopeStatic = {};
    scopedState = new Map();
  });

  function entry(key) {
    let e = scopedState.get(key);
    if (e) scopedState.delete(key); // most recently used last
    else e = { last: null, failures: 0, cutOf: null };
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
    const now = client.now();
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

  function needsStatic(scope) {
    const now = client.now();
    for (let i = 0; i < scope.length; i++) {
      const e = scopeStatic[scope[i]];
      if (!e || now - e.at >= client.ttl) return true;
    }
    return false;
  }

  function result(st, base, q, j, scope, totals, v, sized) {
    const prev = st.last;
    st.last = {
      source: state.source,
      view: v,
      gpus: prev ? shareGpus(prev.gpus, j.gpus) : j.gpus,
      xgmi: prev ? shareMap(prev.xgmi, j.xgmi) : j.xgmi,
      links: prev ? shareMap(prev.links, j.links || {}) : j.links || {},
      fetchedAt: client.fetchedAt(),
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
   * `scope`: Kubernetes node names (= exporter `hostname`); `summary`: add
   * the cluster totals; `small`: the page may be the whole cluster
   * (promql.js smallClusterQuery) — every GPU when at most
   * SMALL_CLUSTER_NODES nodes report, else `scope`'s; the answer says which
   * (`small.exceeded`). A node-exporter source (no `hostname` label) is
   * served from the cluster-wide snapshot cut to the scope.
   */
  function scoped(v, scope, summary, key, small) {
    const st = entry(key);
    if (state.source === 'node-exporter') return hwScoped(st, v, scope, summary, key, small);
    return client.withPrometheus(function (base) {
      // Nothing cached yet for a small-cluster fetch before the node list: statics too.
      const withStatic = small && scope.length === 0 ? true : scope.length > 0 && needsStatic(scope);
      const probing = state.source === null;
      const parts = [];
      if (small) parts.push(smallClusterQuery(withStatic, v, scope));
      else if (scope.length) parts.push(exporterQuery(withStatic, true, v, scope));
      if (summary) parts.push(summaryQuery());
      // smallClusterQuery already carries the gpu_nodes row.
      if (probing && parts.length) {
        parts.push(sourceProbe(!small));
        // node-exporter's page and totals too, where no exporter reports (a
        // few instant aggregates, cheap next to the range series): a
        // node-exporter cluster of any size is told apart AND served here.
        const hw = [];
        if (scope.length) hw.push(nodeExporterScopedQuery(scope));
        if (summary) hw.push(nodeExporterSummaryQuery());
        if (hw.length) parts.push('(' + hw.join(' or ') + ') unless on() (' + gpuNodeCount() + ')');
      }
      if (!parts.length) return Promise.resolve(result(st, base, null, { gpus: [], xgmi: {}, links: {} }, scope, undefined, v));
      const q = parts.join(' or ');
      return client.combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const rows = res.rows;
        const j = joinExporterResults(rows);
        // Summary asked and no aggregate row: nothing reports (zero totals, not "unknown").
        const totals = summary ? totalsOf(rows) || zeroTotals() : undefined;
        const reporting = sizeFromRows(rows.__agg, 'gpu_nodes');
        if (j.gpus.length > 0 || (!!totals && totals.gpus > 0) || reporting > 0) {
          state.source = 'amd-exporter';
        } else if (probing && sizeFromRows(rows.__agg, 'hwmon') > 0) {
          // node-exporter's amdgpu hwmon feeds this Prometheus: every GPU's
          // series came along on a small cluster, the page's and the totals
          // on any (one wave).
          state.source = 'node-exporter';
          return hwAnswer(st, base, q, rows, v, scope, summary, small, joinNodeExporterResults(rows).gpus.length > 0);
        }
        // (No exporter and no amdgpu hwmon: no GPU telemetry — this answer stands.)
        scopeStatics(j, scope, withStatic);
        const sized = small ? { count: reporting, limit: SMALL_CLUSTER_NODES, exceeded: reporting > SMALL_CLUSTER_NODES } : undefined;
        return result(st, base, q, j, scope, totals, v, sized);
      });
    }, function () {
      return staleOrNull(st, STALE_FAILURES, client.invalidate);
    }).then(function (r) {
      return r === NOT_SCOPED ? snaps.cluster(v).then(function (m) { return cut(m, scope, summary, key, small); }) : r;
    });
  }

  /**
   * The page's telemetry on a node-exporter source: its nodes' series through
   * node_uname_info (promql.js nodeExporterScopedQuery) and the totals as
   * server-side aggregates (nodeExporterSummaryQuery) — O(page), like the
   * exporter's `hostname=~` path. `small` keeps its meaning: every GPU while
   * at most SMALL_HWMON_GPUS amdgpu chips report, else `scope`'s.
   */
  function hwScoped(st, v, scope, summary, key, small) {
    return client.withPrometheus(function (base) {
      const hw = hwmonGpuCount();
      const parts = [];
      if (small) {
        parts.push(sizeGuard(nodeExporterProjected(), true, hw, SMALL_HWMON_GPUS));
        if (scope.length) parts.push(sizeGuard(nodeExporterScopedQuery(scope), false, hw, SMALL_HWMON_GPUS));
      } else if (scope.length) parts.push(nodeExporterScopedQuery(scope));
      parts.push(sizeRow(hw, 'hwmon'));
      if (summary) parts.push(nodeExporterSummaryQuery());
      const q = parts.join(' or ');
      return client.combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        return hwAnswer(st, base, q, res.rows, v, scope, summary, small);
      });
    }, function () {
      return staleOrNull(st, STALE_FAILURES, client.invalidate);
    }).then(function (r) {
      return r === NOT_SCOPED ? snaps.cluster(v).then(function (m) { return cut(m, scope, summary, key, small); }) : r;
    });
  }

  /**
   * A node-exporter answer (hwScoped, or the first query's probe) as the
   * page's snapshot. NOT_SCOPED when the cluster reports amdgpu chips but no
   * node_uname_info names a node of the page: node-exporter's `nodename` is
   * not the Kubernetes node name there, so the page is cut from the
   * cluster-wide snapshot instead (its join also tries `node` and `instance`).
   */
  function hwAnswer(st, base, q, rows, v, scope, summary, small, everyGpu) {
    st.failures = 0;
    const chips = sizeFromRows(rows.__agg, 'hwmon');
    const whole = !!small && chips <= SMALL_HWMON_GPUS;
    const j = joinNodeExporterResults(rows);
    // `everyGpu`: the rows hold every GPU (the probe on a small cluster): the
    // totals can be summed here when no aggregate rows came along.
    const allTotals = everyGpu && summary ? totalsOfAll(j) : null;
    if (!whole) {
      const inScope = {};
      for (let i = 0; i < scope.length; i++) inScope[scope[i]] = true;
      j.gpus = j.gpus.filter(function (g) { return inScope[g.nodeName] === true; });
      const un = rows[SERIES.nodeExporter.uname] || [];
      const named = un.some(function (r) { return isRow(r) && inScope[r.metric.nodename] === true; });
      if (scope.length && !j.gpus.length && !named && chips > 0) return NOT_SCOPED;
    }
    const totals = summary ? hwTotalsFromRows(rows.__agg) || allTotals || zeroTotals() : undefined;
    const sized = small ? { count: chips, limit: SMALL_HWMON_GPUS, exceeded: !whole } : undefined;
    return result(st, base, q, j, scope, totals, v, sized);
  }

  /** summarizeMetrics of a join holding every GPU, plus the nodes reporting. */
  function totalsOfAll(j) {
    const seen = {};
    let nodes = 0;
    for (let i = 0; i < j.gpus.length; i++) {
      if (!seen[j.gpus[i].nodeName]) {
        seen[j.gpus[i].nodeName] = true;
        nodes++;
      }
    }
    return Object.assign(summarizeMetrics(j), { nodes: nodes });
  }

  /**
   * One page of GPU nodes ranked by total GPU power (rankedClusterQuery):
   * `scope` is the page's nodes in rank order, `rank` the page, the ranked
   * count and each node's watts. Static series ride along (the page's names
   * are not known before the answer). Stale / null handling as scoped.
   */
  function ranked(v, rank, summary, key) {
    const st = entry(key);
    if (state.source === 'node-exporter') return hwRanked(st, v, rank, summary);
    return client.withPrometheus(function (base) {
      // The page's names come with the answer: ask for the static series
      // while the nodes last shown (most likely shown again) lack a copy.
      const prev = st.last && st.last.scope;
      const withStatic = !prev || prev.length === 0 || needsStatic(prev);
      const q = rankedClusterQuery(v, rank, withStatic) + (summary ? ' or ' + summaryQuery() : '');
      return client.combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const rows = res.rows;
        const j = joinExporterResults(rows);
        const ro = rankOrder(rows);
        const names = ro.names;
        const watts = ro.watts;
        scopeStatics(j, names, withStatic);
        const count = sizeFromRows(rows.__agg, 'ranked');
        const totals = summary ? totalsOf(rows) || zeroTotals() : undefined;
        if (j.gpus.length > 0 || count > 0) state.source = 'amd-exporter';
        // Nothing ranked and no exporter seen: maybe node-exporter feeds this
        // Prometheus (no hostname label to rank by) — the cluster-wide
        // snapshot decides, and a node-exporter source is then ranked its way.
        else if (state.source !== 'amd-exporter') return NOT_SCOPED;
        const out = result(st, base, q, j, names, totals, v, undefined);
        out.rank = { by: rank.by, page: rank.page, per: rank.per, filter: rank.filter, count: count, watts: watts };
        return out;
      });
    }, function () {
      return staleOrNull(st, STALE_FAILURES, client.invalidate);
    }).then(function (r) {
      if (r !== NOT_SCOPED) return r;
      return snaps.cluster(v).then(function (m) {
        return m && state.source === 'node-exporter' ? hwRanked(st, v, rank, summary) : m;
      });
    });
  }

  /** The `agg="rank"` rows of a ranked answer: node names highest power first, and each node's watts. */
  function rankOrder(rows) {
    const order = [];
    const watts = {};
    for (let i = 0; i < rows.__agg.length; i++) {
      const r = rows.__agg[i];
      if (!isRow(r) || r.metric.agg !== 'rank' || typeof r.metric.hostname !== 'string') continue;
      const w = num(r.value[1]);
      order.push([r.metric.hostname, w === null ? -Infinity : w]);
      watts[r.metric.hostname] = w;
    }
    order.sort(function (a, b) { return b[1] - a[1] || (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0); });
    return { names: order.map(function (x) { return x[0]; }), watts: watts };
  }

  /**
   * A page of GPU nodes in power order on a node-exporter source (promql.js
   * rankedHwQuery): Prometheus sums each node's amdgpu chips through
   * node_uname_info and ranks them; the page's series, the ranking and the
   * count come in one request, the totals with it.
   */
  function hwRanked(st, v, rank, summary) {
    return client.withPrometheus(function (base) {
      const q = rankedHwQuery(rank) + (summary ? ' or ' + nodeExporterSummaryQuery() : '');
      return client.combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const rows = res.rows;
        const ro = rankOrder(rows);
        const inRank = {};
        for (let i = 0; i < ro.names.length; i++) inRank[ro.names[i]] = true;
        const j = joinNodeExporterResults(rows);
        j.gpus = j.gpus.filter(function (g) { return inRank[g.nodeName] === true; });
        const totals = summary ? hwTotalsFromRows(rows.__agg) || zeroTotals() : undefined;
        const out = result(st, base, q, j, ro.names, totals, v, undefined);
        out.rank = { by: rank.by, page: rank.page, per: rank.per, filter: rank.filter,
          count: sizeFromRows(rows.__agg, 'ranked'), watts: ro.watts };
        return out;
      });
    }, function () {
      return staleOrNull(st, STALE_FAILURES, client.invalidate);
    });
  }

  /**
   * A cluster-wide snapshot cut to `scope` (node-exporter source), totals
   * summed here. A small-cluster fetch (`small`) keeps its meaning: every GPU
   * when at most SMALL_CLUSTER_NODES nodes report — the page may be asked
   * before the node list names it, and its key then stays put — else
   * `scope`'s, flagged `exceeded` so the caller's key follows the names.
   */
  function cut(m, scope, summary, key, small) {
    if (!m) return null;
    const st = entry(key);
    if (st.cutOf === m && st.last) return st.last;
    const reporting = {};
    let count = 0;
    for (let i = 0; i < m.gpus.length; i++) {
      if (!reporting[m.gpus[i].nodeName]) {
        reporting[m.gpus[i].nodeName] = true;
        count++;
      }
    }
    const whole = !!small && count <= SMALL_CLUSTER_NODES;
    const inScope = whole ? reporting : {};
    if (!whole) for (let i = 0; i < scope.length; i++) inScope[scope[i]] = true;
    const names = whole ? Object.keys(reporting) : scope;
    const xgmi = {};
    const links = {};
    for (let i = 0; i < names.length; i++) {
      if (m.xgmi && m.xgmi[names[i]]) xgmi[names[i]] = m.xgmi[names[i]];
      if (m.links && m.links[names[i]]) links[names[i]] = m.links[names[i]];
    }
    const totals = summary ? Object.assign(summarizeMetrics(m), { nodes: count }) : undefined;
    const out = Object.assign({}, m, {
      gpus: m.gpus.filter(function (g) { return inScope[g.nodeName] === true; }),
      xgmi: xgmi,
      links: links,
      scope: scope,
      totals: totals,
      small: small ? { count: count, limit: SMALL_CLUSTER_NODES, exceeded: !whole } : undefined,
    });
    st.cutOf = m;
    st.last = out;
    return out;
  }

  return { scoped: scoped, ranked: ranked };
}
