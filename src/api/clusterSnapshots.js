/**
 * Cluster-wide and per-node telemetry snapshots.
 *
 *   * `cluster(view)` — every GPU's live series of a METRIC_VIEWS view in ONE
 *     query (the terminal client, the screenshots, the fallback of the paged
 *     views on a node-exporter source). The first query of a session reads
 *     both exporters (promql.js mergedQuery); later ones only the one that
 *     answered. Static series (power cap, HBM size, throttle threshold, link
 *     topology) ride along once per discovery TTL and are kept.
 *   * `node(name)` — one node's GPUs for the native Node / Pod detail pages:
 *     a `hostname`-scoped query, O(GPUs per node) bytes whatever the cluster
 *     size; the cluster-wide snapshot cut to the node when the scoped query
 *     finds nothing (node-exporter carries `instance`, not `hostname`).
 *
 * Reference analog: fetchGpuMetrics (src/api/metrics.ts:96-155): discovery
 * then four instant queries on every fetch, power keyed by PCI chip only.
 */

import { SERIES, STALE_FAILURES } from './series.js';
import {
  exporterNodeQuery,
  exporterQuery,
  gpuNodeCount,
  hwmonGpuCount,
  mergedQuery,
  nodeExporterQuery,
  nodeExporterScopedQuery,
  sizeRow,
} from './promql.js';
import {
  applyStatics,
  isRow,
  joinExporterResults,
  joinNodeExporterResults,
  keyedByHostname,
  nodeSlice,
  shareGpus,
  shareMap,
  sizeFromRows,
  staticsOf,
} from './telemetry.js';
import { UNREACHABLE, staleOrNull } from './promClient.js';

/** Marker: a scoped query found no exporter GPU in its scope (ask cluster-wide). */
export const NOT_SCOPED = Object.freeze({ notScoped: true });

/**
 * @param {PromClient} client
 * @param {{source: ('amd-exporter'|'node-exporter'|null), lean: boolean}} state  shared by every fetcher
 */
export function createClusterSnapshots(client, state) {
  let links = null; // measured xGMI link topology per node (static), refreshed every ttl with `statics`
  let statics = null; // static per-GPU fields (STATIC_GPU_FIELDS), fetched with the topology
  let linksAt = 0;
  let lastBy = {}; // view → previous snapshot, for structural sharing and stale fallbacks
  let failuresBy = {}; // view → consecutive failed fetches against the cached service
  // Per-node snapshots for the detail pages: node → {last, links, statics, staticAt, failures}.
  let nodeStates = {};

  client.onInvalidate(function () {
    links = null;
    statics = null;
    lastBy = {};
    failuresBy = {};
    nodeStates = {};
  });

  function cluster(v) {
    return client.shared('gpus|' + v, function () {
      return client.withPrometheus(function (base) { return snapshotFrom(base, v); }, function () {
        const st = { last: lastBy[v] || null, failures: failuresBy[v] || 0 };
        const r = staleOrNull(st, STALE_FAILURES, client.invalidate);
        failuresBy[v] = st.failures;
        return r;
      });
    });
  }

  /**
   * The cluster-wide answer of `rows` (a combined query result) as a snapshot
   * of `view`: joins whichever exporter answered, keeps the static series,
   * shares structure with the last snapshot of the view.
   */
  function commit(base, view, q, rows, withStatic) {
    failuresBy[view] = 0;
    let joined = { gpus: [], xgmi: {}, links: {} };
    let src = null;
    if (state.source !== 'node-exporter') {
      const j = joinExporterResults(rows);
      if (j.gpus.length) {
        joined = j;
        src = 'amd-exporter';
        if (withStatic) {
          links = j.links;
          statics = staticsOf(j.gpus);
          linksAt = client.now();
          state.lean = keyedByHostname(rows);
        } else {
          joined.links = links;
          // A GPU the static copy does not know yet (node added since):
          // fetch the static series again on the next refresh.
          if (!applyStatics(j.gpus, statics)) linksAt = -Infinity;
        }
      }
    }
    if (!src && state.source !== 'amd-exporter') {
      const j = joinNodeExporterResults(rows);
      if (j.gpus.length) {
        joined = j;
        src = 'node-exporter';
      }
    }
    const last = lastBy[view];
    const same = last && last.source === src;
    state.source = src;
    lastBy[view] = {
      source: src,
      view: view,
      gpus: same ? shareGpus(last.gpus, joined.gpus) : joined.gpus,
      xgmi: same ? shareMap(last.xgmi, joined.xgmi) : joined.xgmi,
      links: same ? shareMap(last.links, joined.links || {}) : joined.links || {},
      fetchedAt: client.fetchedAt(),
      prometheusPath: base,
      // The PromQL this snapshot came from (Metrics page "Query" row).
      query: q,
    };
    return lastBy[view];
  }

  function snapshotFrom(base, view) {
    const withStatic = links === null || client.now() - linksAt >= client.ttl;
    const q = state.source === 'amd-exporter' ? exporterQuery(withStatic, state.lean, view)
      : state.source === 'node-exporter' ? nodeExporterQuery() : mergedQuery(withStatic, view);
    return client.combined(base, q).then(function (res) {
      if (!res.ok) return UNREACHABLE;
      return commit(base, view, q, res.rows, withStatic);
    });
  }

  /**
   * Telemetry of ONE node's GPUs — what the native Node and Pod detail pages
   * show. Static series are re-read per node every discovery TTL, as in the
   * cluster-wide path. Transient failures serve the node's last snapshot
   * marked stale. Resolves to null when Prometheus is unreachable.
   */
  function node(nodeName) {
    const key = String(nodeName);
    return client.shared('node|' + key, function () { return nodeSnapshot(key); });
  }

  function nodeSnapshot(key) {
    if (!nodeStates[key]) nodeStates[key] = { last: null, links: null, statics: null, staticAt: 0, failures: 0 };
    const st = nodeStates[key];
    function clusterWide() {
      return cluster('all').then(function (m) { return m ? nodeSlice(m, key) : null; });
    }
    if (state.source === 'node-exporter') return hwNode(st, key, clusterWide);
    return client.withPrometheus(function (base) {
      const withStatic = st.links === null || client.now() - st.staticAt >= client.ttl;
      // Source not known yet (a detail page opened first): the same request
      // carries the source probe's counts and node-exporter's series of this
      // node — O(one node) either way, one wave on a cluster of either
      // exporter or of none.
      const probing = state.source === null;
      const q = exporterNodeQuery(key, withStatic) + (probing
        ? ' or ' + sizeRow(gpuNodeCount(), 'gpu_nodes') + ' or ' + sizeRow(hwmonGpuCount(), 'hwmon') +
          ' or (' + nodeExporterScopedQuery([key]) + ') unless on() (' + gpuNodeCount() + ')'
        : '');
      return client.combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        st.failures = 0;
        const j = joinExporterResults(res.rows, key);
        if (probing) {
          if (j.gpus.length || sizeFromRows(res.rows.__agg, 'gpu_nodes') > 0) state.source = 'amd-exporter';
          else if (sizeFromRows(res.rows.__agg, 'hwmon') > 0) {
            state.source = 'node-exporter';
            return hwNodeAnswer(st, key, base, res.rows);
          } else return nodeAnswer(st, key, base, { gpus: [] }, 'none'); // no GPU telemetry in this Prometheus
        }
        if (!j.gpus.length) return NOT_SCOPED;
        if (withStatic) {
          st.links = j.links;
          st.statics = staticsOf(j.gpus);
          st.staticAt = client.now();
        } else {
          j.links = st.links;
          if (!applyStatics(j.gpus, st.statics)) st.staticAt = -Infinity;
        }
        return nodeAnswer(st, key, base, j, 'amd-exporter');
      });
    }, function () {
      return staleOrNull(st, STALE_FAILURES, client.invalidate);
    }).then(function (r) { return r === NOT_SCOPED ? clusterWide() : r; });
  }

  /** One node's snapshot from its joined rows `j` ([] : no GPU telemetry at all), sharing structure with the last. */
  function nodeAnswer(st, key, base, j, source) {
    const gpus = j.gpus || [];
    const prev = st.last;
    const same = prev && prev.source === (source === 'none' ? null : source);
    st.last = {
      source: source === 'none' ? null : source,
      gpus: same ? shareGpus(prev.gpus, gpus) : gpus,
      xgmi: same ? shareMap(prev.xgmi, j.xgmi || {}) : j.xgmi || {},
      links: same ? shareMap(prev.links, j.links || {}) : j.links || {},
      fetchedAt: client.fetchedAt(),
      prometheusPath: base,
      scope: key,
    };
    return st.last;
  }

  /**
   * One node's GPUs on a node-exporter source: its series through
   * node_uname_info (promql.js nodeExporterScopedQuery), O(GPUs per node);
   * the cluster-wide snapshot cut to the node when no node_uname_info names
   * it (node-exporter's `nodename` is not the Kubernetes node name there).
   */
  function hwNode(st, key, clusterWide) {
    return client.withPrometheus(function (base) {
      const q = nodeExporterScopedQuery([key]);
      return client.combined(base, q).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        return hwNodeAnswer(st, key, base, res.rows);
      });
    }, function () {
      return staleOrNull(st, STALE_FAILURES, client.invalidate);
    }).then(function (r) { return r === NOT_SCOPED ? clusterWide() : r; });
  }

  /** hwNode's answer (or the probing node query's node-exporter rows): NOT_SCOPED when no node_uname_info names the node. */
  function hwNodeAnswer(st, key, base, rows) {
    st.failures = 0;
    const un = rows[SERIES.nodeExporter.uname] || [];
    if (!un.some(function (r) { return isRow(r) && r.metric.nodename === key; })) return NOT_SCOPED;
    const j = joinNodeExporterResults(rows);
    return nodeAnswer(st, key, base, { gpus: j.gpus.filter(function (g) { return g.nodeName === key; }) }, 'node-exporter');
  }

  return {
    cluster: cluster,
    node: node,
    /**
     * Commit a cluster-wide answer another fetch already holds (the source
     * probe of a scoped query that found node-exporter series): the same
     * snapshot `cluster(view)` would have fetched, without the request.
     */
    commit: commit,
    /** The view's last cluster-wide snapshot (or null). */
    last: function (view) { return lastBy[view] || null; },
  };
}
