/**
 * MI355X telemetry from Prometheus, reached through the Kubernetes service proxy.
 *
 * Reference analog: src/api/metrics.ts (SURVEY.md C4), which finds
 * Prometheus by probing three services serially with no timeout (:77-90),
 * then runs four instant queries on i915 hwmon series and joins power by
 * PCI `chip` only (:127-138, quirk Q1).
 *
 * This client (ADR 002, 003, 006, 008, 009) is assembled from small parts
 * that share one transport and one idea of which exporter feeds Prometheus:
 *
 *   ./series.js          names: services, AMD series, labels, size limits
 *   ./promql.js          the PromQL each page sends (pure builders)
 *   ./telemetry.js       answers → per-GPU telemetry, totals, sharing (pure)
 *   ./promClient.js      discovery, time-boxed requests, in-flight sharing
 *   ./clusterSnapshots.js  cluster-wide and per-node snapshots
 *   ./scopedSnapshots.js   one page of nodes (by name, small-cluster, ranked)
 *   ./ownerSnapshots.js    pod → GPU attribution (GPU Pods page)
 *   ./seriesFetch.js       power / HBM `query_range` series
 *   ./nodeSummaries.js     per-node power / temperature / owner keys and link
 *                          facts, derived as each snapshot arrives
 *
 * In short: the first query goes straight to the preferred service (its
 * answer is the discovery), then parallel time-boxed probes only if that
 * fails; AMD Device Metrics Exporter series (`gpu_*`, optionally
 * pod-labelled), this repo's amdgpu-exporter extensions (power cap, link
 * hops, throttle thresholds) and node-exporter's amdgpu hwmon + DRM
 * collectors as a fallback; every GPU keyed by (node, gpu index); structure
 * shared between snapshots; the last snapshot served marked `stale` through
 * transient failures. Metric and label names are pinned by captures from a
 * real MI355X (tests/fixtures/mi355x).
 *
 * Callers import names, PromQL builders and joins from those modules
 * directly; this module only assembles the client.
 */

import { METRIC_VIEWS } from './series.js';
import { nodeExporterNodePowerQuery, nodePowerQuery, podPowerQuery } from './promql.js';
import { createPromClient } from './promClient.js';
import { createClusterSnapshots } from './clusterSnapshots.js';
import { createScopedSnapshots } from './scopedSnapshots.js';
import { createOwnerSnapshots } from './ownerSnapshots.js';
import { createSeriesFetch, seriesQueryFor } from './seriesFetch.js';
import { primeSnapshot } from './nodeSummaries.js';


/**
 * @param {{ request: (path: string) => Promise<any>, timeoutMs?: number,
 *           clock?: {setTimeout: Function, clearTimeout: Function, now: Function},
 *           services?: Array<{namespace: string, service: string, port: string}>,
 *           discoveryTtlMs?: number,
 *           onTrace?: (span: {name: string, path: string, start: number, end: number, ok: boolean}) => void }} opts
 */
export function createMetricsSource(opts) {
  const client = createPromClient(opts);
  // Which exporter answered ('amd-exporter' | 'node-exporter' | null: not
  // known yet), and whether every exporter series carries `hostname` (lean
  // live queries). Shared by every part; forgotten when Prometheus moves.
  // `deciding`: the telemetry fetch in flight while the source is unknown
  // (its answer decides it); a series window that found no exporter series
  // waits for it before asking node-exporter (seriesFetch.js).
  const state = { source: null, lean: false, deciding: null };
  client.onInvalidate(function () {
    state.source = null;
    state.lean = false;
    state.deciding = null;
  });
  const snaps = createClusterSnapshots(client, state);
  const scoped = createScopedSnapshots(client, state, snaps);
  const owners = createOwnerSnapshots(client, state);
  const series = createSeriesFetch(client, state);

  /**
   * One metrics snapshot of the series `view` needs (METRIC_VIEWS; default
   * 'all'). Resolves to null when no Prometheus is reachable (the page's
   * "Prometheus Unreachable" state).
   *
   * `opts.scope` (GPU node names): that page of nodes only, with the cluster
   * totals when `opts.summary`, size-guarded when `opts.small`
   * (scopedSnapshots.js); `opts.rank` {page, per, filter}: the page
   * Prometheus ranks by total GPU power.
   * @param {string} [view]
   * @returns {Promise<GpuMetrics|null>}
   */
  function fetchGpuMetrics(view, opts) {
    return deciding(telemetry(view, opts)).then(primeSnapshot);
  }

  /**
   * While the source is unknown, a telemetry answer in flight is what
   * decides it: range windows asked meanwhile wait for it before asking
   * node-exporter (seriesFetch.js rangeOf), so a cluster with the exporter
   * never evaluates node-exporter's range joins.
   */
  function deciding(p) {
    if (state.source === null) {
      const d = p.then(function () {}, function () {});
      state.deciding = d;
      d.then(function () { if (state.deciding === d) state.deciding = null; });
    }
    return p;
  }

  function telemetry(view, opts) {
    const v = view === undefined ? 'all' : view;
    if (METRIC_VIEWS.indexOf(v) < 0) return Promise.reject(new Error('fetchGpuMetrics: unknown view ' + JSON.stringify(view)));
    if (opts && opts.rank) {
      const rank = {
        by: 'power',
        page: Math.max(0, Math.floor(opts.rank.page) || 0),
        per: opts.rank.per > 0 ? Math.min(200, Math.floor(opts.rank.per)) : 8,
        filter: String(opts.rank.filter || '').trim().toLowerCase(),
      };
      const rkey = 'rank|' + v + '|' + rank.page + '|' + rank.per + '|' + rank.filter + (opts.summary ? '|sum' : '');
      return client.shared(rkey, function () { return scoped.ranked(v, rank, !!opts.summary, rkey); });
    }
    const scope = opts && Array.isArray(opts.scope) ? opts.scope.map(String) : null;
    if (!scope) return snaps.cluster(v);
    const summary = !!opts.summary;
    const small = !!opts.small;
    const key = v + '|' + (summary ? 'sum' : '') + '|' + (small ? 'small|' : '') + scope.join(',');
    return client.shared('scoped|' + key, function () { return scoped.scoped(v, scope, summary, key, small); });
  }

  return {
    discover: client.discover,
    invalidate: client.invalidate,
    /**
     * Why the last fetch found no Prometheus: 'forbidden' when the proxy
     * answered 401 / 403 (the user lacks `services/proxy` get on the
     * Prometheus service), else 'unreachable'.
     */
    failureReason: client.failureReason,
    fetchGpuMetrics: fetchGpuMetrics,
    /** Telemetry of ONE node's GPUs (native Node / Pod detail pages), `hostname`-scoped. */
    fetchNodeMetrics: function (nodeName) { return deciding(snaps.node(nodeName)).then(primeSnapshot); },
    /** Pod → GPU attribution (ownerSnapshots.js). */
    fetchGpuOwners: function (o) { return owners.owners(o).then(primeSnapshot); },
    /** Per-node power / HBM series over the last `rangeSec` (seriesFetch.js). */
    fetchSeries: series.series,
    /** A pod's GPU power over the last `rangeSec`: {rangeSec, stepSec, power: [[t, W]]}, or null. */
    fetchPodSeries: function (namespace, pod, rangeSec, stepSec) {
      return series.powerSeries('pod|' + namespace + '/' + pod, podPowerQuery(namespace, pod), rangeSec, stepSec);
    },
    /** A node's GPU power over the last `rangeSec` (shape and nulls as fetchPodSeries). */
    fetchNodeSeries: function (nodeName, rangeSec, stepSec) {
      return series.powerSeries('node|' + nodeName, function (source) {
        return seriesQueryFor(source, nodePowerQuery(nodeName), nodeExporterNodePowerQuery(nodeName));
      }, rangeSec, stepSec);
    },
    source: function () { return state.source; },
  };
}
