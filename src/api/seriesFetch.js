/**
 * Power / HBM time series (`query_range`) for the Metrics page and the
 * detail pages' power history. The reference has instant queries only
 * (src/api/metrics.ts:67-75); its mock-up's 30-minute chart was never built
 * (SURVEY Q12).
 *
 *   * `series(range, step, scope, small)`: per-node power + HBM-used, one
 *     request for both, `sum by (__name__, hostname)` server-side, scoped to
 *     the page's nodes with the cluster line alongside. Incremental: samples
 *     are step-aligned and Prometheus never rewrites a past step, so after the
 *     first call only the steps newer than the cache are asked for — and none
 *     at all until the next step boundary.
 *   * `powerSeries(key, q, range, step)`: one pod's or node's total GPU power.
 */

import { SERIES, TOTAL_SERIES } from './series.js';
import {
  nodeExporterScopedSeriesQuery,
  nodeExporterSeriesQuery,
  scopedSeriesQuery,
  seriesQuery,
} from './promql.js';
import { num } from './telemetry.js';
import { UNREACHABLE } from './promClient.js';

/**
 * The range queries of a window: the known source's — the exporter's, or
 * node-exporter's in the exporter's shape (promql.js nodeExporterSeriesQuery)
 * — or, while no answer has told which feeds Prometheus, the exporter's
 * first and node-exporter's second (rangeOf).
 */
export function seriesQueryFor(source, exporterQ, hwQ) {
  if (source === 'node-exporter') return [hwQ];
  if (source === 'amd-exporter') return [exporterQ];
  return [exporterQ, hwQ];
}

/** A range answer with no series at all. */
function noSeries(got) {
  for (const k in got) return false;
  return true;
}

/**
 * `client.range` of qs[0]; when it finds no series and a node-exporter query
 * follows (the source was unknown), qs[1] — but only once the telemetry
 * answer in flight (`st.deciding`) has named node-exporter the source. A
 * cluster with the exporter never pays for node-exporter's joins
 * (node-exporter runs on nearly every node), one without GPU telemetry sends
 * nothing more, and the first window of a node-exporter cluster costs one
 * more round trip.
 */
function rangeOf(client, st, base, qs, start, end, step) {
  return client.range(base, qs[0], start, end, step, TOTAL_SERIES).then(function (got) {
    if (got === UNREACHABLE || qs.length < 2 || !noSeries(got)) return got;
    return Promise.resolve(st.deciding).then(function () {
      return st.source === 'node-exporter' ? client.range(base, qs[1], start, end, step, TOTAL_SERIES) : got;
    });
  });
}

/**
 * @param {PromClient} client
 * @param {{source: ('amd-exporter'|'node-exporter'|null)}} [state]  which exporter feeds Prometheus (shared)
 */
export function createSeriesFetch(client, state) {
  const st = state || { source: 'amd-exporter' };
  let cache = null; // { range, step, end, base, scope, data }
  client.onInvalidate(function () { cache = null; });

  /**
   * @returns {Promise<{rangeSec: number, stepSec: number, power: Record<string, Array<[number, number]>>,
   *   vram: Record<string, Array<[number, number]>>, scope?: string[], total?: any} | null>}
   */
  function series(rangeSec, stepSec, scope, small) {
    const range = rangeSec || 1800;
    const step = stepSec || 30;
    const E = SERIES.exporter;
    const parts = [['power', E.power, 1], ['vram', E.vramUsed, SERIES.exporterVramUnitBytes]];
    const scoped = Array.isArray(scope);
    const src = st.source;
    const sk = (src || '?') + '|' + (scoped ? (small ? 'small:' : '') + scope.map(String).join(',') : '*');
    const qs = seriesQueryFor(src,
      scoped ? scopedSeriesQuery(scope.map(String), !!small) : seriesQuery(),
      scoped ? nodeExporterScopedSeriesQuery(scope.map(String), !!small) : nodeExporterSeriesQuery());
    function from(base) {
      const end = Math.floor(client.now() / 1000 / step) * step;
      const fresh = !cache || cache.range !== range || cache.step !== step ||
        cache.base !== base || cache.scope !== sk || end - cache.end >= range;
      const start = fresh ? end - range : cache.end + step;
      if (!fresh && start > end) return Promise.resolve(cache.data);
      return rangeOf(client, st, base, qs, start, end, step).then(function (got) {
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
          const prev = fresh ? {} : cache.data[key] || {};
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
            const prevTotal = fresh ? [] : (cache.data.total && cache.data.total[key]) || [];
            data.total[key] = prevTotal.concat(add).filter(function (p) { return p[0] >= cutoff; });
          }
        }
        cache = { range: range, step: step, end: end, base: base, scope: sk, data: data };
        return data;
      });
    }
    // A failed range request keeps the last window of the same scope (retried next time).
    return client.shared('series|' + range + '|' + step + '|' + sk, function () {
      return client.withPrometheus(from, function () { return cache && cache.scope === sk ? cache.data : null; });
    });
  }

  /**
   * Total GPU power over the last `rangeSec` of what `q` selects (a pod's or
   * a node's GPUs), step-aligned like series(): `{rangeSec, stepSec, power:
   * [[t, W]]}`; `power` is empty when nothing matches. Null when Prometheus is
   * unreachable.
   */
  function powerSeries(scope, query, rangeSec, stepSec) {
    const range = rangeSec || 1800;
    const step = stepSec || 30;
    // `query`: the PromQL, or a function of the source giving the queries to try (seriesQueryFor)
    const q = typeof query === 'function' ? query(st.source) : query;
    const qs = Array.isArray(q) ? q : [q];
    const key = 'power|' + scope + '|' + range + '|' + step + '|' + st.source;
    return client.shared(key, function () {
      return client.withPrometheus(function (base) {
        const end = Math.floor(client.now() / 1000 / step) * step;
        return rangeOf(client, st, base, qs, end - range, end, step).then(function (got) {
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

  return { series: series, powerSeries: powerSeries };
}
