/**
 * Pod → GPU attribution for the GPU Pods page: the exporter's power gauge of
 * GPUs whose `pod` / `namespace` labels are set — one series per allocated
 * GPU, of the pods on the page (or every owner on a small cluster, or a page
 * Prometheus ranks by power). Nothing else of the GPU is fetched.
 *
 * Kubernetes does not say which device a pod holds (SURVEY §7.3); the
 * reference shows requests only (src/components/PodsPage.tsx:49-88).
 */

import { SMALL_CLUSTER_PODS, STALE_FAILURES } from './series.js';
import { ownersQuery, rankedOwnersQuery } from './promql.js';
import { isRow, joinExporterResults, num, shareGpus, sizeFromRows } from './telemetry.js';
import { UNREACHABLE, staleOrNull } from './promClient.js';

/** Owner answers kept per request key (stale fallbacks, structural sharing). */
const OWNER_KEYS = 16;

/**
 * @param {PromClient} client
 * @param {{source: ('amd-exporter'|'node-exporter'|null)}} state
 */
export function createOwnerSnapshots(client, state) {
  // request key → {last, failures}: a failed refresh of one page's owners
  // serves THAT page's last answer, never another page's.
  let byKey = new Map();
  client.onInvalidate(function () { byKey = new Map(); });

  function entry(key) {
    let e = byKey.get(key);
    if (e) byKey.delete(key);
    else e = { last: null, failures: 0 };
    byKey.set(key, e);
    if (byKey.size > OWNER_KEYS) byKey.delete(byKey.keys().next().value);
    return e;
  }

  /**
   * @param {{pods?: string[], small?: boolean, preview?: number,
   *          rank?: {by: string, page: number, per: number, filter: string}}} [opts]
   *   `pods`: "namespace/name" keys of the page; `small`: every owner when at
   *   most SMALL_CLUSTER_PODS pods own a GPU, else the page's; `preview` (with
   *   `small` and no page yet): on a larger cluster, the `preview` pods
   *   drawing the most power instead, as `preview` = {order, watts, count};
   *   `rank`: the page of pods ranked by the power of the GPUs they hold.
   */
  function owners(opts) {
    const rank = opts && opts.rank;
    if (rank) {
      const rk = 'owners|rank|' + rank.page + '|' + rank.per + '|' + rank.filter;
      return client.shared(rk, function () { return rankedOwners(rank, rk); });
    }
    const pods = opts && Array.isArray(opts.pods) ? opts.pods.map(String) : null;
    const small = !!(opts && opts.small);
    if (small) {
      const pre = !(pods && pods.length) && opts.preview > 0 ? Math.min(200, Math.floor(opts.preview)) : 0;
      const sk = 'owners|small|' + (pre ? 'preview:' + pre + '|' : '') + (pods || []).join(',');
      return client.shared(sk, function () { return ownersOf(pods || [], true, sk, pre); });
    }
    if (pods && pods.length === 0) {
      return Promise.resolve({ source: state.source, gpus: [], xgmi: {}, links: {}, fetchedAt: client.fetchedAt(),
        prometheusPath: client.cachedPath(), scope: 'owners' });
    }
    const k = 'owners|' + (pods ? pods.join(',') : '*');
    return client.shared(k, function () { return ownersOf(pods, false, k); });
  }

  function answer(st, base, j, extra) {
    st.failures = 0;
    const prev = st.last;
    st.last = Object.assign({
      source: j.gpus.length ? 'amd-exporter' : state.source,
      gpus: prev ? shareGpus(prev.gpus, j.gpus) : j.gpus,
      xgmi: {},
      links: {},
      fetchedAt: client.fetchedAt(),
      prometheusPath: base,
      scope: 'owners',
    }, extra);
    return st.last;
  }

  function ownersOf(pods, small, key, preview) {
    const st = entry(key);
    return client.withPrometheus(function (base) {
      return client.combined(base, ownersQuery(pods, small, preview)).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        const owning = small ? sizeFromRows(res.rows.__agg, 'gpu_pods') : 0;
        const exceeded = owning > SMALL_CLUSTER_PODS;
        const r = preview && exceeded ? rankRows(res.rows) : null;
        return answer(st, base, joinExporterResults(res.rows), {
          small: small ? { count: owning, limit: SMALL_CLUSTER_PODS, exceeded: exceeded } : undefined,
          preview: r ? { per: preview, count: owning, order: r.order, watts: r.watts } : undefined,
        });
      });
    }, function () { return staleOrNull(st, STALE_FAILURES, client.invalidate); });
  }

  /** The `agg="rank"` rows of an answer: "namespace/pod" keys highest power first, and the watts per key. */
  function rankRows(rows) {
    const ranked = [];
    const watts = {};
    for (let i = 0; i < rows.__agg.length; i++) {
      const r = rows.__agg[i];
      if (!isRow(r) || r.metric.agg !== 'rank' || typeof r.metric.pod !== 'string') continue;
      const k = (typeof r.metric.namespace === 'string' ? r.metric.namespace : '') + '/' + r.metric.pod;
      const w = num(r.value[1]);
      ranked.push([k, w === null ? -Infinity : w]);
      watts[k] = w;
    }
    ranked.sort(function (a, b) { return b[1] - a[1] || (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0); });
    return { order: ranked.map(function (x) { return x[0]; }), watts: watts };
  }

  /**
   * GPU pods in power order (promql.js rankedOwnersQuery): the page's owners
   * plus `rank` = {by, page, per, filter, count, order: "namespace/pod" keys
   * highest first, watts per key}.
   */
  function rankedOwners(rank, key) {
    const st = entry(key);
    return client.withPrometheus(function (base) {
      return client.combined(base, rankedOwnersQuery(rank)).then(function (res) {
        if (!res.ok) return UNREACHABLE;
        const rows = res.rows;
        const r = rankRows(rows);
        return answer(st, base, joinExporterResults(rows), {
          rank: { by: rank.by, page: rank.page, per: rank.per, filter: rank.filter, count: sizeFromRows(rows.__agg, 'ranked'),
            order: r.order, watts: r.watts },
        });
      });
    }, function () { return staleOrNull(st, STALE_FAILURES, client.invalidate); });
  }

  return { owners: owners };
}
