/**
 * The transport under every telemetry fetch: Prometheus discovery behind the
 * Kubernetes service proxy, time-boxed requests, one in-flight request per
 * key, and the cache reset all fetchers share.
 *
 * Reference analog: findPrometheusPath + queryPrometheus
 * (src/api/metrics.ts:67-90), which probed three services SERIALLY with no
 * timeout before every fetch. Here (ADR 003, 006):
 *   * the first query goes straight to the preferred service — its answer is
 *     the discovery; only when it fails are all candidates probed IN
 *     PARALLEL, each time-boxed; the winner is cached for DISCOVERY_TTL_MS;
 *   * a second caller of the same fetch while it is in flight shares it;
 *   * the HTTP status of a failure is kept, so a page can tell RBAC (403 on
 *     services/proxy) from an outage.
 */

import { DEFAULT_REQUEST_TIMEOUT_MS, withTimeout } from './clusterStore.js';
import { DISCOVERY_TTL_MS, PROMETHEUS_SERVICES, servicePath } from './series.js';
import { isObject } from './k8sCore.js';
import { splitByName, stringLabels } from './telemetry.js';

/** Marker for "the request did not reach a Prometheus". */
export const UNREACHABLE = Object.freeze({ unreachable: true });

/**
 * @param {{ request: (path: string) => Promise<any>, timeoutMs?: number,
 *           clock?: {setTimeout: Function, clearTimeout: Function, now: Function},
 *           services?: Array<{namespace: string, service: string, port: string}>,
 *           discoveryTtlMs?: number,
 *           onTrace?: (span: {name: string, path: string, start: number, end: number, ok: boolean}) => void }} opts
 */
export function createPromClient(opts) {
  const request = opts.request;
  const timeoutMs = opts.timeoutMs || DEFAULT_REQUEST_TIMEOUT_MS;
  const clock = opts.clock || { setTimeout: setTimeout, clearTimeout: clearTimeout, now: Date.now };
  const services = opts.services || PROMETHEUS_SERVICES;
  const ttl = opts.discoveryTtlMs === undefined ? DISCOVERY_TTL_MS : opts.discoveryTtlMs;
  const onTrace = opts.onTrace || null;

  let cachedPath = null;
  let cachedAt = 0;
  let discovering = null;
  const resets = [];

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

  /** Forget the service and every fetcher's cache (each registered with onInvalidate). */
  function invalidate() {
    cachedPath = null;
    for (let i = 0; i < resets.length; i++) resets[i]();
  }

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
   * UNREACHABLE when its request failed; `onCachedFailure()` decides what a
   * failure against a known service returns (a stale answer, or null).
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
   * One range query; resolves {name → {node → [[t, v]]}} or UNREACHABLE.
   * `totalKey` names rows tagged scope="cluster" (the cluster-wide line).
   */
  function range(base, q, start, end, step, totalKey) {
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
          const node = m.scope === 'cluster' ? totalKey
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

  return {
    clock: clock,
    ttl: ttl,
    discover: discover,
    invalidate: invalidate,
    /** Register a cache reset run by invalidate() (Prometheus moved or went away). */
    onInvalidate: function (fn) { resets.push(fn); },
    shared: shared,
    withPrometheus: withPrometheus,
    combined: combined,
    range: range,
    /** The cached service's base path (null until one answered). */
    cachedPath: function () { return cachedPath; },
    failureReason: function () { return lastFailureStatus === 401 || lastFailureStatus === 403 ? 'forbidden' : 'unreachable'; },
    now: function () { return clock.now(); },
    fetchedAt: function () { return new Date(clock.now()).toISOString(); },
  };
}

/**
 * The failure policy every fetcher shares: a transient failure (timeout,
 * 5xx) serves the last answer marked `stale`; STALE_FAILURES in a row mean
 * Prometheus went away (null, and the service is re-discovered).
 * @param {{last: any, failures: number}} st  per-answer state
 * @param {number} limit
 * @param {() => void} invalidate
 */
export function staleOrNull(st, limit, invalidate) {
  st.failures++;
  if (st.last && st.failures < limit) return Object.assign({}, st.last, { stale: true });
  st.last = null;
  invalidate();
  return null;
}
