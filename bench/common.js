/**
 * Shared pieces of the benchmark driver (bench/driver.js): the browser-like
 * HTTP client (keep-alive, 6 sockets per origin), the high-resolution clock,
 * latency statistics, GC-pause accounting and request-trace summaries.
 */
import http from 'http';
import { PerformanceObserver } from 'perf_hooks';

// Garbage-collection pauses (start, duration in ms, performance.now() clock),
// so a timed sample can say how much of it was the collector.
const gcPauses = [];
try {
  new PerformanceObserver(function (list) {
    list.getEntries().forEach(function (e) { gcPauses.push([e.startTime, e.duration]); });
    if (gcPauses.length > 4096) gcPauses.splice(0, gcPauses.length - 4096);
  }).observe({ entryTypes: ['gc'] });
} catch (e) {
  // no GC entries on this runtime
}

/** GC pause time (ms) that started inside [from, to] (performance.now() clock). */
export function gcBetween(from, to) {
  let t = 0;
  for (let i = 0; i < gcPauses.length; i++) if (gcPauses[i][0] >= from && gcPauses[i][0] <= to) t += gcPauses[i][1];
  return t;
}

/** What a request path asks for: nodes, pods, crd, query, query_range or other. */
export function requestKind(path) {
  if (path.indexOf('/proxy/') >= 0) return path.indexOf('/query_range') >= 0 ? 'query_range' : 'query';
  if (path.indexOf('/deviceconfigs') >= 0) return 'crd';
  if (path.indexOf('/api/v1/nodes') === 0) return 'nodes';
  if (path.indexOf('/pods') >= 0) return 'pods';
  return 'other';
}

/**
 * An HTTP/1.1 keep-alive client (6 sockets, the browser's per-origin limit)
 * counting requests and bytes on `counter`; with `counter.log` (an array) it
 * also records each request's kind, wall span and the fake server's own time
 * on it (its `X-Server-Ms` header: work, not the injected latency).
 */
export function makeRequest(base, counter) {
  const agent = new http.Agent({ keepAlive: true, maxSockets: 6 });
  const u = new URL(base);
  return function request(path) {
    counter.n++;
    const t0 = hiResClock.now();
    return new Promise(function (resolve, reject) {
      const req = http.get({ hostname: u.hostname, port: u.port, path: path, agent: agent, headers: { Accept: 'application/json' } }, function (res) {
        const chunks = [];
        res.on('data', function (c) { chunks.push(c); });
        res.on('end', function () {
          const body = Buffer.concat(chunks);
          counter.bytes += body.length;
          const server = parseFloat(res.headers['x-server-ms']);
          if (isFinite(server)) counter.serverMs = (counter.serverMs || 0) + server;
          if (counter.log) {
            counter.log.push({ kind: requestKind(path), start: t0, end: hiResClock.now(), serverMs: isFinite(server) ? server : null });
          }
          let json = null;
          try {
            json = JSON.parse(body.toString('utf8'));
          } catch (e) {
            reject(new Error('bad JSON from ' + path));
            return;
          }
          if (res.statusCode >= 400) {
            const err = new Error((json && json.message) || 'HTTP ' + res.statusCode);
            err.status = res.statusCode;
            // Prometheus answers 4xx with a JSON body the caller may want.
            if (json && json.status === 'error') resolve(json);
            else reject(err);
            return;
          }
          resolve(json);
        });
      });
      req.on('error', reject);
    });
  };
}

export function ms(hr) {
  return hr[0] * 1e3 + hr[1] / 1e6;
}

// Epoch milliseconds with sub-millisecond resolution (Date.now() anchored,
// hrtime deltas): request spans resolve to microseconds instead of 1 ms.
const EPOCH0 = Date.now();
const HR0 = process.hrtime();
export const hiResClock = {
  setTimeout: function (fn, t) { return setTimeout(fn, t); },
  clearTimeout: function (h) { clearTimeout(h); },
  now: function () { return EPOCH0 + ms(process.hrtime(HR0)); },
};

export function stats(xs) {
  const s = xs.slice().sort(function (a, b) { return a - b; });
  const q = function (p) {
    if (!s.length) return null;
    const idx = (s.length - 1) * p;
    const lo = Math.floor(idx);
    const hi = Math.ceil(idx);
    return s[lo] + (s[hi] - s[lo]) * (idx - lo);
  };
  const mean = s.reduce(function (a, b) { return a + b; }, 0) / (s.length || 1);
  return { n: s.length, p50: q(0.5), p95: q(0.95), min: s[0], max: s[s.length - 1], mean: mean };
}

/** p50 latency per traced request kind, plus how many of each were issued. */
export function traceSummary(spans) {
  const by = {};
  for (let i = 0; i < spans.length; i++) {
    const s = spans[i];
    const k = s.name.replace(/-\d+$/, '');
    if (!by[k]) by[k] = [];
    by[k].push(s.end - s.start);
  }
  const out = {};
  for (const k in by) out[k] = { n: by[k].length, p50_ms: stats(by[k]).p50 };
  return out;
}
