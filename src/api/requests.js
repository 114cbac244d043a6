/**
 * Request helpers of the data layer: the per-request time limit (always
 * cleared: reference quirk Q6, IntelGpuDataContext.tsx:75-82), what a failed
 * request says about the resource (absent / refused vs an outage), list
 * identity by version, and the one-node pod list a cold Node detail section
 * reads, shared by callers asking for the same node at once.
 */

import { isKubeList } from './k8sCore.js';

export const DEFAULT_REQUEST_TIMEOUT_MS = 2000;

/**
 * True when two lists hold the same Kubernetes objects at the same versions
 * (uid + resourceVersion, falling back to a JSON comparison for objects
 * without a resourceVersion).
 */
export function sameObjects(a, b) {
  if (a === b) return true;
  if (!a || !b || a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) {
    const ma = a[i] && a[i].metadata;
    const mb = b[i] && b[i].metadata;
    if (!ma || !mb) return false;
    if (ma.resourceVersion && mb.resourceVersion) {
      if (ma.uid !== mb.uid || ma.resourceVersion !== mb.resourceVersion) return false;
    } else if (JSON.stringify(a[i]) !== JSON.stringify(b[i])) {
      return false;
    }
  }
  return true;
}

export const defaultClock = {
  setTimeout: function (fn, ms) { return setTimeout(fn, ms); },
  clearTimeout: function (h) { clearTimeout(h); },
  now: function () { return Date.now(); },
};

/**
 * True when a failed request proves the resource is not there for this user
 * (404 / 403 / 401), as opposed to a timeout or a server / network error.
 * Headlamp's ApiProxy errors carry the HTTP status in `status`.
 */
export function isAbsent(err) {
  const st = err && (err.status || (err.response && err.response.status));
  return st === 404 || st === 403 || st === 401;
}

/**
 * Race `promise` against a timer; the timer is always cleared.
 * @template T
 * @param {Promise<T>} promise
 * @param {number} ms
 * @param {{setTimeout: Function, clearTimeout: Function}} [clock]
 * @returns {Promise<T>}
 */
export function withTimeout(promise, ms, clock) {
  const c = clock || defaultClock;
  return new Promise(function (resolve, reject) {
    let done = false;
    const h = c.setTimeout(function () {
      if (done) return;
      done = true;
      reject(new Error('Request timed out after ' + ms + 'ms'));
    }, ms);
    Promise.resolve(promise).then(
      function (v) {
        if (done) return;
        done = true;
        c.clearTimeout(h);
        resolve(v);
      },
      function (e) {
        if (done) return;
        done = true;
        c.clearTimeout(h);
        reject(e);
      }
    );
  });
}

/** The field selector of one node's pods (the apiserver filters: O(pods on the node)). */
export function nodePodsSelector(nodeName) {
  return 'spec.nodeName=' + nodeName;
}

/** Path of one node's pods: the list request of a field-selected list + watch. */
export function nodePodsPath(nodeName) {
  return '/api/v1/pods?fieldSelector=' + encodeURIComponent(nodePodsSelector(nodeName));
}

/**
 * The pods of ONE node by one field-selected list: the request a cold Node
 * detail page's scoped list + watch starts with (providerCore.js
 * useNodePods), for clients without Headlamp's hooks (the benchmark, the
 * terminal client) — instead of the cluster-wide node + pod lists and the
 * CRD / operator-pod requests the reference's provider mounts there
 * (reference src/index.tsx:152-160, IntelGpuDataContext.tsx:98-165).
 * Resolves to the node's pods; rejects with the request's error.
 * @param {(path: string) => Promise<any>} request
 * @param {string} nodeName
 * @param {number} [timeoutMs]
 * @param {{setTimeout: Function, clearTimeout: Function}} [clock]
 * @returns {Promise<any[]>}
 */
export function fetchNodePods(request, nodeName, timeoutMs, clock) {
  return withTimeout(sharedRequest(request, nodePodsPath(nodeName)), timeoutMs || DEFAULT_REQUEST_TIMEOUT_MS,
    clock || defaultClock).then(function (l) {
    return isKubeList(l) ? l.items : [];
  });
}

// In-flight requests per request function and path: callers asking for the
// same path while it is in flight share one request (two sections of the same
// node, or React 18 StrictMode mounting an effect twice in development).
const inFlight = typeof WeakMap === 'function' ? new WeakMap() : null;

function sharedRequest(request, path) {
  if (!inFlight) return request(path);
  let paths = inFlight.get(request);
  if (!paths) {
    paths = new Map();
    inFlight.set(request, paths);
  }
  const pending = paths.get(path);
  if (pending) return pending;
  const p = Promise.resolve(request(path));
  const done = function () { if (paths.get(path) === p) paths.delete(path); };
  paths.set(path, p);
  p.then(done, done);
  return p;
}
