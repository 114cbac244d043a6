/**
 * Which cluster the UI is showing. Headlamp routes cluster views under
 * `/c/<cluster>/…`; the shared store and the Prometheus discovery cache are
 * keyed by it so switching clusters never mixes data.
 */

/** @param {string} [pathname] @returns {string} */
export function clusterFromPath(pathname) {
  const m = /(?:^|\/)c\/([^/]+)(?:\/|$)/.exec(pathname || '');
  return m ? decodeURIComponent(m[1]) : '__default__';
}

/** Current cluster key (browser location; `__default__` outside a browser). */
export function clusterKey() {
  if (typeof window === 'undefined' || !window.location) return '__default__';
  const hash = window.location.hash && window.location.hash.indexOf('/c/') >= 0 ? window.location.hash : '';
  return clusterFromPath(hash || window.location.pathname);
}
