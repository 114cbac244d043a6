/**
 * Per-object caches of values derived on first use — a node's link
 * statistics, a telemetry snapshot's per-node power keys, a pod's container
 * lines — kept with their objects (WeakMap) and dropped together by
 * resetDerivedCaches().
 *
 * Facts derived when a list arrives (clusterIndex.js nodeFacts / podFacts,
 * computed by the index build) are not here: a page finds them filled. These
 * are computed by the first render that needs them, so a cold mount pays for
 * them. The view memo's reset (pages/common.js clearViewMemo: a cluster
 * switch, tests, the benchmark's first-render-of-a-session mount) resets
 * them too.
 */

const registry = [];

/** A WeakMap-backed cache that resetDerivedCaches() empties. */
export function derivedCache() {
  const c = {
    map: new WeakMap(),
    has: function (k) { return c.map.has(k); },
    get: function (k) { return c.map.get(k); },
    set: function (k, v) { c.map.set(k, v); return v; },
    onReset: null,
  };
  registry.push(c);
  return c;
}

/** Empty every derived cache (and run their reset hooks: structural-sharing "previous" state). */
export function resetDerivedCaches() {
  for (let i = 0; i < registry.length; i++) {
    registry[i].map = new WeakMap();
    if (registry[i].onReset) registry[i].onReset();
  }
}
