/**
 * Seeded fuzzing helpers shared by tests/js/properties.test.js (view-models
 * never throw on malformed objects) and tests/js/shared/fuzz.shared.test.js
 * (what they produce renders on every React tier).
 */

/** mulberry32: tiny deterministic PRNG. */
export function rng(seed) {
  let a = seed >>> 0;
  return function () {
    a = (a + 0x6d2b79f5) >>> 0;
    let t = a;
    t = Math.imul(t ^ (t >>> 15), t | 1);
    t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}
export const int = (r, lo, hi) => lo + Math.floor(r() * (hi - lo + 1));
export const pick = (r, xs) => xs[Math.floor(r() * xs.length)];

/** Values of the wrong shape a real apiserver, an old CRD version or a half-written object can hand over. */
export const WRONG = [null, undefined, 0, 7, -1, '', 'x', 'NaN', true, [], {}, [null], { a: 1 }];

/** Replace a random leaf or subtree of `o` with a value of the wrong shape (or delete it). */
export function mutate(r, o, depth) {
  if (o === null || typeof o !== 'object' || depth > 6) return pick(r, WRONG);
  const keys = Object.keys(o);
  if (!keys.length) return pick(r, WRONG);
  const out = Array.isArray(o) ? o.slice() : Object.assign({}, o);
  const k = pick(r, keys);
  if (r() < 0.35) {
    if (Array.isArray(out)) out.splice(Number(k), 1);
    else delete out[k];
  } else out[k] = r() < 0.5 ? pick(r, WRONG) : mutate(r, o[k], depth + 1);
  return out;
}
