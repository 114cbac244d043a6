/**
 * Incremental classification of a watched Kubernetes list.
 *
 * Headlamp's `useList()` hands the provider a NEW array of every object in
 * the cluster after each watch event (reference: the provider re-filters all
 * of them in a useMemo keyed on the array, IntelGpuDataContext.tsx:200-208,
 * and the Overview page re-aggregates on every render, OverviewPage.tsx:72-130).
 * On a 1000-node cluster that is ~37k pods classified per event, although
 * one pod changed.
 *
 * A tracker remembers, per object, the classification bits it computed and
 * the object version they belong to, and diffs each new list against the
 * previous one:
 *
 *   * the common prefix and suffix of the two arrays (elements `===`) are
 *     unchanged — Headlamp's list cache replaces, inserts or removes the
 *     object an event touched and keeps the others — so they cost one
 *     identity compare each and nothing else;
 *   * each object in the differing middle is compared with the old middle
 *     alongside (new wrappers around the same JSON), else looked up by uid
 *     (namespace/name without one): same object or same `resourceVersion` →
 *     reused, keeping the object ALREADY held, so a re-parsed copy changes
 *     no identity downstream; otherwise classified;
 *   * objects of the old middle that were not reused are deletions.
 *
 * Each subset (e.g. "requests an amd.com resource", "is an operator pod") is
 * an array that keeps its identity unless an object with that bit was
 * added, changed, moved or removed — so unrelated churn invalidates no
 * memoised view. A change is applied to the subset as a delta (replaced,
 * removed and inserted members: O(subset) copying, no re-classification, no
 * pass over the whole list) and reported, so consumers can patch what they
 * derived from the subset too; a reorder falls back to a rebuild from the
 * cached bits. A list that is all new objects (every wrapper or every
 * object re-created) is handled the same way, by lookups instead of compares.
 */

import { unwrapKubeObject } from './k8sCore.js';

function keyOf(raw) {
  const m = raw && raw.metadata;
  if (!m) return null;
  // A uid is a UUID; the fallback starts with a character no uid holds.
  return m.uid ? m.uid : '\u0000' + (m.namespace || '') + '/' + (m.name || '');
}

function versionOf(raw) {
  const m = raw && raw.metadata;
  return m && m.resourceVersion ? m.resourceVersion : null;
}

/**
 * `raw` is the object of record `rec`, at the same version: same uid and
 * resourceVersion. Used for the object alongside in the old list, so a
 * re-parsed list whose order did not change costs two string compares per
 * object instead of a hash lookup.
 */
function samePositional(rec, raw) {
  if (rec.version === null || rec.key === null) return false;
  const m = raw && raw.metadata;
  return !!m && m.resourceVersion === rec.version && m.uid === rec.key;
}

/** Beyond this many changed members a subset is rebuilt instead of patched. */
const MAX_PATCH = 64;

/**
 * @typedef {{replaced: Array<[any, any]>, removed: any[], added: any[]}} SubsetDelta
 *   replaced: [old, new] versions of one object; removed / added: members
 *   that left / joined.
 */

/**
 * @param {Array<(raw: any) => boolean>} predicates  one per subset
 */
export function createListTracker(predicates) {
  const nSub = predicates.length;
  let byKey = new Map();
  let prevItems = []; // the array handed to the previous update
  let prevRec = []; // its records, by position
  let gen = 0;
  // The first list, classified but without records yet ({raws, bits}): a
  // cold open pays the classification only, like a plain filter; the records
  // (and the uid map) are built when a second list arrives.
  let pending = null;
  let subsets = [];
  for (let b = 0; b < nSub; b++) subsets.push([]);
  const stats = { updates: 0, classified: 0, reused: 0, compared: 0, subsetPatches: 0, subsetRebuilds: 0 };

  function classify(raw) {
    let bits = 0;
    for (let b = 0; b < nSub; b++) if (predicates[b](raw)) bits |= 1 << b;
    stats.classified++;
    return bits;
  }

  /**
   * The record of `raw`: reused, or classified afresh. `w.replaced` is set to
   * the record a new version replaces (same key), if any.
   */
  function recordOf(raw, w) {
    const key = keyOf(raw);
    let rec = key === null ? undefined : byKey.get(key);
    w.replaced = null;
    if (rec && rec.gen !== gen && (rec.raw === raw || (rec.version !== null && rec.version === versionOf(raw)))) {
      rec.gen = gen;
      stats.reused++;
      return rec;
    }
    if (rec && rec.gen !== gen) w.replaced = rec;
    const bits = key === null ? 0 : classify(raw);
    rec = { raw: raw, key: key, version: versionOf(raw), bits: bits, gen: gen, pos: -1 };
    if (key !== null) byKey.set(key, rec);
    return rec;
  }

  function materialize() {
    if (!pending) return;
    const raws = pending.raws;
    const bits = pending.bits;
    const recs = new Array(raws.length);
    for (let i = 0; i < raws.length; i++) {
      const raw = raws[i];
      const key = keyOf(raw);
      const rec = { raw: raw, key: key, version: versionOf(raw), bits: bits[i], gen: pending.gen, pos: i };
      if (key !== null) byKey.set(key, rec);
      recs[i] = rec;
    }
    prevRec = recs;
    pending = null;
  }

  function positionOf(raw) {
    materialize();
    const r = byKey.get(keyOf(raw));
    return r ? r.pos : -1;
  }

  /** Insert `raw` into `out` (ordered by list position) where its position belongs. */
  function insertOrdered(out, raw) {
    const p = positionOf(raw);
    let lo = 0;
    let hi = out.length;
    while (lo < hi) {
      const mid = (lo + hi) >> 1;
      if (positionOf(out[mid]) < p) lo = mid + 1;
      else hi = mid;
    }
    out.splice(lo, 0, raw);
  }

  /**
   * Take the new list (raw objects or Headlamp KubeObject wrappers).
   * `deltas[b]`, when not null, is how subset b changed (SubsetDelta), for
   * consumers that patch what they derived from it.
   * @param {any[]|null} items
   * @returns {{subsets: any[][], changed: boolean[], deltas: Array<SubsetDelta|null>}}
   */
  function update(items) {
    stats.updates++;
    const list = Array.isArray(items) ? items : [];
    const n = list.length;
    const pn = prevItems.length;
    const changed = [];
    const deltas = [];
    for (let b = 0; b < nSub; b++) {
      changed.push(false);
      deltas.push(null);
    }
    if (list === prevItems) return { subsets: subsets, changed: changed, deltas: deltas };
    if (pn === 0 && !pending && byKey.size === 0 && n > 0) return firstLoad(list, changed, deltas);
    materialize();
    gen++;
    // Common prefix and suffix: untouched.
    let lo = 0;
    while (lo < n && lo < pn && list[lo] === prevItems[lo]) lo++;
    let hiNew = n;
    let hiOld = pn;
    while (hiNew > lo && hiOld > lo && list[hiNew - 1] === prevItems[hiOld - 1]) {
      hiNew--;
      hiOld--;
    }
    stats.compared += lo + (n - hiNew);

    // The differing middle: reuse or classify each object. `j` walks the old
    // middle alongside, so objects that kept their JSON (new wrappers around
    // the same object) cost a compare, not a lookup.
    let dirty = 0; // bit b: subset b may have changed
    const middle = new Array(hiNew - lo);
    const replacedPairs = []; // old rec, new rec, ...
    const addedRecs = [];
    let ordered = true; // surviving objects kept their relative order
    let lastPos = -1;
    const w = { replaced: null };
    let j = lo;
    for (let i = lo; i < hiNew; i++) {
      const raw = unwrapKubeObject(list[i]);
      let rec;
      const pj = j < hiOld ? prevRec[j] : null;
      if (pj !== null && pj.gen !== gen && (pj.raw === raw || samePositional(pj, raw))) {
        rec = pj;
        if (rec.raw !== raw) stats.reused++;
        rec.gen = gen;
        j++;
        w.replaced = null;
      } else {
        rec = recordOf(raw, w);
        // Resynchronise after an insertion / deletion.
        if (rec.pos >= j && rec.pos < hiOld && prevRec[rec.pos] === rec) j = rec.pos + 1;
      }
      middle[i - lo] = rec;
      const old = w.replaced;
      if (old) {
        replacedPairs.push(old, rec);
        dirty |= old.bits | rec.bits;
        if (old.pos < lastPos) ordered = false;
        lastPos = old.pos;
      } else if (rec.pos < 0) {
        addedRecs.push(rec);
        dirty |= rec.bits;
      } else {
        if (rec.pos < lastPos) ordered = false;
        lastPos = rec.pos;
      }
    }
    // Old middle objects neither reused nor replaced: deleted.
    const removedRecs = [];
    for (let k = lo; k < hiOld; k++) {
      const r = prevRec[k];
      if (r.gen === gen) continue;
      if (r.key === null) continue;
      if (byKey.get(r.key) === r) {
        byKey.delete(r.key);
        removedRecs.push(r);
        dirty |= r.bits;
      }
    }
    // A reordered survivor moves in its subsets too.
    if (!ordered) dirty = (1 << nSub) - 1;

    // Patch the record array in place (no copy of the untouched parts).
    let recs;
    if (lo === 0 && hiOld === pn) recs = middle;
    else if (hiNew === hiOld) {
      recs = prevRec;
      for (let i = lo; i < hiNew; i++) recs[i] = middle[i - lo];
    } else {
      recs = prevRec;
      Array.prototype.splice.apply(recs, [lo, hiOld - lo].concat(middle));
    }
    // Positions from the middle on (the suffix moves when the length changed).
    const to = hiNew === hiOld ? hiNew : recs.length;
    for (let i = lo; i < to; i++) recs[i].pos = i;
    prevItems = list;
    prevRec = recs;

    for (let b = 0; b < nSub; b++) {
      const bit = 1 << b;
      if (!(dirty & bit)) continue;
      const old = subsets[b];
      let out = null;
      let delta = null;
      if (ordered) {
        // Delta: swap replaced members, drop removed ones, insert new ones.
        delta = { replaced: [], removed: [], added: [] };
        for (let k = 0; k < replacedPairs.length; k += 2) {
          const o = replacedPairs[k];
          const r = replacedPairs[k + 1];
          if (o.bits & bit && r.bits & bit) delta.replaced.push([o.raw, r.raw]);
          else if (o.bits & bit) delta.removed.push(o.raw);
          else if (r.bits & bit) delta.added.push(r.raw);
        }
        for (let k = 0; k < removedRecs.length; k++) if (removedRecs[k].bits & bit) delta.removed.push(removedRecs[k].raw);
        for (let k = 0; k < addedRecs.length; k++) if (addedRecs[k].bits & bit) delta.added.push(addedRecs[k].raw);
        if (delta.replaced.length + delta.removed.length + delta.added.length <= MAX_PATCH) {
          out = old.slice();
          for (let k = 0; k < delta.replaced.length && out !== null; k++) {
            const idx = out.indexOf(delta.replaced[k][0]);
            if (idx < 0) out = null;
            else out[idx] = delta.replaced[k][1];
          }
          for (let k = 0; k < delta.removed.length && out !== null; k++) {
            const idx = out.indexOf(delta.removed[k]);
            if (idx < 0) out = null;
            else out.splice(idx, 1);
          }
          for (let k = 0; k < delta.added.length && out !== null; k++) insertOrdered(out, delta.added[k]);
        }
        if (out === null) delta = null;
      }
      if (out === null) {
        out = [];
        for (let i = 0; i < recs.length; i++) if (recs[i].bits & bit) out.push(recs[i].raw);
        stats.subsetRebuilds++;
      } else stats.subsetPatches++;
      let same = old.length === out.length;
      for (let i = 0; same && i < out.length; i++) same = old[i] === out[i];
      if (same) continue;
      subsets[b] = out;
      changed[b] = true;
      deltas[b] = delta;
    }
    return { subsets: subsets, changed: changed, deltas: deltas };
  }

  /** The first non-empty list: classify each object, build the subsets, defer the records. */
  function firstLoad(list, changed, deltas) {
    gen++;
    const n = list.length;
    const raws = new Array(n);
    const bits = new Uint32Array(n);
    for (let i = 0; i < n; i++) {
      const raw = unwrapKubeObject(list[i]);
      raws[i] = raw;
      bits[i] = keyOf(raw) === null ? 0 : classify(raw);
    }
    pending = { raws: raws, bits: bits, gen: gen };
    prevItems = list;
    prevRec = [];
    for (let b = 0; b < nSub; b++) {
      const bit = 1 << b;
      const out = [];
      for (let i = 0; i < n; i++) if (bits[i] & bit) out.push(raws[i]);
      stats.subsetRebuilds++;
      if (out.length === 0 && subsets[b].length === 0) continue;
      subsets[b] = out;
      changed[b] = true;
    }
    return { subsets: subsets, changed: changed, deltas: deltas };
  }

  function reset() {
    pending = null;
    byKey = new Map();
    prevItems = [];
    prevRec = [];
    subsets = [];
    for (let b = 0; b < nSub; b++) subsets.push([]);
  }

  return {
    update: update,
    reset: reset,
    /** Current subsets (same identities as the last update returned). */
    subsets: function () { return subsets; },
    /** List position of an object of the current list (-1 when absent). */
    positionOf: positionOf,
    /** Counters: updates, objects classified, reused by lookup, skipped by compare, subset patches / rebuilds. */
    stats: function () { return Object.assign({}, stats); },
  };
}
