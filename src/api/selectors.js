/**
 * What a list request's options select, evaluated on the client: the
 * namespace, the label selector (`k=v`, `k==v`, `k!=v`, `k in (a,b)`,
 * `k notin (a,b)`, `k`, `!k`) and the field selector (`path=v`, `path==v`,
 * `path!=v`) of Headlamp's `useList(opts)`.
 *
 * The apiserver applies these options; the plugin checks its scoped lists
 * against them only to notice a host that did NOT pass them on (an older
 * Headlamp whose `useList()` drops its argument, ADR 012): such a list
 * comes back with objects outside the selection, and the view then reads
 * its scoped request instead of a cluster-wide watch. The reference only
 * ever passes `{namespace: ''}` (src/api/IntelGpuDataContext.tsx:99), so it
 * has nothing to check.
 */

/** Terms of a selector, split on the commas outside parentheses. */
function terms(sel) {
  const out = [];
  let depth = 0;
  let cur = '';
  for (let i = 0; i < sel.length; i++) {
    const ch = sel[i];
    if (ch === '(') depth++;
    else if (ch === ')') depth--;
    if (ch === ',' && depth === 0) {
      if (cur.trim()) out.push(cur.trim());
      cur = '';
    } else cur += ch;
  }
  if (cur.trim()) out.push(cur.trim());
  return out;
}

const SET_TERM = /^([A-Za-z0-9_./-]+)\s+(in|notin)\s+\(([^)]*)\)$/;

function labelTerm(t) {
  const set = SET_TERM.exec(t);
  if (set) {
    const vals = set[3].split(',').map(function (v) { return v.trim(); }).filter(Boolean);
    const want = set[2] === 'in';
    return function (l) { return (Object.prototype.hasOwnProperty.call(l, set[1]) && vals.indexOf(l[set[1]]) >= 0) === want; };
  }
  const ne = t.indexOf('!=');
  if (ne > 0) {
    const k = t.slice(0, ne).trim();
    const v = t.slice(ne + 2).trim();
    return function (l) { return l[k] !== v; };
  }
  const eq = t.indexOf('=');
  if (eq > 0) {
    const k = t.slice(0, eq).trim();
    const v = t.slice(t.charAt(eq + 1) === '=' ? eq + 2 : eq + 1).trim();
    return function (l) { return l[k] === v; };
  }
  if (t.charAt(0) === '!') {
    const k = t.slice(1).trim();
    return function (l) { return !Object.prototype.hasOwnProperty.call(l, k); };
  }
  return function (l) { return Object.prototype.hasOwnProperty.call(l, t); };
}

function fieldTerm(t) {
  const neg = t.indexOf('!=');
  const eq = neg >= 0 ? neg : t.indexOf('=');
  const path = t.slice(0, eq).trim().split('.');
  const skip = neg >= 0 ? 2 : t.charAt(eq + 1) === '=' ? 2 : 1;
  const want = t.slice(eq + skip).trim();
  return function (o) {
    let cur = o;
    for (let i = 0; i < path.length && cur !== undefined && cur !== null; i++) cur = cur[path[i]];
    const v = cur === undefined || cur === null ? '' : String(cur);
    return neg >= 0 ? v !== want : v === want;
  };
}

/**
 * A predicate over raw objects for list options `opts` ({namespace,
 * labelSelector, fieldSelector}), or null when they select every object
 * (none, or all namespaces without selectors).
 * @param {{namespace?: string, labelSelector?: string, fieldSelector?: string}|null|undefined} opts
 * @returns {((raw: any) => boolean)|null}
 */
export function listSelection(opts) {
  if (!opts) return null;
  const ns = typeof opts.namespace === 'string' && opts.namespace !== '' ? opts.namespace : null;
  const ls = typeof opts.labelSelector === 'string' && opts.labelSelector.trim() ? terms(opts.labelSelector).map(labelTerm) : null;
  const fs = typeof opts.fieldSelector === 'string' && opts.fieldSelector.trim() ? terms(opts.fieldSelector).map(fieldTerm) : null;
  if (!ns && !ls && !fs) return null;
  return function (raw) {
    const m = (raw && raw.metadata) || {};
    if (ns && m.namespace !== ns) return false;
    if (ls) {
      const labels = m.labels && typeof m.labels === 'object' ? m.labels : {};
      for (let i = 0; i < ls.length; i++) if (!ls[i](labels)) return false;
    }
    if (fs) for (let i = 0; i < fs.length; i++) if (!fs[i](raw)) return false;
    return true;
  };
}

/**
 * How many of `items` (raw objects) lie outside what `opts` selects: 0 for a
 * host that applied the options (or options selecting everything).
 */
export function countOutside(items, opts) {
  const sel = listSelection(opts);
  if (!sel || !items) return 0;
  let n = 0;
  for (let i = 0; i < items.length; i++) if (!sel(items[i])) n++;
  return n;
}
