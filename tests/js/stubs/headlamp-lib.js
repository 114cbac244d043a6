/**
 * '@kinvolk/headlamp-plugin/lib' stand-in for the Node-12 harness: records
 * every registration call and lets a spec script what `useList()` and
 * `ApiProxy.request()` return (the reference mocks the same surface with
 * vi.mock, src/api/IntelGpuDataContext.test.tsx:7-15).
 */

export const registry = { sidebar: [], routes: [], details: [], columns: [], settings: [] };

export const lists = {
  // [items, error]; items null = still loading
  Node: [null, null],
  Pod: [null, null],
  calls: { Node: [], Pod: [] },
  selected: {},
  // A host whose useList() drops its options (an older Headlamp): every list
  // holds every object, whatever namespace / selector was asked for.
  ignoreOptions: false,
};

export const api = {
  calls: [],
  handler: function () { return Promise.reject(Object.assign(new Error('no handler'), { status: 404 })); },
};

export function resetHeadlamp() {
  registry.sidebar.length = 0;
  registry.routes.length = 0;
  registry.details.length = 0;
  registry.columns.length = 0;
  registry.settings.length = 0;
  lists.Node = [null, null];
  lists.Pod = [null, null];
  lists.calls.Node.length = 0;
  lists.calls.Pod.length = 0;
  lists.selected = {};
  lists.ignoreOptions = false;
  api.calls.length = 0;
  api.handler = function () { return Promise.reject(Object.assign(new Error('no handler'), { status: 404 })); };
}

export function registerSidebarEntry(e) { registry.sidebar.push(e); }
export function registerRoute(r) { registry.routes.push(r); }
export function registerDetailsViewSection(f) { registry.details.push(f); }
export function registerResourceTableColumnsProcessor(f) { registry.columns.push(f); }
export function registerPluginSettings(name, component, showSave) { registry.settings.push({ name: name, component: component, showSave: showSave }); }

/** Terms of a selector string, split on the commas outside parentheses. */
function terms(sel) {
  const out = [];
  let depth = 0;
  let cur = '';
  for (let i = 0; i < sel.length; i++) {
    const ch = sel[i];
    if (ch === '(') depth++;
    if (ch === ')') depth--;
    if (ch === ',' && depth === 0) {
      out.push(cur.trim());
      cur = '';
    } else cur += ch;
  }
  if (cur.trim()) out.push(cur.trim());
  return out;
}

/** `key in (a,b)`, `key=v` and `key!=v` terms of a label selector, as a predicate over labels. */
function labelPredicate(sel) {
  const preds = terms(sel).map(function (t) {
    const set = /^([^\s!=]+)\s+(in|notin)\s+\((.*)\)$/.exec(t);
    if (set) {
      const vals = set[3].split(',').map(function (v) { return v.trim(); });
      return function (l) { return (vals.indexOf(l[set[1]]) >= 0) === (set[2] === 'in'); };
    }
    const ne = t.split('!=');
    if (ne.length === 2) return function (l) { return l[ne[0].trim()] !== ne[1].trim(); };
    const eq = t.split('=');
    return function (l) { return l[eq[0].trim()] === eq[eq.length - 1].trim(); };
  });
  return function (labels) { return preds.every(function (p) { return p(labels || {}); }); };
}

/** `path=v` / `path!=v` terms of a field selector (spec.nodeName, metadata.namespace, ...). */
function fieldPredicate(sel) {
  const preds = terms(sel).map(function (t) {
    const neg = t.indexOf('!=') >= 0;
    const kv = neg ? t.split('!=') : t.split('=');
    const path = kv[0].trim().split('.');
    const want = kv[kv.length - 1].trim();
    return function (o) {
      let cur = o;
      for (let i = 0; i < path.length && cur !== undefined && cur !== null; i++) cur = cur[path[i]];
      const v = cur === undefined || cur === null ? '' : String(cur);
      return neg ? v !== want : v === want;
    };
  });
  return function (o) { return preds.every(function (p) { return p(o); }); };
}

/**
 * What the list options select, as a predicate over raw objects, or null for
 * every object (no options, or all namespaces without selectors).
 */
function selection(opts) {
  if (!opts) return null;
  const ns = typeof opts.namespace === 'string' && opts.namespace !== '' ? opts.namespace : null;
  const ls = typeof opts.labelSelector === 'string' && opts.labelSelector ? labelPredicate(opts.labelSelector) : null;
  const fs = typeof opts.fieldSelector === 'string' && opts.fieldSelector ? fieldPredicate(opts.fieldSelector) : null;
  if (!ns && !ls && !fs) return null;
  return function (raw) {
    const m = (raw && raw.metadata) || {};
    if (ns && m.namespace !== ns) return false;
    if (ls && !ls(m.labels)) return false;
    if (fs && !fs(raw)) return false;
    return true;
  };
}

function resourceClass(kind) {
  return {
    useList: function (opts) {
      lists.calls[kind].push(opts === undefined ? null : opts);
      // A namespaced or selected list holds what the apiserver would return
      // for it (identity kept while the underlying list is unchanged).
      const pred = lists.ignoreOptions ? null : selection(opts);
      const res = lists[kind];
      if (pred === null || !res || !Array.isArray(res[0])) return res;
      const sig = JSON.stringify(opts);
      const cache = lists.selected[kind] || (lists.selected[kind] = {});
      if (!cache[sig] || cache[sig].from !== res) {
        const items = res[0].filter(function (o) { return pred(o && o.jsonData ? o.jsonData : o); });
        cache[sig] = { from: res, value: [items, res[1]] };
      }
      return cache[sig].value;
    },
  };
}

export const K8s = { ResourceClasses: { Node: resourceClass('Node'), Pod: resourceClass('Pod') } };

export const ApiProxy = {
  request: function (path) {
    api.calls.push(path);
    return api.handler(path);
  },
};
