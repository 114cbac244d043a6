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
  api.calls.length = 0;
  api.handler = function () { return Promise.reject(Object.assign(new Error('no handler'), { status: 404 })); };
}

export function registerSidebarEntry(e) { registry.sidebar.push(e); }
export function registerRoute(r) { registry.routes.push(r); }
export function registerDetailsViewSection(f) { registry.details.push(f); }
export function registerResourceTableColumnsProcessor(f) { registry.columns.push(f); }
export function registerPluginSettings(name, component, showSave) { registry.settings.push({ name: name, component: component, showSave: showSave }); }

/** `spec.nodeName=<n>` of a field selector, or null (the only selector the plugin sends). */
function selectedNode(opts) {
  const m = opts && typeof opts.fieldSelector === 'string' ? /^spec\.nodeName=(.*)$/.exec(opts.fieldSelector) : null;
  return m ? m[1] : null;
}

function resourceClass(kind) {
  return {
    useList: function (opts) {
      lists.calls[kind].push(opts === undefined ? null : opts);
      // A field-selected list holds what the apiserver would return for it:
      // the objects on that node (identity kept while the list is unchanged).
      const node = selectedNode(opts);
      const res = lists[kind];
      if (node === null || !res || !Array.isArray(res[0])) return res;
      if (!lists.selected[kind] || lists.selected[kind].from !== res || lists.selected[kind].node !== node) {
        const items = res[0].filter(function (o) {
          const raw = o && o.jsonData ? o.jsonData : o;
          return raw && raw.spec && raw.spec.nodeName === node;
        });
        lists.selected[kind] = { from: res, node: node, value: [items, res[1]] };
      }
      return lists.selected[kind].value;
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
