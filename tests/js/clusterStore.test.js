/**
 * Data-layer specs (analog of reference src/api/IntelGpuDataContext.test.tsx,
 * 8 cases) plus the parallel-fetch, SWR, race and shared-cache behaviour the
 * reference lacks.
 */
import fs from 'fs';
import { createClusterStore, fetchNodePods, getSharedStore, nodePodsPath, resetSharedStores, withTimeout } from '../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH, PLUGIN_POD_QUERIES } from '../../src/api/k8sCore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod, NOW } from './fixtures.js';
import { nodeDetailView } from '../../src/view/pages/details.js';
import { metricsView } from '../../src/view/pages/metricsPage.js';
import { rowValue, text } from '../../src/view/ir.js';

function deferred() {
  let resolve;
  let reject;
  const promise = new Promise((a, b) => {
    resolve = a;
    reject = b;
  });
  return { promise, resolve, reject };
}

/** request() stub answering by path. */
function router(table) {
  return vi.fn((path) => {
    const h = table[path];
    if (h === undefined) return Promise.reject(new Error('404 ' + path));
    return typeof h === 'function' ? h(path) : Promise.resolve(h);
  });
}

function baseRoutes(extra) {
  const r = {};
  r[DEVICE_CONFIG_LIST_PATH] = { items: [makeDeviceConfig()] };
  r[PLUGIN_POD_QUERIES[0]] = { items: [makePluginPod('dp-0'), makePluginPod('dp-1')] };
  r[PLUGIN_POD_QUERIES[1]] = { items: [makePluginPod('dp-0'), makePlainPod('other')] };
  r['/api/v1/nodes'] = { items: [makeGpuNode('mi355x-0'), makeNode('cpu-0')] };
  r['/api/v1/pods'] = { items: [makeGpuPod('train-0'), makePlainPod('web')] };
  return Object.assign(r, extra || {});
}

describe('withTimeout', () => {
  it('resolves with the value and clears its timer', async () => {
    vi.useFakeTimers();
    const v = await withTimeout(Promise.resolve(7), 2000);
    expect(v).toBe(7);
    expect(vi.getTimerCount()).toBe(0);
    vi.useRealTimers();
  });
  it('rejects after the deadline', async () => {
    vi.useFakeTimers();
    const p = withTimeout(new Promise(() => {}), 2000);
    vi.advanceTimersByTime(2000);
    await expect(p).rejects.toThrow('Request timed out after 2000ms');
    vi.useRealTimers();
  });
});

describe('createClusterStore', () => {
  it('requires a request function', () => {
    expect(() => createClusterStore({})).toThrow('request(path) is required');
  });

  it('is loading until nodes, pods and the first refresh arrive', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    expect(store.getSnapshot().loading).toBe(true);
    store.setNodes([], null);
    store.setPods([], null);
    expect(store.getSnapshot().loading).toBe(true);
    await store.refresh();
    expect(store.getSnapshot().loading).toBe(false);
  });

  it('filters GPU nodes and pods from Headlamp KubeObject wrappers', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes([{ jsonData: makeGpuNode('g0') }, { jsonData: makeNode('c0') }], null);
    store.setPods([{ jsonData: makeGpuPod('p0', { node: 'g0' }) }, { jsonData: makePlainPod('x') }], null);
    const s = store.getSnapshot();
    expect(s.gpuNodes.map((n) => n.metadata.name)).toEqual(['g0']);
    expect(s.gpuPods.map((p) => p.metadata.name)).toEqual(['p0']);
    expect(s.index.nodeStats.get('g0').inUse).toBe(1);
  });

  it('issues the CRD and every plugin-pod query concurrently', async () => {
    const gates = {};
    const request = vi.fn((path) => {
      gates[path] = deferred();
      return gates[path].promise;
    });
    const store = createClusterStore({ request });
    const done = store.refresh();
    // All three requests are in flight before any of them resolves.
    expect(request).toHaveBeenCalledTimes(1 + PLUGIN_POD_QUERIES.length);
    Object.keys(gates).forEach((k) => gates[k].resolve({ items: [] }));
    await done;
    expect(store.getSnapshot().crdAvailable).toBe(true);
  });

  it('derives operator pods from the pod list once it is in: a refresh is one request', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    store.setPods([makePluginPod('dp-0'), makePluginPod('dp-1'), makePlainPod('web')], null);
    await store.refresh();
    expect(request).toHaveBeenCalledTimes(1);
    expect(request.mock.calls[0][0]).toBe(DEVICE_CONFIG_LIST_PATH);
    const s = store.getSnapshot();
    expect(s.pluginPods.map((p) => p.metadata.name).sort()).toEqual(['dp-0', 'dp-1']);
    expect(s.pluginInstalled).toBe(true);
  });

  it('does not query operator pods while the pod list is pending', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    await Promise.all([store.loadLists(), store.refresh()]);
    const paths = request.mock.calls.map((c) => c[0]).sort();
    expect(paths).toEqual(['/api/v1/nodes', '/api/v1/pods', DEVICE_CONFIG_LIST_PATH].sort());
    expect(store.getSnapshot().loading).toBe(false);
  });

  it('falls back to the plugin-pod requests when the pod list fails', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    store.setPods(null, 'pods is forbidden');
    await store.refresh();
    const s = store.getSnapshot();
    expect(s.pluginPods.map((p) => p.metadata.name).sort()).toEqual(['dp-0', 'dp-1']);
    expect(s.error).toContain('pods is forbidden');
    expect(request.mock.calls.map((c) => c[0])).toContain(PLUGIN_POD_QUERIES[1]);
  });

  it('keeps the derived operator-pod list identity while it is unchanged', () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    const dp = makePluginPod('dp-0');
    store.setPods([dp, makePlainPod('a')], null);
    const a = store.getSnapshot().pluginPods;
    store.setPods([dp, makePlainPod('b')], null);
    expect(store.getSnapshot().pluginPods).toBe(a);
  });

  it('keeps the last DeviceConfigs through a transient CRD failure, clears them on 404', async () => {
    const r = baseRoutes();
    const request = router(r);
    const store = createClusterStore({ request });
    await store.refresh();
    const before = store.getSnapshot().deviceConfigs;
    const fail = (status) => () => Promise.reject(Object.assign(new Error('HTTP ' + status), { status }));
    r[DEVICE_CONFIG_LIST_PATH] = fail(503);
    await store.refresh();
    expect(store.getSnapshot().crdAvailable).toBe(true);
    expect(store.getSnapshot().deviceConfigs).toBe(before);
    r[DEVICE_CONFIG_LIST_PATH] = fail(404);
    await store.refresh();
    expect(store.getSnapshot().crdAvailable).toBe(false);
    expect(store.getSnapshot().deviceConfigs).toHaveLength(0);
  });

  it('sets crdAvailable and deviceConfigs from the CRD list', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    await store.refresh();
    const s = store.getSnapshot();
    expect(s.crdAvailable).toBe(true);
    expect(s.deviceConfigs).toHaveLength(1);
    expect(s.deviceConfigs[0].metadata.name).toBe('gpu-operator');
    expect(s.pluginInstalled).toBe(true);
  });

  it('drops non-DeviceConfig items from the CRD list', async () => {
    const r = baseRoutes();
    r[DEVICE_CONFIG_LIST_PATH] = { items: [makeDeviceConfig(), { kind: 'Other', metadata: { name: 'x' } }] };
    const store = createClusterStore({ request: router(r) });
    await store.refresh();
    expect(store.getSnapshot().deviceConfigs).toHaveLength(1);
  });

  it('degrades silently when the CRD is missing', async () => {
    const r = baseRoutes();
    delete r[DEVICE_CONFIG_LIST_PATH];
    const store = createClusterStore({ request: router(r) });
    await store.refresh();
    const s = store.getSnapshot();
    expect(s.crdAvailable).toBe(false);
    expect(s.deviceConfigs).toHaveLength(0);
    expect(s.error).toBeNull();
    expect(s.pluginInstalled).toBe(true); // found via pods
  });

  it('treats a CRD timeout as missing and does not wait for it', async () => {
    vi.useFakeTimers();
    const r = baseRoutes();
    r[DEVICE_CONFIG_LIST_PATH] = () => new Promise(() => {});
    const store = createClusterStore({ request: router(r), timeoutMs: 2000 });
    let settled = false;
    const p = store.refresh().then(() => {
      settled = true;
    });
    await vi.advanceTimersByTimeAsync(1999);
    expect(settled).toBe(false);
    await vi.advanceTimersByTimeAsync(1);
    await p;
    expect(store.getSnapshot().crdAvailable).toBe(false);
    expect(vi.getTimerCount()).toBe(0);
    vi.useRealTimers();
  });

  it('merges and dedupes plugin pods across queries', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    await store.refresh();
    expect(store.getSnapshot().pluginPods.map((p) => p.metadata.name)).toEqual(['dp-0', 'dp-1']);
  });

  it('ignores failing plugin-pod queries', async () => {
    const r = baseRoutes();
    delete r[PLUGIN_POD_QUERIES[0]];
    const store = createClusterStore({ request: router(r) });
    await store.refresh();
    expect(store.getSnapshot().pluginPods.map((p) => p.metadata.name)).toEqual(['dp-0']);
    expect(store.getSnapshot().error).toBeNull();
  });

  it('reports pluginInstalled=false when nothing is found', async () => {
    const store = createClusterStore({ request: router({}) });
    await store.refresh();
    expect(store.getSnapshot().pluginInstalled).toBe(false);
  });

  it('keeps data visible while a refresh is in flight (stale-while-revalidate)', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes([], null);
    store.setPods([], null);
    await store.refresh();
    const p = store.refresh();
    const mid = store.getSnapshot();
    expect(mid.loading).toBe(false);
    expect(mid.refreshing).toBe(true);
    expect(mid.deviceConfigs).toHaveLength(1);
    await p;
    expect(store.getSnapshot().refreshing).toBe(false);
  });

  it('drops results of a superseded refresh', async () => {
    const first = deferred();
    let calls = 0;
    const request = vi.fn((path) => {
      if (path === DEVICE_CONFIG_LIST_PATH) {
        calls++;
        return calls === 1 ? first.promise : Promise.resolve({ items: [makeDeviceConfig('new')] });
      }
      return Promise.resolve({ items: [] });
    });
    const store = createClusterStore({ request });
    const a = store.refresh();
    const b = store.refresh();
    await b;
    first.resolve({ items: [makeDeviceConfig('old')] });
    await a;
    expect(store.getSnapshot().deviceConfigs[0].metadata.name).toBe('new');
  });

  it('refresh re-issues the imperative requests', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    await store.refresh();
    const n = request.mock.calls.length;
    await store.refresh();
    expect(request.mock.calls.length).toBe(2 * n);
  });

  it('aggregates node, pod and async errors', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes(null, 'nodes forbidden');
    store.setPods(null, 'pods forbidden');
    expect(store.getSnapshot().error).toBe('nodes forbidden; pods forbidden');
  });

  it('memoises filters on input identity', () => {
    const store = createClusterStore({ request: router({}) });
    const nodes = [makeGpuNode('g')];
    store.setNodes(nodes, null);
    const a = store.getSnapshot().gpuNodes;
    store.setPods([], null);
    expect(store.getSnapshot().gpuNodes).toBe(a);
  });

  it('notifies subscribers and supports unsubscribe', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    const fn = vi.fn();
    const off = store.subscribe(fn);
    store.setNodes([], null);
    expect(fn).toHaveBeenCalledTimes(1);
    off();
    store.setPods([], null);
    expect(fn).toHaveBeenCalledTimes(1);
  });

  it('snapshots are immutable and versioned', () => {
    const store = createClusterStore({ request: router({}) });
    const a = store.getSnapshot();
    store.setNodes([], null);
    const b = store.getSnapshot();
    expect(a).not.toBe(b);
    expect(b.version).toBeGreaterThan(a.version);
    expect(Object.isFrozen(b)).toBe(true);
  });

  it('loadLists fetches nodes and pods directly', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    await Promise.all([store.loadLists(), store.refresh()]);
    const s = store.getSnapshot();
    expect(s.loading).toBe(false);
    expect(s.gpuNodes).toHaveLength(1);
    expect(s.gpuPods).toHaveLength(1);
  });

  it('loadLists surfaces list errors', async () => {
    const store = createClusterStore({ request: router({}) });
    await store.loadLists();
    expect(store.getSnapshot().error).toContain('404 /api/v1/nodes');
  });

  it('emits a trace span per request', async () => {
    const spans = [];
    const store = createClusterStore({ request: router(baseRoutes()), onTrace: (s) => spans.push(s) });
    await store.refresh();
    expect(spans.map((s) => s.name).sort()).toEqual(['crd', 'plugin-pods-0', 'plugin-pods-1']);
    expect(spans.every((s) => s.end >= s.start && s.ok)).toBe(true);
  });
});

describe('degraded RBAC: an errored list is settled, not loading', () => {
  const idle = { metrics: null, fetchError: null, fetching: false };
  const cases = [
    ['pods forbidden', (st) => { st.setNodes([makeGpuNode('mi355x-0')], null); st.setPods(null, 'pods is forbidden'); }],
    ['nodes forbidden', (st) => { st.setNodes(null, 'nodes is forbidden'); st.setPods([makeGpuPod('train-0')], null); }],
    ['both forbidden', (st) => { st.setNodes(null, 'nodes is forbidden'); st.setPods(null, 'pods is forbidden'); }],
  ];
  it.each(cases)('%s: loading clears after refresh', async (_name, feed) => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    feed(store);
    await store.refresh();
    const s = store.getSnapshot();
    expect(s.loading).toBe(false);
    expect(s.error).toContain('forbidden');
  });
  it.each(cases)('%s: the Metrics Refresh button is enabled', async (_name, feed) => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    feed(store);
    await store.refresh();
    const vm = metricsView(store.getSnapshot(), idle, { now: NOW });
    expect(vm.refresh.disabled).toBe(false);
    expect(vm.refresh.label).toBe('Refresh');
  });
  it.each(cases)('%s: Node detail does not say Loading…', async (_name, feed) => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    feed(store);
    await store.refresh();
    const snap = store.getSnapshot();
    const sec = nodeDetailView(makeGpuNode('mi355x-0'), snap, {});
    const pods = text(rowValue(sec, 'GPU Workload Pods'));
    expect(pods).not.toBe('Loading…');
    if (snap.podsState === 'error') {
      expect(pods).toContain('Unavailable');
      expect(rowValue(sec, 'GPU Allocation')).toBeUndefined();
    } else {
      expect(pods).toBe('train-0');
    }
  });
  it('a list still in flight keeps the page loading', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes(null, null);
    store.setPods([], null);
    await store.refresh();
    expect(store.getSnapshot().loading).toBe(true);
    expect(store.getSnapshot().nodesState).toBe('pending');
    store.setNodes([], null);
    expect(store.getSnapshot().loading).toBe(false);
  });
  it('a fresh list hook reporting "no items yet" keeps the list already held', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes([makeGpuNode('mi355x-0')], null);
    store.setPods([makeGpuPod('train-0')], null);
    await store.refresh();
    const before = store.getSnapshot();
    store.setNodes(null, null);
    store.setPods(null, null);
    const s = store.getSnapshot();
    expect(s).toBe(before);
    expect(s.loading).toBe(false);
    expect(s.gpuNodes).toHaveLength(1);
    expect(s.gpuPods).toHaveLength(1);
  });
  it('a refresh after the first load never brings the loader back', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes([], null);
    store.setPods([], null);
    await store.refresh();
    const p = store.refresh();
    expect(store.getSnapshot().loading).toBe(false);
    expect(store.getSnapshot().refreshing).toBe(true);
    await p;
  });
  it('a list that recovers from an error clears the error', async () => {
    const store = createClusterStore({ request: router(baseRoutes()) });
    store.setNodes([], null);
    store.setPods(null, 'pods is forbidden');
    await store.refresh();
    store.setPods([makeGpuPod('train-0')], null);
    const s = store.getSnapshot();
    expect(s.error).toBeNull();
    expect(s.podsState).toBe('ready');
    expect(s.gpuPods).toHaveLength(1);
  });
});

describe('revalidate', () => {
  it('joins an in-flight refresh instead of starting another', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    const a = store.refresh();
    const b = store.revalidate(0);
    expect(b).toBe(a);
    await a;
    expect(request).toHaveBeenCalledTimes(1 + PLUGIN_POD_QUERIES.length);
  });
  it('skips when data is fresh and refreshes when stale', async () => {
    let now = 1000;
    const request = router(baseRoutes());
    const store = createClusterStore({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    await store.revalidate(5000);
    const n = request.mock.calls.length;
    now += 1000;
    await store.revalidate(5000);
    expect(request.mock.calls.length).toBe(n);
    now += 10000;
    await store.revalidate(5000);
    expect(request.mock.calls.length).toBe(2 * n);
  });
});

describe('pod list feeds: operator pods from the watched list, else from the plugin-pod requests', () => {
  const ppNames = (store) => store.getSnapshot().pluginPods.map((p) => p.metadata.name).sort();
  const queried = (request) => request.mock.calls.filter((c) => PLUGIN_POD_QUERIES.indexOf(c[0]) >= 0).length;

  it('while a feed is mounted, a refresh is the CRD request alone and operator pods follow the list', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    const detach = store.attachPodFeed();
    store.setPods([makePluginPod('dp-live'), makePlainPod('web')], null);
    await store.refresh();
    expect(queried(request)).toBe(0);
    expect(ppNames(store)).toEqual(['dp-live']);
    expect(store.getSnapshot().pluginPodsLoading).toBe(false);
    detach();
  });

  it('after the last feed unmounts: the list\'s last word is kept, the next refresh asks the requests', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    const detach = store.attachPodFeed();
    store.setPods([makePluginPod('dp-live')], null);
    await store.refresh();
    detach();
    detach(); // idempotent
    expect(ppNames(store)).toEqual(['dp-live']);
    expect(store.getSnapshot().pluginPodsLoading).toBe(false);
    await store.refresh();
    expect(queried(request)).toBe(PLUGIN_POD_QUERIES.length);
    expect(ppNames(store)).toEqual(['dp-0', 'dp-1']);
  });

  it('a feed mounted again makes the list the source again, without re-querying', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    store.attachPodFeed()();
    store.setPods([makePluginPod('dp-live')], null);
    const detach = store.attachPodFeed();
    expect(ppNames(store)).toEqual(['dp-live']);
    await store.refresh();
    expect(queried(request)).toBe(0);
    detach();
  });

  it('revalidate asks for operator pods nobody knows even when the DeviceConfigs are fresh', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    const detach = store.attachPodFeed(); // the pod list never arrives before the route unmounts
    store.setPods(null, null); // what the feed reports while its list is in flight
    await store.refresh();
    expect(queried(request)).toBe(0);
    detach();
    expect(store.getSnapshot().pluginPodsLoading).toBe(true);
    await store.revalidate(60000);
    expect(queried(request)).toBe(PLUGIN_POD_QUERIES.length);
    expect(store.getSnapshot().pluginPodsLoading).toBe(false);
    expect(ppNames(store)).toEqual(['dp-0', 'dp-1']);
    await store.revalidate(60000); // now known and fresh: nothing more
    expect(request).toHaveBeenCalledTimes(2 + PLUGIN_POD_QUERIES.length);
  });

  it('an operator pod feed: its lists are the operator pods, a refresh is the CRD request alone', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    const detach = store.attachOperatorFeed();
    store.setOperatorPods(null, null);
    expect(store.getSnapshot().pluginPodsLoading).toBe(true);
    store.setOperatorPods([makePluginPod('dp-watched')], null);
    expect(store.getSnapshot().pluginPodsLoading).toBe(false);
    expect(ppNames(store)).toEqual(['dp-watched']);
    await store.refresh();
    expect(queried(request)).toBe(0);
    store.setOperatorPods(null, null); // a re-mounted list reporting "no items yet" keeps what is held
    expect(ppNames(store)).toEqual(['dp-watched']);
    detach();
    expect(ppNames(store)).toEqual(['dp-watched']); // kept as the last known answer
    await store.refresh(); // nothing watches them now
    expect(queried(request)).toBe(PLUGIN_POD_QUERIES.length);
  });

  it('both operator pod lists failing hand over to the plugin-pod requests', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    store.attachOperatorFeed();
    store.setOperatorPods(null, 'pods is forbidden');
    await new Promise((r) => setTimeout(r, 0));
    await store.settled();
    expect(queried(request)).toBe(PLUGIN_POD_QUERIES.length);
    expect(ppNames(store)).toEqual(['dp-0', 'dp-1']);
  });

  it('loadOperatorPods feeds the operator pod lists by their list requests', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    store.attachOperatorFeed();
    await Promise.all([store.loadOperatorPods(), store.refresh()]);
    expect(request).toHaveBeenCalledTimes(1 + PLUGIN_POD_QUERIES.length);
    expect(ppNames(store)).toEqual(['dp-0', 'dp-1']);
    expect(store.getSnapshot().pluginPodsLoading).toBe(false);
  });

  it('a store no feed ever attached to (harness, terminal client) treats setPods / loadLists as current', async () => {
    const request = router(baseRoutes());
    const store = createClusterStore({ request });
    await store.loadLists();
    await store.refresh();
    expect(queried(request)).toBe(0);
    expect(store.getSnapshot().pluginPodsLoading).toBe(false);
  });
});

describe('snapshot shape', () => {
  it('has exactly the fields src/api/types.ts declares for ClusterSnapshot (no tsc offline: this pins the drift)', async () => {
    const src = fs.readFileSync(new URL('../../src/api/types.ts', import.meta.url), 'utf8');
    const body = /export interface ClusterSnapshot \{([\s\S]*?)\n\}/.exec(src)[1];
    const declared = body.split('\n').map((l) => /^\s{2}(\w+)\??:/.exec(l)).filter(Boolean).map((m) => m[1]).sort();
    const store = createClusterStore({ request: router(baseRoutes()) });
    await store.refresh();
    expect(Object.keys(store.getSnapshot()).sort()).toEqual(declared);
  });
});

describe('getSharedStore', () => {
  it('returns one store per cluster key', () => {
    resetSharedStores();
    const f = vi.fn(() => createClusterStore({ request: router({}) }));
    const a = getSharedStore('c1', f);
    const b = getSharedStore('c1', f);
    const c = getSharedStore('c2', f);
    expect(a).toBe(b);
    expect(a).not.toBe(c);
    expect(f).toHaveBeenCalledTimes(2);
    resetSharedStores();
  });
});

describe('CRD refused vs absent', () => {
  it('a 403 on the DeviceConfig list sets crdForbidden; a 404 does not', async () => {
    for (const [st, forbidden] of [[403, true], [404, false]]) {
      const store = createClusterStore({
        request: () => Promise.reject(Object.assign(new Error('HTTP ' + st), { status: st })),
      });
      store.setNodes([], null);
      store.setPods([], null);
      await store.refresh();
      const snap = store.getSnapshot();
      expect(snap.crdAvailable).toBe(false);
      expect(snap.crdForbidden).toBe(forbidden);
      expect(snap.error).toBeNull();
    }
  });
});

describe('fetchNodePods', () => {
  function deferredRequest() {
    const calls = [];
    const pending = [];
    const request = (p) => {
      calls.push(p);
      return new Promise((resolve, reject) => pending.push({ resolve, reject }));
    };
    return { request, calls, pending };
  }

  it('callers asking for the same node while it is in flight share one request', async () => {
    const d = deferredRequest();
    const a = fetchNodePods(d.request, 'n1');
    const b = fetchNodePods(d.request, 'n1');
    const c = fetchNodePods(d.request, 'n2');
    expect(d.calls).toEqual([nodePodsPath('n1'), nodePodsPath('n2')]);
    d.pending[0].resolve({ kind: 'PodList', items: [makeGpuPod('p', { node: 'n1' })] });
    d.pending[1].resolve({ kind: 'PodList', items: [] });
    const [ra, rb, rc] = await Promise.all([a, b, c]);
    expect(ra).toHaveLength(1);
    expect(rb).toBe(ra);
    expect(rc).toEqual([]);
    // settled: the next read is a new request
    fetchNodePods(d.request, 'n1');
    expect(d.calls).toHaveLength(3);
  });

  it('a failure reaches every sharer and is not cached', async () => {
    const d = deferredRequest();
    const a = fetchNodePods(d.request, 'n1');
    const b = fetchNodePods(d.request, 'n1');
    d.pending[0].reject(Object.assign(new Error('403 Forbidden'), { status: 403 }));
    let errs = 0;
    await a.catch(() => { errs++; });
    await b.catch(() => { errs++; });
    expect(errs).toBe(2);
    fetchNodePods(d.request, 'n1');
    expect(d.calls).toHaveLength(2);
  });

  it('different request functions (clusters) do not share', () => {
    const d1 = deferredRequest();
    const d2 = deferredRequest();
    fetchNodePods(d1.request, 'n1');
    fetchNodePods(d2.request, 'n1');
    expect(d1.calls).toHaveLength(1);
    expect(d2.calls).toHaveLength(1);
  });
});
