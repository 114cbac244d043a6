/**
 * Runner-agnostic specs of the provider core (src/api/providerCore.js): the
 * context contract, requests on mount and refresh, list classification,
 * degraded RBAC, the metrics hooks and the cold Node detail's pod read.
 * They run on the harness React offline and on real React 18 + react-dom in
 * networked CI (see plugin.shared.test.js for the two tiers); the specs that
 * need fake timers or harness internals stay in tests/js/provider.test.js.
 * Mirrors the reference's provider specs (src/api/IntelGpuDataContext.test.tsx:46-176:
 * outside-provider throw, request issuing, CRD absent vs present).
 */
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import { OUTSIDE_PROVIDER, PROMETHEUS_UNREACHABLE, createProviderCore } from '../../../src/api/providerCore.js';
import { resetSharedStores } from '../../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH, PLUGIN_POD_QUERIES } from '../../../src/api/k8sCore.js';
import { DEFAULT_SETTINGS } from '../../../src/api/settings.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../fixtures.js';
import { BASE0, exporterData, prom } from '../promFake.js';

const h = React.createElement;

function kubeList(items) {
  return { kind: 'List', apiVersion: 'v1', metadata: {}, items: items };
}

function notFound() {
  return Promise.reject(Object.assign(new Error('404 page not found'), { status: 404 }));
}

/** API server fake: CRD → `dcs` (or `crd` handler), plugin-pod queries → `pluginPods`. */
function apiServer(o) {
  const opt = Object.assign({ dcs: [makeDeviceConfig()], pluginPods: [] }, o || {});
  return vi.fn((path) => {
    if (path === DEVICE_CONFIG_LIST_PATH) return opt.crd ? opt.crd() : Promise.resolve(kubeList(opt.dcs));
    if (PLUGIN_POD_QUERIES.indexOf(path) >= 0) return Promise.resolve(kubeList(opt.pluginPods));
    if (opt.prom) return opt.prom(path);
    return notFound();
  });
}

const crdCalls = (request) => request.mock.calls.filter((c) => c[0] === DEVICE_CONFIG_LIST_PATH).length;

let settings;

function core(request) {
  return createProviderCore(React, lib, {
    request: request,
    clusterKey: () => 'test-cluster',
    loadSettings: () => settings,
  });
}

/** A consumer that records every context value it renders with. */
function probe(c) {
  const seen = [];
  function Probe() {
    const ctx = c.useAmdGpuContext();
    seen.push(ctx);
    return h('div', null, ctx.loading ? 'loading' : 'nodes=' + ctx.gpuNodes.length + ' pods=' + ctx.gpuPods.length);
  }
  return { Probe, seen, last: () => seen[seen.length - 1] };
}

function mount(c, p) {
  return render(h(c.AmdGpuDataProvider, null, h(p.Probe)));
}

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  settings = Object.assign({}, DEFAULT_SETTINGS);
});

describe('shared: createProviderCore (' + tier + ')', () => {
  it('requires the React hooks it uses', () => {
    expect(() => createProviderCore({ createElement: React.createElement }, lib)).toThrow('React.createContext is required');
  });
  it('checks useRef up front (the metrics hooks keep their back-off flag in a ref)', () => {
    const noRef = Object.assign({}, React);
    delete noRef.useRef;
    expect(() => createProviderCore(noRef, lib)).toThrow('React.useRef is required');
  });
});

describe('shared: useAmdGpuContext (' + tier + ')', () => {
  it('throws outside a provider', () => {
    const c = core(apiServer());
    const { Probe } = probe(c);
    expect(() => render(h(Probe))).toThrow(OUTSIDE_PROVIDER);
  });

  it('exposes the reference context contract inside a provider', async () => {
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    const ctx = p.last();
    ['deviceConfigs', 'pluginInstalled', 'gpuNodes', 'gpuPods', 'pluginPods', 'crdAvailable', 'loading', 'error'].forEach((k) =>
      expect(ctx).toHaveProperty(k)
    );
    expect(typeof ctx.refresh).toBe('function');
    r.unmount();
  });
});

describe('shared: AmdGpuDataProvider requests (' + tier + ')', () => {
  it('issues exactly one CRD request on mount while the pod watch is in flight', async () => {
    const request = apiServer();
    const c = core(request);
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(request).toHaveBeenCalledTimes(1);
    expect(request.mock.calls[0][0]).toBe(DEVICE_CONFIG_LIST_PATH);
    expect(p.last().crdAvailable).toBe(true);
    expect(p.last().deviceConfigs).toHaveLength(1);
    r.unmount();
  });

  it('asks Headlamp for nodes and for pods in all namespaces', async () => {
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    expect(lib.lists.calls.Node[0]).toBeNull();
    expect(lib.lists.calls.Pod[0]).toEqual({ namespace: '' });
    await r.settle();
    r.unmount();
  });

  it('a second provider mounted at the same time adds no request', async () => {
    const request = apiServer();
    const c = core(request);
    const a = probe(c);
    const b = probe(c);
    const r = render(h('div', null, h(c.AmdGpuDataProvider, null, h(a.Probe)), h(c.AmdGpuDataProvider, null, h(b.Probe))));
    await r.settle();
    expect(crdCalls(request)).toBe(1);
    expect(a.last().deviceConfigs).toBe(b.last().deviceConfigs);
    r.unmount();
  });

  it('a remount within STALE_MS renders the cached data at once with no request', async () => {
    const request = apiServer();
    lib.lists.Node = [[makeGpuNode('mi355x-0')], null];
    lib.lists.Pod = [[makeGpuPod('train-a')], null];
    const c = core(request);
    const p1 = probe(c);
    const r1 = mount(c, p1);
    await r1.settle();
    r1.unmount();
    expect(crdCalls(request)).toBe(1);

    const p2 = probe(c);
    const r2 = mount(c, p2);
    expect(p2.seen[0].loading).toBe(false);
    expect(p2.seen[0].deviceConfigs).toHaveLength(1);
    expect(r2.text()).toBe('nodes=1 pods=1');
    await r2.settle();
    expect(crdCalls(request)).toBe(1);
    r2.unmount();
  });

  it('refresh() re-fetches the CRD only (the pod list comes from the watch)', async () => {
    const request = apiServer();
    lib.lists.Pod = [[makePlainPod('web-0')], null];
    const c = core(request);
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    const before = request.mock.calls.length;
    r.act(() => p.last().refresh());
    await r.settle();
    expect(request.mock.calls.length).toBe(before + 1);
    expect(request.mock.calls[before][0]).toBe(DEVICE_CONFIG_LIST_PATH);
    r.unmount();
  });
});

describe('shared: AmdGpuDataProvider data (' + tier + ')', () => {
  it('classifies the useList nodes and pods', async () => {
    lib.lists.Node = [[makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1'), makeNode('cpu-0')], null];
    lib.lists.Pod = [[makeGpuPod('train-a'), makePlainPod('web-0'), makePluginPod('amdgpu-dp-1')], null];
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().gpuNodes.map((n) => n.metadata.name)).toEqual(['mi355x-0', 'mi355x-1']);
    expect(p.last().gpuPods.map((x) => x.metadata.name)).toEqual(['train-a']);
    expect(p.last().pluginPods.map((x) => x.metadata.name)).toEqual(['amdgpu-dp-1']);
    expect(r.text()).toBe('nodes=2 pods=1');
    r.unmount();
  });

  it('reads the object form of a list result ({items, errors, isLoading}) as well as the tuple', async () => {
    lib.lists.Node = { items: [makeGpuNode('mi355x-0'), makeNode('cpu-0')], errors: null, isLoading: false };
    lib.lists.Pod = { items: [makeGpuPod('train-a')], error: null, isLoading: false };
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().loading).toBe(false);
    expect(p.last().gpuNodes.map((n) => n.metadata.name)).toEqual(['mi355x-0']);
    expect(p.last().gpuPods.map((x) => x.metadata.name)).toEqual(['train-a']);
    r.unmount();
  });

  it('unwraps Headlamp KubeObject wrappers (jsonData)', async () => {
    lib.lists.Node = [[{ jsonData: makeGpuNode('mi355x-0') }], null];
    lib.lists.Pod = [[{ jsonData: makeGpuPod('train-a') }], null];
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().gpuNodes[0].metadata.name).toBe('mi355x-0');
    expect(p.last().gpuPods[0].metadata.name).toBe('train-a');
    r.unmount();
  });

  it('stays loading while the lists are in flight, then settles', async () => {
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().loading).toBe(true);
    expect(r.text()).toBe('loading');
    lib.lists.Node = [[makeGpuNode('mi355x-0')], null];
    lib.lists.Pod = [[], null];
    r.rerender(h(c.AmdGpuDataProvider, null, h(p.Probe)));
    await r.settle();
    expect(p.last().loading).toBe(false);
    r.unmount();
  });

  it('a watch event on an unrelated pod keeps the GPU pod list identity', async () => {
    const gpu = makeGpuPod('train-a');
    lib.lists.Node = [[makeGpuNode('mi355x-0')], null];
    lib.lists.Pod = [[gpu, makePlainPod('web-0')], null];
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    const before = p.last().gpuPods;
    lib.lists.Pod = [[gpu, makePlainPod('web-0'), makePlainPod('web-1')], null];
    r.rerender(h(c.AmdGpuDataProvider, null, h(p.Probe)));
    await r.settle();
    expect(p.last().gpuPods).toBe(before);
    r.unmount();
  });

  it('CRD 404 → crdAvailable false, no error', async () => {
    const c = core(apiServer({ crd: notFound }));
    lib.lists.Node = [[], null];
    lib.lists.Pod = [[], null];
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().crdAvailable).toBe(false);
    expect(p.last().error).toBeNull();
    expect(p.last().loading).toBe(false);
    r.unmount();
  });

  it('a transient CRD failure after a success keeps the last known DeviceConfigs', async () => {
    let fail = false;
    const crd = () => (fail ? Promise.reject(Object.assign(new Error('503'), { status: 503 })) : Promise.resolve(kubeList([makeDeviceConfig()])));
    const c = core(apiServer({ crd }));
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    fail = true;
    r.act(() => p.last().refresh());
    await r.settle();
    expect(p.last().crdAvailable).toBe(true);
    expect(p.last().deviceConfigs).toHaveLength(1);
    r.unmount();
  });
});

describe('shared: AmdGpuDataProvider under degraded RBAC (' + tier + ')', () => {
  it('pods forbidden: leaves loading, reports the error, finds operator pods by query', async () => {
    const request = apiServer({ pluginPods: [makePluginPod('amdgpu-dp-1')] });
    lib.lists.Node = [[makeGpuNode('mi355x-0')], null];
    lib.lists.Pod = [null, new Error('pods is forbidden')];
    const c = core(request);
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().loading).toBe(false);
    expect(p.last().error).toContain('pods is forbidden');
    expect(p.last().pluginPods.map((x) => x.metadata.name)).toEqual(['amdgpu-dp-1']);
    PLUGIN_POD_QUERIES.forEach((q) => expect(request.mock.calls.map((x) => x[0])).toContain(q));
    r.unmount();
  });

  it('nodes forbidden: leaves loading with no GPU nodes and the error', async () => {
    lib.lists.Node = [null, new Error('nodes is forbidden')];
    lib.lists.Pod = [[makeGpuPod('train-a')], null];
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().loading).toBe(false);
    expect(p.last().gpuNodes).toEqual([]);
    expect(p.last().error).toContain('nodes is forbidden');
    r.unmount();
  });

  it('both forbidden: leaves loading and reports both errors', async () => {
    lib.lists.Node = [null, 'nodes is forbidden'];
    lib.lists.Pod = [null, 'pods is forbidden'];
    const c = core(apiServer());
    const p = probe(c);
    const r = mount(c, p);
    await r.settle();
    expect(p.last().loading).toBe(false);
    expect(p.last().error).toContain('nodes is forbidden');
    expect(p.last().error).toContain('pods is forbidden');
    r.unmount();
  });
});

describe('shared: metrics hooks (' + tier + ')', () => {
  function metricsProbe(useHook) {
    const seen = [];
    function M() {
      const m = useHook();
      seen.push(m);
      return h('div', null, m.fetching ? 'fetching' : m.fetchError || (m.metrics ? 'gpus=' + m.metrics.gpus.length : 'idle'));
    }
    return { M, seen, last: () => seen[seen.length - 1] };
  }

  it('useGpuMetrics: Prometheus unreachable → the reference error text', async () => {
    const request = apiServer({ prom: () => Promise.reject(new Error('503')) });
    const c = core(request);
    const mp = metricsProbe(() => c.useGpuMetrics(true, false));
    const r = render(h(mp.M));
    expect(mp.last().fetching).toBe(true);
    await r.settle();
    expect(mp.last().fetching).toBe(false);
    expect(mp.last().fetchError).toBe(PROMETHEUS_UNREACHABLE);
    expect(r.text()).toBe(PROMETHEUS_UNREACHABLE);
    r.unmount();
  });

  it('useGpuMetrics: exporter reachable → per-GPU metrics and series', async () => {
    const request = apiServer({ prom: prom() });
    const c = core(request);
    const mp = metricsProbe(() => c.useGpuMetrics(true, true));
    const r = render(h(mp.M));
    await r.settle();
    expect(mp.last().fetchError).toBeNull();
    expect(mp.last().metrics.gpus).toHaveLength(8);
    expect(mp.last().series.power.n0.length).toBeGreaterThan(1);
    expect(request.mock.calls.every((x) => x[0].indexOf(BASE0) === 0)).toBe(true);
    expect(r.text()).toBe('gpus=8');
    r.unmount();
  });

  it('useGpuMetrics: refresh() fetches again; discovery is cached', async () => {
    const request = apiServer({ prom: prom() });
    const c = core(request);
    const mp = metricsProbe(() => c.useGpuMetrics(true, false));
    const r = render(h(mp.M));
    await r.settle();
    const n = request.mock.calls.length;
    const probes = () => request.mock.calls.filter((x) => x[0].indexOf('query=1') >= 0).length;
    const p0 = probes();
    r.act(() => mp.last().refresh());
    await r.settle();
    expect(request.mock.calls.length).toBeGreaterThan(n);
    expect(probes()).toBe(p0);
    r.unmount();
  });

  it('useNodeGpuMetrics(null) fetches nothing', async () => {
    const request = apiServer({ prom: prom() });
    const c = core(request);
    const mp = metricsProbe(() => c.useNodeGpuMetrics(null, true));
    const r = render(h(mp.M));
    await r.settle();
    expect(request).not.toHaveBeenCalled();
    expect(r.text()).toBe('idle');
    r.unmount();
  });

  it('useNodeGpuMetrics(node) reads one node through a hostname-scoped query', async () => {
    const request = apiServer({ prom: prom() });
    const c = core(request);
    const mp = metricsProbe(() => c.useNodeGpuMetrics('n0', true));
    const r = render(h(mp.M));
    await r.settle();
    expect(mp.last().metrics.gpus).toHaveLength(8);
    const scoped = request.mock.calls.filter((x) => decodeURIComponent(x[0]).indexOf('hostname="n0"') >= 0);
    expect(scoped.length).toBeGreaterThan(0);
    r.unmount();
  });

  it('switching node while a fetch is in flight drops the old answer', async () => {
    let release;
    const gate = new Promise((res) => (release = res));
    const inner = prom({ data: exporterData(['n0', 'n1']) });
    const slow = (path) => decodeURIComponent(path).indexOf('hostname="n0"') >= 0;
    const request = apiServer({ prom: (path) => (slow(path) ? gate.then(() => inner(path)) : inner(path)) });
    const c = core(request);
    let node = 'n0';
    const mp = metricsProbe(() => c.useNodeGpuMetrics(node, true));
    const r = render(h(mp.M));
    await r.settle();
    node = 'n1';
    r.rerender(h(mp.M));
    await r.settle();
    expect(mp.last().metrics.gpus[0].nodeName).toBe('n1');
    release();
    await r.settle();
    expect(mp.last().metrics.gpus.every((g) => g.nodeName === 'n1')).toBe(true);
    r.unmount();
  });

  it('useGpuOwners fetches pod attribution only', async () => {
    const request = apiServer({ prom: prom() });
    const c = core(request);
    const mp = metricsProbe(() => c.useGpuOwners());
    const r = render(h(mp.M));
    await r.settle();
    expect(mp.last().fetchError).toBeNull();
    const qs = request.mock.calls.map((x) => decodeURIComponent(x[0])).filter((q) => q.indexOf('query=') >= 0 && q.indexOf('query=1') < 0);
    expect(qs.length).toBeGreaterThan(0);
    qs.forEach((q) => expect(q).toContain('pod!=""'));
    r.unmount();
  });
});

describe('shared: useNodePods, the cold Node detail read (' + tier + ')', () => {
  function Section(c, node) {
    return function S() {
      const np = c.useNodePods(node);
      const r = np[0];
      return h('div', null, np[1], r.loading ? 'loading'
        : r.podsState + ':' + r.gpuPods.map((p) => p.metadata.name).join(',') + (r.podsSeeded ? ' (seeded)' : ''));
    };
  }

  /** The scoped request of one node's pods, answered from lib.lists.Pod as an apiserver would. */
  function nodePodsServer() {
    return vi.fn((path) => {
      const m = /^\/api\/v1\/pods\?fieldSelector=(.*)$/.exec(path);
      if (!m) return notFound();
      const node = decodeURIComponent(m[1]).replace(/^spec\.nodeName=/, '');
      return Promise.resolve(kubeList((lib.lists.Pod[0] || []).filter((p) => p.spec && p.spec.nodeName === node)));
    });
  }

  it('one list + watch scoped to the node (the host hook), GPU pods of that node only, no request of its own', async () => {
    const request = vi.fn(() => notFound());
    lib.lists.Pod = [[makeGpuPod('a', { node: 'n1' }), makeGpuPod('b', { node: 'n2' }), makePlainPod('web')], null];
    const r = render(h(Section(core(request), 'n1')));
    await r.settle();
    expect(r.text()).toBe('ready:a');
    expect(lib.lists.calls.Pod.every((o) => o.fieldSelector === 'spec.nodeName=n1' && o.namespace === '')).toBe(true);
    expect(request).not.toHaveBeenCalled();
    r.unmount();
  });

  it('loading until the list is in; a first failure says the pods are unreadable', async () => {
    lib.lists.Pod = [null, null];
    const S = Section(core(vi.fn(() => notFound())), 'n1');
    const r = render(h(S));
    await r.settle();
    expect(r.text()).toBe('loading');
    lib.lists.Pod = [null, 'pods is forbidden'];
    r.rerender(h(S));
    await r.settle();
    expect(r.text()).toBe('error:');
    r.unmount();
  });

  it('the store\'s last pod list (no feed mounted) seeds the first paint; the node\'s own list then replaces it', async () => {
    const c = core(vi.fn(() => notFound()));
    const store = c.storeFor(c.clusterKey());
    store.setPods([makeGpuPod('old', { node: 'n1' }), makeGpuPod('x', { node: 'n2' })], null);
    lib.lists.Pod = [null, null];
    const S = Section(c, 'n1');
    const r = render(h(S));
    // the store's list can be of any age: the context says these pods are seeded, not current
    expect(r.text()).toBe('ready:old (seeded)');
    lib.lists.Pod = [[makeGpuPod('new', { node: 'n1' })], null];
    r.rerender(h(S));
    await r.settle();
    expect(r.text()).toBe('ready:new');
    r.unmount();
  });

  it('a host that ignores the field selector: counted, the watch unmounted, the field-selected request read instead', async () => {
    const request = nodePodsServer();
    const c = core(request);
    lib.lists.ignoreOptions = true;
    lib.lists.Pod = [[makeGpuPod('a', { node: 'n1' }), makeGpuPod('b', { node: 'n2' }), makePlainPod('web', { node: 'n2' })], null];
    const S = Section(c, 'n1');
    const r = render(h(S));
    await r.settle();
    expect(r.text()).toBe('ready:a');
    expect(c.storeFor(c.clusterKey()).counters().selectorIgnored).toEqual({ nodePods: 2, operatorPods: 0 });
    expect(request.mock.calls.map((x) => x[0])).toEqual(['/api/v1/pods?fieldSelector=' + encodeURIComponent('spec.nodeName=n1')]);
    // No list hook is mounted any more: a re-render calls none.
    lib.lists.calls.Pod.length = 0;
    r.rerender(h(S));
    await r.settle();
    expect(lib.lists.calls.Pod).toHaveLength(0);
    expect(r.text()).toBe('ready:a');
    // A later section on this cluster reads the request from the start.
    r.unmount();
    const r2 = render(h(Section(c, 'n2')));
    await r2.settle();
    expect(lib.lists.calls.Pod).toHaveLength(0);
    expect(r2.text()).toBe('ready:b');
    r2.unmount();
  });
});

describe('shared: the operator pods on a host that ignores list options (' + tier + ')', () => {
  const OPS = { nodes: false, pods: false, crd: true, operatorPods: true };

  it('the operator pod feed is swapped for the plugin-pod requests: same pods, no unscoped list left mounted', async () => {
    const dp = makePluginPod('amdgpu-dp-0');
    const all = [dp, makePlainPod('web-0'), makeGpuPod('train-a')];
    lib.lists.ignoreOptions = true;
    lib.lists.Pod = [all, null];
    const request = apiServer({ pluginPods: [dp] });
    const c = core(request);
    const p = probe(c);
    const r = render(h(c.AmdGpuDataProvider, { needs: OPS }, h(p.Probe)));
    await r.settle();
    const counters = c.storeFor(c.clusterKey()).counters();
    expect(counters.selectorIgnored.operatorPods).toBeGreaterThan(0);
    expect(p.last().pluginPods.map((x) => x.metadata.name)).toEqual(['amdgpu-dp-0']);
    expect(request.mock.calls.filter((x) => PLUGIN_POD_QUERIES.indexOf(x[0]) >= 0).length).toBe(PLUGIN_POD_QUERIES.length);
    lib.lists.calls.Pod.length = 0;
    r.rerender(h(c.AmdGpuDataProvider, { needs: OPS }, h(p.Probe)));
    await r.settle();
    expect(lib.lists.calls.Pod).toHaveLength(0);
    expect(p.last().pluginPods.map((x) => x.metadata.name)).toEqual(['amdgpu-dp-0']);
    r.unmount();
  });

  it('a host that applies the options is not flagged', async () => {
    lib.lists.Pod = [[makePluginPod('amdgpu-dp-0'), makePlainPod('web-0')], null];
    const c = core(apiServer());
    const p = probe(c);
    const r = render(h(c.AmdGpuDataProvider, { needs: OPS }, h(p.Probe)));
    await r.settle();
    expect(c.storeFor(c.clusterKey()).counters().selectorIgnored).toBeNull();
    expect(lib.lists.calls.Pod.length).toBeGreaterThan(0);
    r.unmount();
  });
});
