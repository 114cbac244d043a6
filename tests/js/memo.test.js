/**
 * Structural sharing + view memoisation: unchanged inputs → identical IR
 * objects (what React.memo and renderSection's cache rely on); changed
 * inputs → recomputed sections.
 */
import { createMemo, sections } from '../../src/view/ir.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { podDetailView } from '../../src/view/pages/details.js';
import { metricsView } from '../../src/view/pages/metricsPage.js';
import { nodesView } from '../../src/view/pages/nodes.js';
import { overviewView } from '../../src/view/pages/overview.js';
import { podsView } from '../../src/view/pages/pods.js';
import { renderSection } from '../../src/view/html.js';
import { createClusterStore, sameObjects } from '../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH, PLUGIN_POD_QUERIES } from '../../src/api/k8sCore.js';
import { NOW, makeContext, makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from './fixtures.js';

describe('createMemo', () => {
  it('returns the cached value while deps are identical', () => {
    const memo = createMemo(4);
    const a = {};
    const f = vi.fn(() => ({ v: 1 }));
    const x = memo('k', [a, 1], f);
    expect(memo('k', [a, 1], f)).toBe(x);
    expect(f).toHaveBeenCalledTimes(1);
  });
  it('recomputes when any dep changes', () => {
    const memo = createMemo(4);
    const f = vi.fn(() => ({}));
    memo('k', [{}], f);
    memo('k', [{}], f);
    expect(f).toHaveBeenCalledTimes(2);
  });
  it('evicts the oldest slot beyond its limit', () => {
    const memo = createMemo(2);
    memo('a', [], () => 1);
    memo('b', [], () => 2);
    memo('c', [], () => 3);
    expect(memo.size()).toBe(2);
  });
});

describe('view memoisation', () => {
  beforeEach(() => clearViewMemo());

  it('overview returns the same sections for the same snapshot data', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0' })] });
    const a = overviewView(ctx, { now: NOW });
    const b = overviewView(Object.assign({}, ctx, { refreshing: true }), { now: NOW + 200 });
    expect(b.items).toBe(a.items);
    expect(b.refresh.label).toBe('Refreshing…');
  });

  it('recomputes when an age label it shows changes, not on every clock tick', () => {
    // A running pod started 10 s ago: "10s" turns "11s" one second later.
    const young = makeGpuPod('a', { node: 'g0' });
    young.metadata.creationTimestamp = new Date(NOW - 10000).toISOString();
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [young] });
    const a = overviewView(ctx, { now: NOW });
    expect(overviewView(ctx, { now: NOW + 500 }).items).toBe(a.items);
    const b = overviewView(ctx, { now: NOW + 1000 });
    expect(b.items).not.toBe(a.items);
    expect(JSON.stringify(b)).toContain('"11s"');
  });

  it('holds a section whose ages only show hours until the next hour of age', () => {
    // Node and pods an hour old or more: no label changes for a while.
    const old = makeGpuPod('a', { node: 'g0' });
    old.metadata.creationTimestamp = new Date(NOW - 3600 * 1000).toISOString();
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [old] });
    const a = podsView(ctx, { now: NOW });
    expect(podsView(ctx, { now: NOW + 59 * 60 * 1000 }).items).toBe(a.items);
    const b = podsView(ctx, { now: NOW + 3600 * 1000 });
    expect(b.items).not.toBe(a.items);
    expect(JSON.stringify(b)).toContain('"2h"');
  });

  it('does not reuse a section for an earlier clock', () => {
    const young = makeGpuPod('a', { node: 'g0' });
    young.metadata.creationTimestamp = new Date(NOW - 10000).toISOString();
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [young] });
    const a = podsView(ctx, { now: NOW });
    expect(podsView(ctx, { now: NOW - 2000 }).items).not.toBe(a.items);
  });

  it('recomputes when the pod list changes', () => {
    const ctx = makeContext({ pods: [makeGpuPod('a')] });
    const a = podsView(ctx, { now: NOW });
    const ctx2 = makeContext({ pods: [makeGpuPod('a'), makeGpuPod('b')] });
    expect(podsView(ctx2, { now: NOW }).items).not.toBe(a.items);
  });

  it('reuses unchanged node cards and rebuilds changed ones', () => {
    const n0 = makeGpuNode('g0');
    const n1 = makeGpuNode('g1');
    const ctx = makeContext({ nodes: [n0, n1] });
    const a = sections(nodesView(ctx, { now: NOW }));
    const metrics = { gpus: [], xgmi: { g1: { '0-1': 12.5 } } };
    const b = sections(nodesView(ctx, { now: NOW, metrics }));
    const card = (ss, name) => ss.find((s) => s.title === name);
    expect(card(b, 'g0')).toBe(card(a, 'g0'));
    expect(card(b, 'g1')).not.toBe(card(a, 'g1'));
  });

  it('keeps node cards when only telemetry values change, not ownership', () => {
    const n0 = makeGpuNode('g0');
    const ctx = makeContext({ nodes: [n0] });
    const gpu = (power) => ({ nodeName: 'g0', gpu: '0', pod: 'train', namespace: 'ml', powerWatts: power });
    const a = sections(nodesView(ctx, { now: NOW, metrics: { gpus: [gpu(900)], xgmi: {}, links: {} } }));
    const b = sections(nodesView(ctx, { now: NOW, metrics: { gpus: [gpu(1200)], xgmi: {}, links: {} } }));
    expect(b.find((s) => s.title === 'g0')).toBe(a.find((s) => s.title === 'g0'));
    const c = sections(nodesView(ctx, { now: NOW, metrics: { gpus: [Object.assign(gpu(1200), { pod: 'eval' })], xgmi: {}, links: {} } }));
    expect(c.find((s) => s.title === 'g0')).not.toBe(a.find((s) => s.title === 'g0'));
  });

  it('metrics page reuses a node section while its GPU objects are reused', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')] });
    const g = { nodeName: 'g0', gpu: '0', pod: null, namespace: null, powerWatts: 900, powerCapWatts: 1400,
      vramUsedBytes: 1, vramTotalBytes: 2, gfxActivityPct: 50, memActivityPct: 20, tempC: 60 };
    const m1 = { source: 'amd-exporter', gpus: [g], xgmi: {}, links: {}, fetchedAt: new Date(NOW).toISOString() };
    const m2 = Object.assign({}, m1, { fetchedAt: new Date(NOW + 5000).toISOString() });
    const find = (vm) => sections(vm).find((s) => s.title.indexOf('g0 — ') === 0);
    const a = find(metricsView(ctx, { metrics: m1, fetchError: null, fetching: false }, { now: NOW }));
    const b = find(metricsView(ctx, { metrics: m2, fetchError: null, fetching: false }, { now: NOW }));
    expect(b).toBe(a);
  });

  it('metrics page: a watch event (new context, same snapshot) rebuilds none of its sections; a new snapshot rebuilds the summary', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')] });
    const g = { nodeName: 'g0', gpu: '0', pod: null, namespace: null, powerWatts: 900, powerCapWatts: 1400,
      vramUsedBytes: 1, vramTotalBytes: 2, gfxActivityPct: 50, memActivityPct: 20, tempC: 60 };
    const m1 = { source: 'amd-exporter', gpus: [g], xgmi: {}, links: {}, fetchedAt: new Date(NOW).toISOString() };
    const series = { rangeSec: 1800, power: { g0: [[1, 900], [2, 950]] }, vram: { g0: [[1, 1], [2, 1]] } };
    const st = { metrics: m1, series, fetchError: null, fetching: false };
    const a = sections(metricsView(ctx, st, { now: NOW }));
    const b = sections(metricsView(Object.assign({}, ctx), st, { now: NOW + 1000 }));
    expect(a.map((s) => s.title)).toEqual(['Metric Availability', 'GPU Power Summary', 'Power & HBM (last 30 min)', 'g0 — 1 × MI355X']);
    b.forEach((s, i) => expect(s).toBe(a[i]));
    const m2 = Object.assign({}, m1, { fetchedAt: new Date(NOW + 5000).toISOString() });
    const c = sections(metricsView(ctx, Object.assign({}, st, { metrics: m2 }), { now: NOW }));
    expect(c[1]).not.toBe(a[1]);
    expect(c[2]).toBe(a[2]); // same series window
    expect(c[3]).toBe(a[3]); // same GPU objects
  });

  it('pod detail sections are cached per pod object', () => {
    const p = makeGpuPod('p');
    expect(podDetailView(p)).toBe(podDetailView({ jsonData: p }));
  });

  it('renderSection reuses HTML for the same section object', () => {
    const s = podDetailView(makeGpuPod('q'));
    const h = renderSection(s);
    expect(renderSection(s)).toBe(h);
  });
});

describe('structural sharing in the store', () => {
  it('keeps the GPU pod / node lists when only unrelated pods change', () => {
    const store = createClusterStore({ request: () => Promise.resolve({ items: [] }) });
    const g = makeGpuPod('train', { node: 'g0' });
    const n = makeGpuNode('g0');
    store.setNodes([n], null);
    store.setPods([g, makePlainPod('web-1')], null);
    const a = store.getSnapshot();
    store.setPods([g, makePlainPod('web-2'), makePlainPod('web-3')], null);
    store.setNodes([n, makeNode('cpu-9')], null);
    const b = store.getSnapshot();
    expect(b.gpuPods).toBe(a.gpuPods);
    expect(b.gpuNodes).toBe(a.gpuNodes);
    expect(b.index).toBe(a.index);
  });

  it('sameObjects compares uid + resourceVersion', () => {
    const a = [{ metadata: { uid: 'x', resourceVersion: '1' } }];
    expect(sameObjects(a, [{ metadata: { uid: 'x', resourceVersion: '1' } }])).toBe(true);
    expect(sameObjects(a, [{ metadata: { uid: 'x', resourceVersion: '2' } }])).toBe(false);
    expect(sameObjects(a, [])).toBe(false);
  });
  it('sameObjects falls back to deep comparison without resourceVersion', () => {
    expect(sameObjects([makeDeviceConfig('a')], [makeDeviceConfig('a')])).toBe(true);
    expect(sameObjects([makeDeviceConfig('a')], [makeDeviceConfig('b')])).toBe(false);
  });
  it('keeps list identity across refreshes that return unchanged objects', async () => {
    const request = (path) => {
      if (path === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ items: [makeDeviceConfig()] });
      if (path === PLUGIN_POD_QUERIES[0]) return Promise.resolve({ items: [makePluginPod('dp')] });
      return Promise.resolve({ items: [] });
    };
    const store = createClusterStore({ request });
    await store.refresh();
    const a = store.getSnapshot();
    await store.refresh();
    const b = store.getSnapshot();
    expect(b).not.toBe(a);
    expect(b.deviceConfigs).toBe(a.deviceConfigs);
    expect(b.pluginPods).toBe(a.pluginPods);
  });
});
