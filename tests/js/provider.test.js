/**
 * Provider core (src/api/providerCore.js) specs that need the harness React
 * (tests/js/stubs/react.js) or fake timers: STALE_MS revalidation, the
 * auto-refresh poller, the metrics back-off and the cold Node detail's
 * periodic re-read, plus the pure list-result reader. Everything that only
 * renders and reads text, requests and context values is runner-agnostic
 * and lives in tests/js/shared/provider.shared.test.js, which also runs on
 * real React 18 in CI.
 */
import React, { render } from './stubs/react.js';
import * as lib from './stubs/headlamp-lib.js';
import { PROMETHEUS_FORBIDDEN, PROMETHEUS_UNREACHABLE, STALE_MS, createProviderCore, listResult } from '../../src/api/providerCore.js';
import { resetSharedStores } from '../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH, PLUGIN_POD_QUERIES } from '../../src/api/k8sCore.js';
import { DEFAULT_SETTINGS } from '../../src/api/settings.js';
import { makeDeviceConfig, makeGpuPod } from './fixtures.js';

const h = React.createElement;

function kubeList(items) {
  return { kind: 'List', apiVersion: 'v1', metadata: {}, items: items };
}

function notFound() {
  return Promise.reject(Object.assign(new Error('404 page not found'), { status: 404 }));
}

function apiServer(o) {
  const opt = Object.assign({ dcs: [makeDeviceConfig()], pluginPods: [] }, o || {});
  return vi.fn((path) => {
    if (path === DEVICE_CONFIG_LIST_PATH) return Promise.resolve(kubeList(opt.dcs));
    if (PLUGIN_POD_QUERIES.indexOf(path) >= 0) return Promise.resolve(kubeList(opt.pluginPods));
    if (opt.prom) return opt.prom(path);
    return notFound();
  });
}

function crdCalls(request) {
  return request.mock.calls.filter((c) => c[0] === DEVICE_CONFIG_LIST_PATH).length;
}

let settings;

function core(request) {
  return createProviderCore(React, lib, {
    request: request,
    clusterKey: () => 'test-cluster',
    loadSettings: () => settings,
  });
}

function probe(c) {
  function Probe() {
    const ctx = c.useAmdGpuContext();
    return h('div', null, ctx.loading ? 'loading' : 'nodes=' + ctx.gpuNodes.length);
  }
  return { Probe };
}

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  settings = Object.assign({}, DEFAULT_SETTINGS);
});

afterEach(() => {
  vi.useRealTimers();
});

describe('listResult', () => {
  it('loading, errors array, tuple', () => {
    expect(listResult(undefined)).toEqual([null, null]);
    expect(listResult([null, null])).toEqual([null, null]);
    expect(listResult([[1], 'e'])).toEqual([[1], 'e']);
    expect(listResult({ items: [], isLoading: true })).toEqual([null, null]);
    expect(listResult({ items: null, errors: ['pods is forbidden'] })).toEqual([null, 'pods is forbidden']);
    expect(listResult({ items: [1], errors: [] })).toEqual([[1], null]);
  });
});

describe('AmdGpuDataProvider — timers', () => {
  it('a remount after STALE_MS revalidates once', async () => {
    vi.useFakeTimers();
    const request = apiServer();
    const c = core(request);
    const p1 = probe(c);
    const r1 = render(h(c.AmdGpuDataProvider, null, h(p1.Probe)));
    await r1.settle();
    r1.unmount();
    vi.setSystemTime(Date.now() + STALE_MS + 1);
    const p2 = probe(c);
    const r2 = render(h(c.AmdGpuDataProvider, null, h(p2.Probe)));
    await r2.settle();
    expect(crdCalls(request)).toBe(2);
  });

  it('auto-refresh (settings) revalidates on the poller period', async () => {
    vi.useFakeTimers();
    settings.refreshIntervalSec = 15;
    const request = apiServer();
    const c = core(request);
    const p = probe(c);
    const r = render(h(c.AmdGpuDataProvider, null, h(p.Probe)));
    await r.settle();
    expect(crdCalls(request)).toBe(1);
    await vi.advanceTimersByTimeAsync(15000);
    await r.settle();
    expect(crdCalls(request)).toBe(2);
    r.unmount();
    await vi.advanceTimersByTimeAsync(60000);
    expect(crdCalls(request)).toBe(2);
  });
});

describe('metrics hooks — auto-refresh back-off', () => {
  function metricsProbe(useHook) {
    const seen = [];
    function M() {
      const m = useHook();
      seen.push(m);
      return h('div', null, m.fetching ? 'fetching' : m.fetchError || 'idle');
    }
    return { M, seen, last: () => seen[seen.length - 1] };
  }

  for (const [why, fail, text] of [
    ['unreachable', () => Promise.reject(new Error('503')), PROMETHEUS_UNREACHABLE],
    ['refused (403)', () => Promise.reject(Object.assign(new Error('forbidden'), { status: 403 })), PROMETHEUS_FORBIDDEN],
  ]) {
  it('useGpuMetrics auto-refresh backs off while Prometheus is ' + why, async () => {
    vi.useFakeTimers();
    settings.refreshIntervalSec = 10;
    const request = apiServer({ prom: fail });
    const c = core(request);
    const mp = metricsProbe(() => c.useGpuMetrics(true, false));
    const r = render(h(mp.M));
    await r.settle();
    const fetches = () => mp.seen.filter((m, i) => m.fetching && (i === 0 || !mp.seen[i - 1].fetching)).length;
    expect(fetches()).toBe(1);
    for (let i = 0; i < 30; i++) {
      await vi.advanceTimersByTimeAsync(10000);
      await r.settle();
    }
    // 30 ticks of 10 s: without back-off 30 more fetches; with it one per 1 + 2 + 4 + 8 + 8 ... ticks
    expect(fetches()).toBeGreaterThan(2);
    expect(fetches()).toBeLessThanOrEqual(7);
    expect(mp.last().fetchError).toBe(text);
    r.unmount();
  });
  }
});

describe('useNodePods (cold Node detail) — a scoped list + watch', () => {
  it('follows the watch: pods scheduled later show up; a re-list or a failed watch keeps what is shown', async () => {
    const c = core(vi.fn(() => notFound()));
    let renders = 0;
    function S() {
      renders++;
      const np = c.useNodePods('n1');
      const res = np[0];
      return h('div', null, np[1], res.loading ? 'loading' : res.podsState + ':' + res.gpuPods.map((p) => p.metadata.name).join(','));
    }
    lib.lists.Pod = [[makeGpuPod('a', { node: 'n1' }), makeGpuPod('b', { node: 'n2' })], null];
    const r = render(h(S));
    await r.settle();
    expect(r.text()).toBe('ready:a');
    expect(lib.lists.calls.Pod[0]).toEqual({ namespace: '', fieldSelector: 'spec.nodeName=n1' });
    lib.lists.Pod = [[makeGpuPod('a', { node: 'n1' }), makeGpuPod('c', { node: 'n1' })], null];
    r.rerender(h(S));
    await r.settle();
    expect(r.text()).toBe('ready:a,c');
    lib.lists.Pod = [null, null]; // the host re-lists
    r.rerender(h(S));
    await r.settle();
    expect(r.text()).toBe('ready:a,c');
    lib.lists.Pod = [null, 'watch closed'];
    r.rerender(h(S));
    await r.settle();
    expect(r.text()).toBe('ready:a,c');
    expect(renders).toBeLessThan(12);
    r.unmount();
  });
});
