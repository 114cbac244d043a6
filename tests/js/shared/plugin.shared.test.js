/**
 * Runner-agnostic specs of the shipped React layer: every page route, both
 * detail sections, loading → data, the Refresh path, StrictMode and the
 * pager, asserted on rendered text, aria-labels and the requests sent.
 *
 * They import their render API from 'amd-test-harness' and nothing from the
 * harness React, so the same file runs
 *   * on the harness React (tests/js/harness/stub.js): `npm run test:node12`,
 *     `npm test` and the pytest bridge, offline;
 *   * on real React 18.3.1 + react-dom, offline: the UMD builds over a
 *     minimal DOM (tests/js/harness/umd.js; tests/test_js_real_react.py);
 *   * on real React 18 + react-dom in jsdom with @testing-library/react
 *     (tests/js/harness/dom.js): `npm run test:react`
 *     (vitest.react.config.mts), networked CI only.
 * Only '@kinvolk/headlamp-plugin/lib[/CommonComponents]' is mocked, as the
 * reference's component tests do (reference src/components/OverviewPage.test.tsx:8-61).
 * Assertions on harness internals (component instances, render counters)
 * live in the harness-only files (tests/js/plugin.test.js, react.test.js,
 * provider.test.js).
 */
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import '../../../src/index.tsx';
import { resetSharedStores } from '../../../src/api/clusterStore.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { DEFAULT_SETTINGS, invalidateSettings, saveSettings } from '../../../src/api/settings.js';
import { isAmdGpuPluginPod } from '../../../src/api/amdPods.js';
import { DEVICE_CONFIG_LIST_PATH, PLUGIN_POD_QUERIES } from '../../../src/api/k8sCore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../fixtures.js';
import { exporterData, prom } from '../promFake.js';

const h = React.createElement;

// Registration ran at import (src/index.tsx); keep it before any reset.
const reg = { routes: lib.registry.routes.slice(), details: lib.registry.details.slice() };

const nodeNames = (n) => Array.from({ length: n }, (_, i) => 'mi355x-' + String(i).padStart(3, '0'));

function route(path) {
  const r = reg.routes.find((x) => x.path === path);
  expect(r).toBeTruthy();
  return r.component;
}

/** A cluster: GPU + CPU nodes, GPU / plain / operator pods, one DeviceConfig, a Prometheus with exporter series. */
function cluster(o) {
  const opt = Object.assign({ gpuNodes: ['mi355x-000', 'mi355x-001'], loading: false }, o || {});
  const nodes = opt.gpuNodes.map((n) => makeGpuNode(n)).concat([makeNode('cpu-0')]);
  const pods = [
    makeGpuPod('train-a', { gpus: 4, node: opt.gpuNodes[0] }),
    makeGpuPod('train-b', { gpus: 2, node: opt.gpuNodes[1] || opt.gpuNodes[0] }),
    makePlainPod('web-0'),
    makePluginPod('amdgpu-dp-0'),
  ];
  lib.lists.Node = opt.loading ? [null, null] : [nodes, null];
  // podsLoading: the node list is in, the all-namespaces pod list still in flight.
  lib.lists.Pod = opt.loading || opt.podsLoading ? [null, null] : [pods, null];
  // nodeExporter: no exporter series, node-exporter's amdgpu hwmon chips instead (the fallback source).
  const fake = opt.nodeExporter ? prom({ data: {}, ne: nodeExporterData(opt.gpuNodes) }) : prom({ data: exporterData(opt.gpuNodes) });
  lib.api.handler = (path) => {
    if (path === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
    if (path.indexOf('/proxy/api/v1/') >= 0) return fake(path);
    const fs = /^\/api\/v1\/pods\?fieldSelector=(.*)$/.exec(path);
    if (fs) {
      const node = decodeURIComponent(fs[1]).replace(/^spec\.nodeName=/, '');
      return Promise.resolve({ kind: 'List', metadata: {}, items: pods.filter((p) => p.spec.nodeName === node) });
    }
    // The plugin-pod requests: operator pods by label across namespaces, and the operator namespace.
    const q = PLUGIN_POD_QUERIES.indexOf(path);
    if (q >= 0) {
      const items = pods.filter((p) => (q === 0 ? isAmdGpuPluginPod(p) && p.metadata.namespace !== 'kube-amd-gpu' : p.metadata.namespace === 'kube-amd-gpu'));
      return Promise.resolve({ kind: 'List', metadata: {}, items: items });
    }
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
  fake.pods = pods;
  return fake;
}

/** node-exporter series of GPU nodes: one amdgpu hwmon chip each, node_uname_info naming the node. */
function nodeExporterData(nodes) {
  const ne = { node_uname_info: [], node_hwmon_chip_names: [], node_hwmon_power_average_watt: [] };
  nodes.forEach((n, k) => {
    const inst = '10.0.0.' + (k + 1) + ':9100';
    ne.node_uname_info.push({ metric: { __name__: 'node_uname_info', instance: inst, nodename: n }, value: [0, '1'] });
    ne.node_hwmon_chip_names.push({ metric: { __name__: 'node_hwmon_chip_names', chip_name: 'amdgpu', instance: inst, chip: '0000:05:00_0' }, value: [0, '1'] });
    ne.node_hwmon_power_average_watt.push({ metric: { __name__: 'node_hwmon_power_average_watt', instance: inst, chip: '0000:05:00_0' }, value: [0, '650'] });
  });
  return ne;
}

/** A list hook call for every pod of the cluster (all namespaces, no selector). */
const allPods = (o) => !!o && o.namespace === '' && !o.labelSelector && !o.fieldSelector;

const crdCalls = () => lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH).length;
const promQueries = (fake) => fake.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => /\/query\?query=(?!1$)/.test(p));

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  clearViewMemo();
  invalidateSettings();
  // jsdom has a sessionStorage: the pages keep their pager state there (plugin.js usePager).
  if (typeof sessionStorage !== 'undefined' && sessionStorage) sessionStorage.clear();
});

describe('shared: every route mounts and renders its page (' + tier + ')', () => {
  const pages = [
    ['/amd-gpu', 'AMD GPU — Overview', 'GPU Nodes'],
    ['/amd-gpu/device-plugins', 'AMD GPU — Device Plugins', 'DeviceConfig: gpu-operator'],
    ['/amd-gpu/nodes', 'AMD GPU — Nodes', 'GPU Node Summary'],
    ['/amd-gpu/pods', 'AMD GPU — Pods', 'All GPU Pods'],
    ['/amd-gpu/metrics', 'AMD GPU — Metrics', 'GPU Power Summary'],
  ];
  pages.forEach(([path, title, section]) => {
    it(path + ' → "' + title + '" with "' + section + '"', async () => {
      cluster();
      const r = render(h(route(path)));
      await r.settle();
      expect(r.text()).toContain(title);
      expect(r.text()).toContain(section);
      r.unmount();
    });
  });

  it('shows the loader while the lists are loading, then no page header', async () => {
    cluster({ loading: true });
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    expect(r.text()).toContain('Loading AMD GPU data...');
    expect(r.text()).not.toContain('AMD GPU — Overview');
    r.unmount();
  });
});

describe('shared: progressive cold open — a page waits only for the lists it draws (' + tier + ')', () => {
  it('Metrics renders its telemetry while the pod list is still pending', async () => {
    cluster({ podsLoading: true });
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    expect(r.text()).toContain('AMD GPU — Metrics');
    expect(r.text()).toContain('GPU Power Summary');
    expect(r.text()).toContain('mi355x-000 — 8 × MI355X');
    expect(r.text()).not.toContain('Loading AMD GPU data...');
    r.unmount();
  });

  it('Metrics on a node-exporter-only cluster: the GPU cards from the first answer, one Prometheus query', async () => {
    // A Prometheus this session has not met (its client is keyed by the settings that shape it).
    saveSettings(Object.assign({}, DEFAULT_SETTINGS, { requestTimeoutMs: DEFAULT_SETTINGS.requestTimeoutMs + 1 }));
    const fake = cluster({ nodeExporter: true });
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    saveSettings(DEFAULT_SETTINGS);
    expect(r.text()).toContain('mi355x-000 — 1 × MI355X');
    expect(r.text()).toContain('mi355x-001 — 1 × MI355X');
    expect(r.text()).not.toContain('fetching telemetry');
    expect(r.text()).not.toContain('No AMD GPU Metrics in Prometheus');
    expect(promQueries(fake)).toHaveLength(1);
    r.unmount();
  });

  it('GPU Nodes renders its cards from the node list; the pod cells fill in when the pods arrive', async () => {
    const fake = cluster({ podsLoading: true });
    const r = render(h(route('/amd-gpu/nodes')));
    await r.settle();
    expect(r.text()).toContain('GPU Node Summary');
    expect(r.text()).toContain('Loading…');
    expect(r.text()).not.toContain('train-a');
    lib.lists.Pod = [fake.pods, null];
    r.rerender(h(route('/amd-gpu/nodes')));
    await r.settle();
    expect(r.text()).toContain('train-a');
    expect(r.text()).not.toContain('Loading…');
    r.unmount();
  });

  it('Overview shows nodes, capacity and DeviceConfigs first, a loader where the pods go', async () => {
    const fake = cluster({ podsLoading: true });
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    expect(r.text()).toContain('AMD GPU — Overview');
    expect(r.text()).toContain('Device Config Status');
    expect(r.text()).toContain('Total GPU Devices');
    expect(r.text()).toContain('Loading GPU pods...');
    expect(r.text()).not.toContain('Plugin Not Detected');
    expect(r.text()).not.toContain('GPU Workloads');
    lib.lists.Pod = [fake.pods, null];
    r.rerender(h(route('/amd-gpu')));
    await r.settle();
    expect(r.text()).toContain('GPU Workloads');
    expect(r.text()).toContain('Active GPU Pods');
    expect(r.text()).not.toContain('Loading GPU pods...');
    r.unmount();
  });

  it('Device Plugins watches the operator pods alone: no all-namespaces pod list, no node list, no plugin-pod requests', async () => {
    cluster();
    const r = render(h(route('/amd-gpu/device-plugins')));
    await r.settle();
    expect(r.text()).toContain('DeviceConfig: gpu-operator');
    expect(r.text()).toContain('amdgpu-dp-0');
    expect(r.text()).not.toContain('Loading operator pods...');
    expect(lib.lists.calls.Node).toHaveLength(0);
    expect(lib.lists.calls.Pod.some(allPods)).toBe(false);
    expect(lib.lists.calls.Pod.some((o) => o && o.namespace === 'kube-amd-gpu')).toBe(true);
    expect(lib.lists.calls.Pod.some((o) => o && o.labelSelector === 'name in (amdgpu-dp-ds,amdgpu-labeller-ds)')).toBe(true);
    expect(PLUGIN_POD_QUERIES.some((q) => lib.api.calls.indexOf(q) >= 0)).toBe(false);
    r.unmount();
  });

  it('Device Plugins: operator pods are live (a new one shows without Refresh) and Refresh is the DeviceConfig request alone', async () => {
    const fake = cluster();
    const r = render(h(route('/amd-gpu/device-plugins')));
    await r.settle();
    const n = lib.api.calls.length;
    lib.lists.Pod = [fake.pods.concat([makePluginPod('amdgpu-dp-1', { node: 'mi355x-001' })]), null];
    r.rerender(h(route('/amd-gpu/device-plugins')));
    await r.settle();
    expect(r.text()).toContain('amdgpu-dp-1');
    r.click(r.byLabel('Refresh device plugin data'));
    await r.settle();
    expect(lib.api.calls.slice(n)).toEqual([DEVICE_CONFIG_LIST_PATH]);
    r.unmount();
  });

  it('Device Plugins: the operator pod lists refused, the plugin-pod requests stand in', async () => {
    cluster();
    lib.lists.Pod = [null, 'pods is forbidden'];
    const r = render(h(route('/amd-gpu/device-plugins')));
    await r.settle();
    PLUGIN_POD_QUERIES.forEach((q) => expect(lib.api.calls).toContain(q));
    expect(r.text()).toContain('DeviceConfig: gpu-operator');
    expect(r.text()).not.toContain('Loading operator pods...');
    r.unmount();
  });

  it('Device Plugins after a page that watched every pod: the operator pods at once, no plugin-pod request', async () => {
    cluster();
    const r1 = render(h(route('/amd-gpu')));
    await r1.settle();
    r1.unmount();
    const r2 = render(h(route('/amd-gpu/device-plugins')));
    expect(r2.text()).toContain('amdgpu-dp-0');
    await r2.settle();
    expect(r2.text()).toContain('amdgpu-dp-0');
    expect(PLUGIN_POD_QUERIES.some((q) => lib.api.calls.indexOf(q) >= 0)).toBe(false);
    r2.unmount();
  });

  it('GPU Pods: while the pod list loads, the exporter\'s GPU owners as a partial page; the list then replaces it', async () => {
    const fake = cluster({ podsLoading: true });
    const r = render(h(route('/amd-gpu/pods')));
    await r.settle();
    expect(r.text()).not.toContain('Loading GPU pod data...');
    expect(r.text()).toContain('Partial — the pod list is loading');
    expect(r.text()).toContain('train-0');
    lib.lists.Pod = [fake.pods, null];
    r.rerender(h(route('/amd-gpu/pods')));
    await r.settle();
    expect(r.text()).not.toContain('Partial');
    expect(r.text()).toContain('train-a');
    r.unmount();
  });

  it('Overview on a cluster of more than one page: the exporter\'s GPU owners stand in for the pod sections while the list loads', async () => {
    const fake = cluster({ gpuNodes: Array.from({ length: 9 }, (_, i) => 'mi355x-' + String(i).padStart(3, '0')), podsLoading: true });
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    expect(r.text()).toContain('Partial — the pod list is loading');
    expect(r.text()).toContain('train-0');
    expect(r.text()).toContain('Loading GPU pods...');
    lib.lists.Pod = [fake.pods, null];
    r.rerender(h(route('/amd-gpu')));
    await r.settle();
    expect(r.text()).not.toContain('Partial');
    expect(r.text()).toContain('Active GPU Pods');
    r.unmount();
  });

  it('Overview on a one-page cluster sends no Prometheus request, its pod list pending or not', async () => {
    cluster({ podsLoading: true });
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    expect(lib.api.calls.filter((c) => c.indexOf('/proxy/') >= 0)).toEqual([]);
    expect(r.text()).not.toContain('Partial');
    r.unmount();
  });

  it('GPU Pods without telemetry waits for the pod list (the list is its content)', async () => {
    // A Prometheus this session has not met (no earlier answer to serve stale).
    saveSettings(Object.assign({}, DEFAULT_SETTINGS, { requestTimeoutMs: DEFAULT_SETTINGS.requestTimeoutMs + 2 }));
    cluster({ podsLoading: true });
    const api = lib.api.handler;
    lib.api.handler = (path) => (path.indexOf('/proxy/') >= 0
      ? Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 })) : api(path));
    const r = render(h(route('/amd-gpu/pods')));
    await r.settle();
    saveSettings(DEFAULT_SETTINGS);
    expect(r.text()).toContain('Loading GPU pod data...');
    r.unmount();
  });
});

describe('shared: refresh and StrictMode (' + tier + ')', () => {
  it('the Overview Refresh button re-fetches the DeviceConfig list', async () => {
    cluster();
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    const before = crdCalls();
    r.click(r.byLabel('Refresh AMD GPU data'));
    await r.settle();
    expect(crdCalls()).toBe(before + 1);
    r.unmount();
  });

  it('the Metrics Refresh button sends one more live query', async () => {
    const fake = cluster();
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    const before = promQueries(fake).length;
    expect(before).toBe(1);
    r.click(r.byLabel('Refresh metrics'));
    await r.settle();
    expect(promQueries(fake).length).toBe(before + 1);
    r.unmount();
  });

  it('the GPU Nodes and GPU Pods Refresh buttons renew the telemetry only (the lists are watches)', async () => {
    for (const [path, label] of [['/amd-gpu/nodes', 'Refresh node data'], ['/amd-gpu/pods', 'Refresh pod data']]) {
      lib.resetHeadlamp();
      resetSharedStores();
      const fake = cluster();
      const r = render(h(route(path)));
      await r.settle();
      const crd = crdCalls();
      const live = fake.mock.calls.length;
      r.click(r.byLabel(label));
      await r.settle();
      expect(crdCalls()).toBe(crd);
      expect(fake.mock.calls.length).toBe(live + 1);
      r.unmount();
    }
  });

  it('under StrictMode a route mounts with one CRD request and one live query', async () => {
    let fake = cluster();
    let r = render(h(route('/amd-gpu')), { strict: true });
    await r.settle();
    expect(crdCalls()).toBe(1);
    r.unmount();
    lib.resetHeadlamp();
    resetSharedStores();
    fake = cluster();
    r = render(h(route('/amd-gpu/metrics')), { strict: true });
    await r.settle();
    expect(promQueries(fake)).toHaveLength(1);
    expect(r.text()).toContain('GPU Power Summary');
    r.unmount();
  });

  it('each route mounts only what its page draws: Metrics the node list alone, Device Plugins no list at all', async () => {
    const expected = {
      '/amd-gpu': [true, true, 1], '/amd-gpu/device-plugins': [false, false, 1], '/amd-gpu/nodes': [true, true, 0],
      '/amd-gpu/pods': [true, true, 0], '/amd-gpu/metrics': [true, false, 0],
    };
    for (const path of Object.keys(expected)) {
      lib.resetHeadlamp();
      resetSharedStores();
      cluster();
      const r = render(h(route(path)));
      await r.settle();
      const [nodes, pods, crd] = expected[path];
      expect([path, lib.lists.calls.Node.length > 0, lib.lists.calls.Pod.some(allPods), crdCalls()]).toEqual([path, nodes, pods, crd]);
      r.unmount();
    }
  });

  it('Metrics in an allocation order mounts the pod list too, and ranks by the GPUs held', async () => {
    cluster({ gpuNodes: nodeNames(12) }); // train-a (4 GPUs) on mi355x-000, train-b (2) on mi355x-001
    lib.lists.Pod = [[makeGpuPod('hog', { gpus: 8, node: 'mi355x-010' })].concat(lib.lists.Pod[0]), null];
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    expect(lib.lists.calls.Pod).toHaveLength(0);
    r.change(r.byLabel('Sort GPU nodes'), 'in-use');
    await r.settle();
    expect(lib.lists.calls.Pod.length).toBeGreaterThan(0);
    const titles = r.byTag('h2').map((n) => r.textOf(n)).filter((t) => /^mi355x-/.test(t));
    expect(titles[0]).toBe('mi355x-010 — 8 × MI355X');
    r.unmount();
  });
});

describe('shared: the pager drives what is rendered and fetched (' + tier + ')', () => {
  it('GPU Nodes: Next page shows and queries the next 8 nodes; the filter narrows them', async () => {
    const fake = cluster({ gpuNodes: nodeNames(20) });
    const r = render(h(route('/amd-gpu/nodes')));
    await r.settle();
    expect(r.text()).toContain('Showing 1–8 of 20 GPU nodes');
    expect(r.text()).not.toContain('mi355x-008');
    r.click(r.byLabel('Next page'));
    await r.settle();
    expect(r.text()).toContain('mi355x-008');
    expect(r.text()).not.toContain('mi355x-007');
    expect(promQueries(fake).pop()).toContain('hostname=~"' + nodeNames(16).slice(8).join('|') + '"');
    r.change(r.byLabel('Filter GPU nodes by name'), '019');
    await r.settle();
    expect(r.text()).toContain('Showing 1–1 of 1 matching "019" (20 GPU nodes)');
    expect(r.value(r.byLabel('Filter GPU nodes by name'))).toBe('019');
    expect(r.isDisabled(r.byLabel('Next page'))).toBe(true);
    r.unmount();
  });
});

describe('shared: the node order drives the page and its query (' + tier + ')', () => {
  it('GPU Nodes: "Most GPUs in use" puts the busiest node first and scopes the query to that page', async () => {
    const fake = cluster({ gpuNodes: nodeNames(12) }); // train-a (4 GPUs) on mi355x-000, train-b (2) on mi355x-001
    lib.lists.Pod = [[makeGpuPod('hog', { gpus: 8, node: 'mi355x-010' })].concat(lib.lists.Pod[0]), null];
    const r = render(h(route('/amd-gpu/nodes')));
    await r.settle();
    expect(r.value(r.byLabel('Sort GPU nodes'))).toBe('name');
    r.change(r.byLabel('Sort GPU nodes'), 'in-use');
    await r.settle();
    expect(r.value(r.byLabel('Sort GPU nodes'))).toBe('in-use');
    const titles = r.byTag('h2').map((n) => r.textOf(n)).filter((t) => /^mi355x-/.test(t));
    expect(titles.slice(0, 3)).toEqual(['mi355x-010', 'mi355x-000', 'mi355x-001']);
    expect(promQueries(fake).pop()).toContain('hostname=~"mi355x-010|mi355x-000|mi355x-001|');
    r.unmount();
  });
});

describe('shared: Metrics in power order (' + tier + ')', () => {
  it('"Highest GPU power" asks Prometheus for the ranked page and shows the hottest node first', async () => {
    const fake = cluster({ gpuNodes: nodeNames(12) });
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    r.change(r.byLabel('Sort GPU nodes'), 'power');
    await r.settle();
    expect(promQueries(fake).filter((q) => q.indexOf('topk(8,') >= 0).length).toBeGreaterThan(0);
    expect(r.text()).toContain('Showing 1–8 of 12 GPU nodes reporting');
    r.unmount();
  });
});

describe('shared: GPU Pods in power order (' + tier + ')', () => {
  it('"Highest GPU power" asks Prometheus for the ranked page of pods and lists the hungriest first', async () => {
    const fake = cluster();
    // the exporter fixture labels GPU 0 / 1 of each node with pods ml/train-0 (700 W) and ml/train-1 (701 W)
    lib.lists.Pod = [[makeGpuPod('train-0', { gpus: 1, node: 'mi355x-000' }), makeGpuPod('train-1', { gpus: 1, node: 'mi355x-001' })], null];
    const r = render(h(route('/amd-gpu/pods')));
    await r.settle();
    expect(r.byLabel('Filter or sort GPU pods')).toBeTruthy(); // one page: the count line and this button
    r.click(r.byLabel('Filter or sort GPU pods'));
    await r.settle();
    r.change(r.byLabel('Sort GPU pods'), 'power');
    await r.settle();
    expect(promQueries(fake).filter((q) => q.indexOf('sum by (namespace, pod)') >= 0).length).toBeGreaterThan(0);
    expect(r.text()).toContain('Showing 1–2 of 2 GPU pods drawing power');
    const text = r.text();
    expect(text.indexOf('train-1')).toBeLessThan(text.indexOf('train-0'));
    // the controls keep their names when the count narrows to the pods drawing power
    expect(r.value(r.byLabel('Sort GPU pods'))).toBe('power');
    r.unmount();
  });
});

describe('shared: native-view sections (' + tier + ')', () => {
  it('Node detail on a cold store: the node\'s own pods by a scoped list + watch, no cluster-wide list', async () => {
    cluster();
    const r = render(reg.details[0]({ resource: { kind: 'Node', jsonData: makeGpuNode('mi355x-001') } }));
    await r.settle();
    expect(r.text()).toContain('AMD GPU');
    expect(r.text()).toContain('train-b');
    expect(lib.lists.calls.Node).toHaveLength(0);
    expect(lib.lists.calls.Pod.every((o) => o && o.fieldSelector === 'spec.nodeName=mi355x-001')).toBe(true);
    r.unmount();
  });

  it('Node detail on a cold store is live: a pod scheduled onto the node after mount shows without remount', async () => {
    const fake = cluster();
    const el = () => reg.details[0]({ resource: { kind: 'Node', jsonData: makeGpuNode('mi355x-001') } });
    const r = render(el());
    await r.settle();
    expect(r.text()).toContain('train-b');
    expect(r.text()).not.toContain('late-job');
    lib.lists.Pod = [fake.pods.concat([makeGpuPod('late-job', { gpus: 2, node: 'mi355x-001' })]), null];
    r.rerender(el());
    await r.settle();
    expect(r.text()).toContain('late-job');
    expect(r.text()).toContain('train-b');
    r.unmount();
  });

  it('Pod detail: a GPU pod renders its resources without a cluster request', async () => {
    cluster();
    const r = render(reg.details[1]({ resource: { kind: 'Pod', jsonData: makeGpuPod('train-a', { gpus: 4, node: null }) } }));
    await r.settle();
    expect(r.text()).toContain('AMD GPU Resources');
    expect(crdCalls()).toBe(0);
    r.unmount();
  });

  it('nothing for CPU nodes and non-GPU pods', async () => {
    cluster();
    const a = render(h('div', null, reg.details[0]({ resource: { kind: 'Node', jsonData: makeNode('cpu-0') } })));
    const b = render(h('div', null, reg.details[1]({ resource: { kind: 'Pod', jsonData: makePlainPod('web-0') } })));
    await a.settle();
    await b.settle();
    expect(a.byTag('section')).toHaveLength(0);
    expect(b.byTag('section')).toHaveLength(0);
    a.unmount();
    b.unmount();
  });
});
