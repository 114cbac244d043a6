/**
 * Small-cluster mode (the first wave needs no node list on a cluster that
 * fits one page: size-guarded queries) and the source probe (the first
 * scoped answer decides exporter / node-exporter / no telemetry in one wave).
 * The pager and the scoped queries themselves are in paging.test.js.
 */
import React, { render } from './stubs/react.js';
import * as lib from './stubs/headlamp-lib.js';
import * as CC from './stubs/CommonComponents.js';
import { createPlugin } from '../../src/plugin.js';
import { resetSharedStores } from '../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../src/api/k8sCore.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { metricsView } from '../../src/view/pages/metricsPage.js';
import { NODES_PER_PAGE, PODS_PER_PAGE } from '../../src/view/pages/paging.js';
import { ownersScope } from '../../src/view/pages/pods.js';
import { sectionTitles } from '../../src/view/ir.js';
import { createMetricsSource } from '../../src/api/metrics.js';
import { SERIES, SMALL_CLUSTER_NODES, SMALL_CLUSTER_PODS } from '../../src/api/series.js';
import { makeContext, makeDeviceConfig, makeGpuNode, makeGpuPod } from './fixtures.js';
import { exporterData, prom } from './promFake.js';

const h = React.createElement;
const names = (n) => Array.from({ length: n }, (_, i) => 'mi355x-' + String(i).padStart(3, '0'));
const decoded = (fake) => fake.mock.calls.map((c) => decodeURIComponent(c[0]));

beforeEach(() => {
  clearViewMemo();
  resetSharedStores();
});

describe('small-cluster mode: the first wave needs no node list on a cluster of one page', () => {
  it('a small cluster answers with every GPU (statics included) in one request, before any node name is known', async () => {
    const fake = prom({ data: exporterData(names(2)) });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuMetrics('topology', { scope: [], small: true });
    expect(fake.mock.calls).toHaveLength(1);
    expect(decoded(fake)[0]).toContain('and on() (count(count by (hostname) ({__name__="gpu_power_usage"})) <= ' + SMALL_CLUSTER_NODES + ')');
    expect(m.small).toEqual({ count: 2, limit: SMALL_CLUSTER_NODES, exceeded: false });
    expect(m.gpus).toHaveLength(16);
    expect(m.gpus[0].vramTotalBytes).toBeGreaterThan(0);
    expect(m.source).toBe('amd-exporter');
  });
  it('a larger cluster answers with nothing before the node list, then with the scope only; never cluster-wide', async () => {
    const fake = prom({ data: exporterData(names(9)) });
    const s = createMetricsSource({ request: fake });
    const early = await s.fetchGpuMetrics('topology', { scope: [], small: true });
    expect(early.gpus).toHaveLength(0);
    expect(early.small.exceeded).toBe(true);
    expect(fake.mock.calls).toHaveLength(1); // the GPU count says "exporter present": no cluster-wide fallback
    const later = await s.fetchGpuMetrics('topology', { scope: ['mi355x-004'], small: true });
    expect(Array.from(new Set(later.gpus.map((g) => g.nodeName)))).toEqual(['mi355x-004']);
    expect(fake.mock.calls).toHaveLength(2);
  });
  it('the Metrics summary rides along; the node count row is no total', async () => {
    const fake = prom({ data: exporterData(names(3)) });
    const m = await createMetricsSource({ request: fake }).fetchGpuMetrics('gauges', { scope: names(3), summary: true, small: true });
    expect([m.totals.gpus, m.totals.nodes]).toEqual([24, 3]);
    expect(m.gpus).toHaveLength(24);
  });
  it('owners and series have the same guarded form', async () => {
    const fake = prom({ data: exporterData(['n0']) });
    const s = createMetricsSource({ request: fake });
    const o = await s.fetchGpuOwners({ pods: [], small: true });
    expect(o.gpus.map((g) => g.pod)).toEqual(['train-0', 'train-1']);
    expect(decoded(fake)[0]).toContain('pod!=""})) and on() (count(count by (namespace, pod)');
    expect(o.small).toEqual({ count: 2, limit: SMALL_CLUSTER_PODS, exceeded: false });
    const sr = await s.fetchSeries(1800, 30, [], true);
    expect(decoded(fake)[1]).toContain('and on() (count(');
    expect(sr.total.power.length).toBe(2);
  });
  it('plugin: a cold GPU Nodes page on a small cluster asks once, before the node list, and keeps that answer', async () => {
    lib.resetHeadlamp();
    lib.lists.Node = [null, null];
    lib.lists.Pod = [null, null];
    const fake = prom({ data: exporterData(names(2)) });
    lib.api.handler = (p) => {
      if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
      if (p.indexOf('/proxy/api/v1/') >= 0) return fake(p);
      return Promise.reject(Object.assign(new Error('503'), { status: 503 }));
    };
    const plugin = createPlugin({ React: React, lib: lib, CommonComponents: CC });
    const Page = plugin.routeComponent('nodes');
    const r = render(h(Page));
    await r.settle();
    const live = () => decoded(fake).filter((q) => /\/query\?query=(?!1$)/.test(q));
    expect(live()).toHaveLength(1); // sent while the lists load
    lib.lists.Node = [names(2).map((x) => makeGpuNode(x)), null];
    lib.lists.Pod = [[makeGpuPod('train-0', { node: 'mi355x-000' })], null];
    r.rerender(h(Page));
    await r.settle();
    expect(live()).toHaveLength(1); // the node list arriving sends nothing more
    expect(r.text()).toContain('mi355x-001');
    r.click(r.getByLabelText('Refresh node data'));
    await r.settle();
    expect(live()).toHaveLength(2);
    r.unmount();
  });
});

describe('small-cluster mode: guards and pages agree', () => {
  it('the node guard is one page of nodes; the pod guard what such a cluster can run, one GPU each', () => {
    expect(SMALL_CLUSTER_NODES).toBe(NODES_PER_PAGE);
    expect(SMALL_CLUSTER_PODS).toBe(NODES_PER_PAGE * 8);
    expect(SMALL_CLUSTER_PODS).toBeGreaterThanOrEqual(PODS_PER_PAGE);
    const pods = (n) => Array.from({ length: n }, (_, i) => makeGpuPod('p' + i, { node: 'mi355x-000' }));
    expect(ownersScope(makeContext({ nodes: [makeGpuNode('mi355x-000')], pods: pods(64) }), {}).small).toBe(true);
    expect(ownersScope(makeContext({ nodes: [makeGpuNode('mi355x-000')], pods: pods(65) }), {}).small).toBe(undefined);
  });
  it('an answer that found more than one page of nodes is asked again with the names, once the list has them', async () => {
    lib.resetHeadlamp();
    lib.lists.Node = [null, null];
    lib.lists.Pod = [null, null];
    // Two GPU nodes listed; the exporter still reports eight removed ones (stale series).
    const fake = prom({ data: exporterData(names(10)) });
    lib.api.handler = (p) => {
      if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [] });
      if (p.indexOf('/proxy/api/v1/') >= 0) return fake(p);
      return Promise.reject(Object.assign(new Error('503'), { status: 503 }));
    };
    const plugin = createPlugin({ React: React, lib: lib, CommonComponents: CC });
    const Page = plugin.routeComponent('nodes');
    const r = render(h(Page));
    await r.settle();
    const live = () => decoded(fake).filter((q) => /\/query\?query=(?!1$)/.test(q));
    expect(live()).toHaveLength(1);
    lib.lists.Node = [names(2).map((x) => makeGpuNode(x)), null];
    lib.lists.Pod = [[], null];
    r.rerender(h(Page));
    await r.settle();
    expect(live()).toHaveLength(2);
    expect(live()[1]).toContain('hostname=~"mi355x-000|mi355x-001"');
    r.rerender(h(Page));
    await r.settle();
    expect(live()).toHaveLength(2); // settled: no refetch loop
    r.unmount();
  });
});

describe('scoped fetches: the first answer decides the telemetry source (one wave)', () => {
  const neOf = (nodes, chipsPerNode) => {
    const ne = { node_uname_info: [], node_hwmon_power_input_watt: [] };
    ne[SERIES.nodeExporter.chips] = [];
    nodes.forEach((n, i) => {
      const inst = '10.0.0.' + i + ':9100';
      ne.node_uname_info.push({ metric: { __name__: 'node_uname_info', instance: inst, nodename: n }, value: [0, '1'] });
      for (let c = 0; c < chipsPerNode; c++) {
        const chip = '0000:' + String(5 + c).padStart(2, '0') + ':00_0';
        ne[SERIES.nodeExporter.chips].push({ metric: { __name__: 'node_hwmon_chip_names', chip_name: 'amdgpu', instance: inst, chip: chip }, value: [0, '1'] });
        ne.node_hwmon_power_input_watt.push({ metric: { __name__: 'node_hwmon_power_input_watt', instance: inst, chip: chip }, value: [0, '500'] });
      }
    });
    return ne;
  };

  it('a cluster without GPU telemetry: one request per fetch, never a cluster-wide look; the view keeps the warning', async () => {
    const fake = prom({ data: {} });
    const s = createMetricsSource({ request: fake });
    const m1 = await s.fetchGpuMetrics('gauges', { scope: [], summary: true, small: true });
    expect(fake.mock.calls.length).toBe(1); // exporter rows + totals + source probe, one answer
    expect(decoded(fake)[0]).toContain('"agg", "hwmon"');
    expect(m1.totals.gpus).toBe(0);
    const m2 = await s.fetchGpuMetrics('gauges', { scope: [], summary: true, small: true });
    expect(fake.mock.calls.length).toBe(2);
    expect(s.source()).toBe(null);
    // The Metrics page says so on every refresh, not only the first (zero totals, not "unknown").
    for (const m of [m1, m2]) {
      const vm = metricsView(makeContext({ nodes: [] }), { metrics: m, series: null, fetchError: null, fetching: false });
      expect(sectionTitles(vm)).toContain('No AMD GPU Metrics in Prometheus');
    }
  });

  it('the GPU Nodes page of a cluster without GPU telemetry asks once per refresh too', async () => {
    const fake = prom({ data: {} });
    const s = createMetricsSource({ request: fake });
    await s.fetchGpuMetrics('topology', { scope: names(3), small: true });
    await s.fetchGpuMetrics('topology', { scope: names(3) });
    expect(fake.mock.calls.length).toBe(2);
  });

  it('a node-exporter-only cluster of one page gets its hwmon telemetry in the first answer', async () => {
    const fake = prom({ data: {}, ne: neOf(names(2), 8) });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuMetrics('gauges', { scope: [], summary: true, small: true });
    expect(fake.mock.calls.length).toBe(1);
    expect(s.source()).toBe('node-exporter');
    expect(m.totals.gpus).toBe(16);
    expect(m.totals.powerWatts).toBe(16 * 500);
    // later refreshes ask node-exporter directly: one cluster-wide request
    await s.fetchGpuMetrics('gauges', { scope: names(2), summary: true, small: true });
    expect(fake.mock.calls.length).toBe(2);
    expect(decoded(fake)[1]).not.toContain('gpu_power_usage');
  });

  it('a larger node-exporter cluster (more amdgpu chips than one page) is served in the first wave, page-scoped', async () => {
    const fake = prom({ data: {}, ne: neOf(names(9), 8) });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuMetrics('gauges', { scope: names(8), summary: true });
    // the probe carries node-exporter's page and totals, dropped where the exporter reports (`unless on()`)
    expect(fake.mock.calls.length).toBe(1);
    expect(decoded(fake)[0]).toContain(') unless on() (count(count by (hostname)');
    expect(s.source()).toBe('node-exporter');
    expect(m.totals.gpus).toBe(72);
    expect(m.gpus.length).toBe(64);
    // the page's nodes through node_uname_info and the totals: nothing cluster-wide, then and on every refresh
    await s.fetchGpuMetrics('gauges', { scope: names(8), summary: true });
    expect(fake.mock.calls.length).toBe(2);
    [0, 1].forEach((i) => {
      expect(decoded(fake)[i]).toContain('and on(instance) node_uname_info{nodename=~');
      expect(decoded(fake)[i]).not.toMatch(/\{__name__=~"[^"]*"\}\)( or|$)/);
    });
  });
});
