/**
 * O(visible) GPU Nodes and Metrics pages: the pager (pages.js nodePage), the
 * scoped telemetry queries (metrics.js exporterQuery / summaryQuery /
 * scopedSeriesQuery with `hostname=~`), and the pages built from them.
 *
 * The reference renders one card per GPU node (NodesPage.tsx:285-291) and
 * one per chip on its Metrics page (MetricsPage.tsx:348-350), with every
 * node's telemetry per fetch; here what a page renders and fetches is bounded
 * by NODES_PER_PAGE, whatever the cluster size.
 */
import React, { render, textOf as textOfNode } from './stubs/react.js';
import * as lib from './stubs/headlamp-lib.js';
import * as CC from './stubs/CommonComponents.js';
import { createPlugin } from '../../src/plugin.js';
import { resetSharedStores } from '../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../src/api/k8sCore.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { devicePluginsView } from '../../src/view/pages/devicePlugins.js';
import { ALL_NODES_SERIES, metricsView } from '../../src/view/pages/metricsPage.js';
import { nodesView, telemetryScope } from '../../src/view/pages/nodes.js';
import { OVERVIEW_PLUGIN_PODS, overviewView } from '../../src/view/pages/overview.js';
import {
  NODE_SORTS,
  nodePage,
  NODES_PER_PAGE,
  nodeSortOf,
  POD_SORTS,
  podPage,
  PODS_PER_PAGE,
  podSortOf,
  RANKED_NODE_SORTS,
  RANKED_POD_SORTS,
} from '../../src/view/pages/paging.js';
import { ownersScope, podsView } from '../../src/view/pages/pods.js';
import { renderText } from '../../src/view/text.js';
import { countRows, findSection, pagerOf, pagerText, rowValue, sectionTitles } from '../../src/view/ir.js';
import { rankedSlice } from '../../src/view/pages/paging.js';
import { renderPage } from '../../src/view/html.js';
import { createMetricsSource } from '../../src/api/metrics.js';
import {
  hostnameMatcher,
  powerRankQuery,
  regexLiteral,
  scopedSeriesQuery,
  summaryQuery,
} from '../../src/api/promql.js';
import { SERIES, TOTAL_SERIES } from '../../src/api/series.js';
import { joinExporterResults, splitByName, summarizeMetrics, totalsFromRows } from '../../src/api/telemetry.js';
import { makeContext, makeDeviceConfig, makeGpuNode, makeGpuPod, makePluginPod } from './fixtures.js';
import { BASE0, exporterData, flatten, prom } from './promFake.js';

const h = React.createElement;
const names = (n) => Array.from({ length: n }, (_, i) => 'mi355x-' + String(i).padStart(3, '0'));
const ctxOf = (n) => makeContext({ nodes: names(n).map((x) => makeGpuNode(x)), pods: [makeGpuPod('train-0', { node: 'mi355x-000' })] });
const cards = (vm) => sectionTitles(vm).filter((t) => /^mi355x-/.test(t));
const decoded = (fake) => fake.mock.calls.map((c) => decodeURIComponent(c[0]));

beforeEach(() => {
  clearViewMemo();
  resetSharedStores();
});

describe('nodePage', () => {
  const nodes = names(20).map((x) => makeGpuNode(x));
  it('slices NODES_PER_PAGE nodes and counts the pages', () => {
    const p = nodePage(nodes, { page: 0 });
    expect(NODES_PER_PAGE).toBe(8);
    expect(p.names).toEqual(names(8));
    expect([p.page, p.pages, p.from, p.to, p.total, p.matched]).toEqual([0, 3, 0, 8, 20, 20]);
    expect(nodePage(nodes, { page: 2 }).names).toEqual(names(20).slice(16));
  });
  it('clamps the page into range', () => {
    expect(nodePage(nodes, { page: 99 }).page).toBe(2);
    expect(nodePage(nodes, { page: -3 }).page).toBe(0);
    expect(nodePage([], { page: 4 })).toEqual(Object.assign({}, nodePage([], {}), {}));
    expect(nodePage([], {}).pages).toBe(1);
  });
  it('filters by a case-insensitive name substring (surrounding spaces ignored) and keeps the raw text', () => {
    const p = nodePage(nodes, { filter: ' X-01 ' });
    expect(p.names).toEqual(['mi355x-010', 'mi355x-011', 'mi355x-012', 'mi355x-013', 'mi355x-014', 'mi355x-015', 'mi355x-016', 'mi355x-017']);
    expect([p.matched, p.pages, p.filter]).toEqual([10, 2, ' X-01 ']);
    expect(nodePage(nodes, { filter: 'nope' }).matched).toBe(0);
  });
  it('returns the same object for the same list and state (memo)', () => {
    expect(nodePage(nodes, { page: 1 })).toBe(nodePage(nodes, { page: 1 }));
    expect(nodePage(nodes, { page: 1 })).not.toBe(nodePage(nodes.slice(), { page: 1 }));
  });
  it('pager text', () => {
    expect(pagerText(Object.assign({ noun: 'GPU nodes' }, nodePage(nodes, { page: 1 })))).toBe('Showing 9–16 of 20 GPU nodes · page 2 of 3');
    expect(pagerText(Object.assign({ noun: 'GPU nodes' }, nodePage(nodes, { filter: 'x-01' })))).toBe(
      'Showing 1–8 of 10 matching "x-01" (20 GPU nodes) · page 1 of 2'
    );
    expect(pagerText(Object.assign({ noun: 'GPU nodes' }, nodePage(nodes, { filter: 'zz' })))).toBe('No GPU nodes match "zz"');
  });
});

describe('node order', () => {
  // 12 GPU nodes; mi355x-005 holds 6 GPUs, mi355x-009 holds 2, mi355x-003 is not ready.
  function ctxSorted() {
    const nodes = names(12).map((x) => makeGpuNode(x, { ready: x !== 'mi355x-003' }));
    const pods = [makeGpuPod('big', { gpus: 6, node: 'mi355x-005' }), makeGpuPod('small', { gpus: 2, node: 'mi355x-009' })];
    return makeContext({ nodes, pods });
  }
  it('name order by default and for an unknown sort', () => {
    const ctx = ctxSorted();
    expect(nodePage(ctx.gpuNodes, {}, ctx.index).names).toEqual(names(8));
    expect(nodeSortOf({ sort: 'bogus' })).toBe('name');
    expect(nodePage(ctx.gpuNodes, { sort: 'bogus' }, ctx.index).names).toEqual(names(8));
  });
  it('most GPUs in use / most free / not ready first, ties in name order', () => {
    const ctx = ctxSorted();
    expect(nodePage(ctx.gpuNodes, { sort: 'in-use' }, ctx.index).names.slice(0, 3)).toEqual(['mi355x-005', 'mi355x-009', 'mi355x-000']);
    const free = nodePage(ctx.gpuNodes, { sort: 'free', page: 1 }, ctx.index).names;
    expect(free.slice(-2)).toEqual(['mi355x-009', 'mi355x-005']);
    expect(nodePage(ctx.gpuNodes, { sort: 'attention' }, ctx.index).names[0]).toBe('mi355x-003');
  });
  it('the sorted page is memoised on the list and the index; the filter applies after sorting', () => {
    const ctx = ctxSorted();
    expect(nodePage(ctx.gpuNodes, { sort: 'in-use' }, ctx.index)).toBe(nodePage(ctx.gpuNodes, { sort: 'in-use' }, ctx.index));
    expect(nodePage(ctx.gpuNodes, { sort: 'in-use', filter: 'x-01' }, ctx.index).names).toEqual(['mi355x-010', 'mi355x-011']);
    expect(nodePage(ctx.gpuNodes, { sort: 'in-use', filter: '00' }, ctx.index).names.slice(0, 3)).toEqual(['mi355x-005', 'mi355x-009', 'mi355x-000']);
  });
  it('the pager offers the orders; telemetry follows the sorted page', () => {
    const ctx = ctxSorted();
    const vm = nodesView(ctx, { pager: { sort: 'in-use' } });
    const p = pagerOf(vm);
    expect(p.sorts.map((o) => o.value)).toEqual(NODE_SORTS.map((o) => o.value).concat(['power']));
    expect(p.sort).toBe('in-use');
    expect(cards(vm)[0]).toBe('mi355x-005');
    expect(renderPage(vm)).toContain('<option value="in-use" selected>Most GPUs in use</option>');
    expect(renderText(vm)).toContain('sorted: Most GPUs in use');
    expect(telemetryScope(ctx, { sort: 'in-use' }).scope[0]).toBe('mi355x-005');
  });
  it('Metrics offers the same orders over the node list', async () => {
    const ctx = ctxSorted();
    const fake = prom({ data: exporterData(names(12)) });
    const s = createMetricsSource({ request: fake });
    const scope = telemetryScope(ctx, { sort: 'in-use' }).scope;
    const m = await s.fetchGpuMetrics('gauges', { scope: scope, summary: true });
    const vm = metricsView(ctx, { metrics: m, series: null, fetchError: null, fetching: false }, { pager: { sort: 'in-use' } });
    expect(cards(vm)[0]).toBe('mi355x-005 — 8 × MI355X');
    expect(pagerOf(vm).sort).toBe('in-use');
  });
});

describe('GPU Pods order', () => {
  function podsCtx() {
    const nodes = [makeGpuNode('mi355x-000')];
    const pods = [
      makeGpuPod('a-small', { gpus: 1, node: 'mi355x-000' }),
      makeGpuPod('b-big', { gpus: 8, node: 'mi355x-000' }),
      makeGpuPod('c-wait', { gpus: 2, phase: 'Pending', node: null, waiting: 'Unschedulable' }),
      makeGpuPod('d-mid', { gpus: 4, node: 'mi355x-000' }),
    ];
    pods[3].metadata.creationTimestamp = '2030-01-01T00:00:00Z';
    return makeContext({ nodes, pods });
  }
  const order = (ctx, sort) => podPage(ctx.gpuPods, { sort }).names.map((k) => k.split('/')[1]);
  it('namespace / name by default; most GPUs held, newest, not running first on request', () => {
    const ctx = podsCtx();
    expect(order(ctx, undefined)).toEqual(['a-small', 'b-big', 'c-wait', 'd-mid']);
    expect(order(ctx, 'gpus')).toEqual(['b-big', 'd-mid', 'c-wait', 'a-small']);
    expect(order(ctx, 'newest')[0]).toBe('d-mid');
    expect(order(ctx, 'attention')[0]).toBe('c-wait');
    expect(podSortOf({ sort: 'power' })).toBe('name');
  });
  it('the table and the owner query follow the order; operator pods keep theirs', () => {
    const ctx = podsCtx();
    const vm = podsView(ctx, { pager: { sort: 'gpus' } });
    expect(findSection(vm, 'All GPU Pods').blocks[0].rows[0][0]).toBe('b-big');
    const p = pagerOf(vm);
    expect([p.sort, p.sorts.map((o) => o.value)]).toEqual(['gpus', RANKED_POD_SORTS.map((o) => o.value)]);
    expect(RANKED_POD_SORTS.map((o) => o.value)).toEqual(POD_SORTS.map((o) => o.value).concat(['power']));
    expect(ownersScope(ctx, { sort: 'gpus' }).pods[0]).toBe('ml/b-big');
    expect(podPage(ctx.gpuPods, { sort: 'gpus' }, 'plugin-pod').names[0]).toBe('ml/a-small');
  });
});

describe('GPU Pods in power order: Prometheus ranks the pods by the power of the GPUs they hold', () => {
  // 30 GPU pods on one node; pod i holds GPU i % 8 and draws 100 + 10 * ((i * 7) % 30) W, so power order is not name order.
  function cluster() {
    const nodes = [makeGpuNode('mi355x-000')];
    const pods = [];
    const d = exporterData(['mi355x-000']);
    const E = SERIES.exporter;
    d[E.power] = [];
    for (let i = 0; i < 30; i++) {
      const name = 'job-' + String(i).padStart(2, '0');
      pods.push(makeGpuPod(name, { gpus: 1, node: 'mi355x-000' }));
      d[E.power].push({ metric: { __name__: E.power, hostname: 'mi355x-000', gpu_id: String(i % 8), instance: 'x', pod: name, namespace: 'ml' },
        value: [0, String(100 + 10 * ((i * 7) % 30))] });
    }
    d[E.power].push({ metric: { __name__: E.power, hostname: 'mi355x-000', gpu_id: '7', instance: 'x' }, value: [0, '999'] }); // no owner
    return { ctx: makeContext({ nodes, pods }), fake: prom({ data: d }) };
  }
  const watts = (i) => 100 + 10 * ((i * 7) % 30);
  const byPower = Array.from({ length: 30 }, (_, i) => i).sort((a, b) => watts(b) - watts(a)).map((i) => 'job-' + String(i).padStart(2, '0'));

  it('the owner query asks Prometheus for one ranked page; the table shows it in power order with its GPUs', async () => {
    const { ctx, fake } = cluster();
    const state = { sort: 'power', page: 0 };
    const o = ownersScope(ctx, state);
    expect(o.rank).toEqual({ by: 'power', page: 0, per: PODS_PER_PAGE, filter: '' });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuOwners({ rank: o.rank });
    expect(m.rank.count).toBe(30);
    expect(m.rank.order).toEqual(byPower.slice(0, PODS_PER_PAGE).map((n) => 'ml/' + n));
    expect(decoded(fake).filter((q) => q.indexOf('topk(' + PODS_PER_PAGE + ', sum by (namespace, pod)') >= 0).length).toBe(1);
    const vm = podsView(ctx, { metrics: m, pager: state });
    const rows = findSection(vm, 'All GPU Pods').blocks[0].rows;
    expect(rows.map((r) => r[0])).toEqual(byPower.slice(0, PODS_PER_PAGE));
    expect(findSection(vm, 'All GPU Pods').blocks[0].columns).toContain('GPU Power');
    expect(pagerText(pagerOf(vm))).toBe('Showing 1–25 of 30 GPU pods drawing power · page 1 of 2');
    // the count narrows to the pods drawing power; the controls keep their names
    expect([pagerOf(vm).noun, pagerOf(vm).label]).toEqual(['GPU pods drawing power', 'GPU pods']);
  });

  it('page 2 and a name filter are ranked by Prometheus too', async () => {
    const { ctx, fake } = cluster();
    const s = createMetricsSource({ request: fake });
    const p2 = await s.fetchGpuOwners({ rank: ownersScope(ctx, { sort: 'power', page: 1 }).rank });
    expect(p2.rank.order).toEqual(byPower.slice(PODS_PER_PAGE).map((n) => 'ml/' + n));
    const f = await s.fetchGpuOwners({ rank: ownersScope(ctx, { sort: 'power', filter: ' JOB-1' }).rank });
    expect(f.rank.count).toBe(10);
    expect(f.rank.order.every((k) => /^ml\/job-1\d$/.test(k))).toBe(true);
    const vm = podsView(ctx, { metrics: f, pager: { sort: 'power', filter: ' JOB-1' } });
    expect(findSection(vm, 'All GPU Pods').blocks[0].rows).toHaveLength(10);
  });

  it('a page past the end of the ranking (the count shrank) says so and the page moves to the last one', async () => {
    const { ctx, fake } = cluster();
    const p = rankedSlice({ page: 5, per: PODS_PER_PAGE, count: 30 }, 0, {});
    expect(p).toMatchObject({ page: 1, pages: 2, from: 25, to: 25, beyond: true });
    const t = pagerText({ noun: 'GPU pods drawing power', page: p.page, pages: p.pages, from: p.from, to: p.to, total: p.total,
      matched: p.matched, filter: '', beyond: true });
    expect(t).toBe('Moving to page 2 of 2 (30 GPU pods drawing power)');
    expect(rankedSlice({ page: 1, per: PODS_PER_PAGE, count: 30 }, 5, {})).toMatchObject({ page: 1, from: 25, to: 30, beyond: false });
    // The plugin: a stored page 6 in power order is moved to page 2, which is asked for and shown.
    lib.resetHeadlamp();
    lib.lists.Node = [ctx.gpuNodes, null];
    lib.lists.Pod = [ctx.gpuPods, null];
    lib.api.handler = (path) => (path.indexOf('/proxy/api/v1/') >= 0 ? fake(path)
      : Promise.reject(Object.assign(new Error('404'), { status: 404 })));
    const mem = {};
    const storage = { getItem: (k) => (k in mem ? mem[k] : null), setItem: (k, v) => { mem[k] = v; } };
    storage.setItem('headlamp-amd-gpu-plugin.view.__default__|pods', JSON.stringify({ page: 5, filter: '', sort: 'power' }));
    const plugin = createPlugin({ React, lib, CommonComponents: CC, viewStorage: storage });
    const view = render(h(plugin.routeComponent('pods')));
    await view.settle(20);
    expect(view.text()).toContain('Showing 26–30 of 30 GPU pods drawing power · page 2 of 2');
    expect(JSON.parse(mem['headlamp-amd-gpu-plugin.view.__default__|pods']).page).toBe(1);
    view.unmount();
  });

  it('before the ranked answer the page shows the name order; the client orders never ask Prometheus to rank', () => {
    const { ctx } = cluster();
    const vm = podsView(ctx, { pager: { sort: 'power' } });
    expect(findSection(vm, 'All GPU Pods').blocks[0].rows[0][0]).toBe('job-00');
    expect(pagerOf(vm).sort).toBe('power');
    expect(ownersScope(ctx, { sort: 'gpus' }).rank).toBeUndefined();
    expect(podSortOf({ sort: 'power' }, RANKED_POD_SORTS)).toBe('power');
  });
});

describe('Metrics in power order: Prometheus ranks the page', () => {
  // 12 reporting nodes; node i draws 700 + g + 10 * (i % 5) W per GPU, so the ranking is not the name order.
  function hot(n) {
    const d = exporterData(names(n));
    d[SERIES.exporter.power].forEach((r) => {
      const i = Number(r.metric.hostname.slice(-3));
      r.value = [r.value[0], String(parseFloat(r.value[1]) + 10 * (i % 5))];
    });
    return d;
  }
  const rank = (page, filter) => ({ by: 'power', page: page, per: 8, filter: filter || '' });
  it('the rank query pages with topk and `unless`; a name filter is a lowercase substring', () => {
    expect(powerRankQuery(0, 8, '')).toBe('topk(8, sum by (hostname) ({__name__="gpu_power_usage"}))');
    expect(powerRankQuery(2, 8, 'Rack-1')).toContain('topk(24, sum by (hostname) ({__name__="gpu_power_usage", hostname=~".*rack-1.*"})) unless on(hostname) topk(16,');
    expect(powerRankQuery(0, 8, 'a.b')).toContain('hostname=~".*a\\\\.b.*"');
  });
  it('one request answers the page in power order, the ranked count and the totals', async () => {
    const fake = prom({ data: hot(12) });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuMetrics('gauges', { rank: rank(0), summary: true });
    expect(fake.mock.calls).toHaveLength(1);
    expect(m.scope.slice(0, 3)).toEqual(['mi355x-004', 'mi355x-009', 'mi355x-003']);
    expect(m.rank.count).toBe(12);
    expect(new Set(m.gpus.map((g) => g.nodeName)).size).toBe(8);
    expect(m.totals.gpus).toBe(96);
    const p1 = await s.fetchGpuMetrics('gauges', { rank: rank(1), summary: true });
    expect(p1.scope).toHaveLength(4);
    expect(p1.scope.filter((x) => m.scope.indexOf(x) >= 0)).toEqual([]);
    // The same page again: its nodes' static series are cached, the query is live-only, the GPUs keep their caps.
    const again = await s.fetchGpuMetrics('gauges', { rank: rank(0), summary: true });
    const qs = decoded(fake);
    const pagePart = (q) => q.split(') and on(hostname)')[0];
    expect(pagePart(qs[0])).toContain(SERIES.exporter.vramTotal);
    expect(pagePart(qs[2])).not.toContain(SERIES.exporter.vramTotal);
    expect(again.gpus[0].vramTotalBytes).toBeGreaterThan(0);
  });
  it('telemetryScope asks for the ranked page when the page can rank (GPU Nodes, Metrics)', () => {
    const ctx = ctxOf(12);
    expect(telemetryScope(ctx, { sort: 'power', page: 1, filter: ' X-0 ' }, true)).toEqual({ enabled: true, rank: { by: 'power', page: 1, per: 8, filter: 'x-0' } });
    expect(telemetryScope(ctx, { sort: 'power' }).rank).toBe(undefined); // no `ranked`: name order
    expect(RANKED_NODE_SORTS.map((o) => o.value)).toEqual(NODE_SORTS.map((o) => o.value).concat(['power']));
  });
  it('metricsView shows the ranked page: cards in power order, pager over the nodes ranked', async () => {
    const s = createMetricsSource({ request: prom({ data: hot(12) }) });
    const m = await s.fetchGpuMetrics('gauges', { rank: rank(0), summary: true });
    const vm = metricsView(ctxOf(12), { metrics: m, series: null, fetchError: null, fetching: false }, { pager: { sort: 'power' } });
    expect(cards(vm).slice(0, 2)).toEqual(['mi355x-004 — 8 × MI355X', 'mi355x-009 — 8 × MI355X']);
    const p = pagerOf(vm);
    expect([p.sort, p.noun, p.pages, p.total]).toEqual(['power', 'GPU nodes reporting', 2, 12]);
    expect(pagerText(p)).toBe('Showing 1–8 of 12 GPU nodes reporting · page 1 of 2');
  });
  it('GPU Nodes in power order: the ranked page as node cards, topology view, no series', async () => {
    lib.resetHeadlamp();
    lib.lists.Node = [names(12).map((x) => makeGpuNode(x)), null];
    lib.lists.Pod = [[], null];
    const fake = prom({ data: hot(12) });
    lib.api.handler = (p) => {
      if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [] });
      if (p.indexOf('/proxy/api/v1/') >= 0) return fake(p);
      return Promise.reject(Object.assign(new Error('503'), { status: 503 }));
    };
    const plugin = createPlugin({ React: React, lib: lib, CommonComponents: CC });
    const r = render(h(plugin.routeComponent('nodes')));
    await r.settle();
    const before = fake.mock.calls.length;
    r.change(r.getByLabelText('Sort GPU nodes'), 'power');
    await r.settle();
    const sent = decoded(fake).slice(before);
    expect(sent).toHaveLength(1);
    expect(sent[0]).toContain('topk(8,');
    expect(sent[0]).toContain('xgmi');
    const titles = r.byTag('h2').map((n) => textOfNode(n)).filter((t) => /^mi355x-/.test(t));
    expect(titles.slice(0, 2)).toEqual(['mi355x-004', 'mi355x-009']);
    expect(r.text()).toContain('Showing 1–8 of 12 GPU nodes reporting');
    r.unmount();
  });
  it('plugin: choosing "Highest GPU power" on Metrics sends one ranked query, then the page\'s series', async () => {
    lib.resetHeadlamp();
    lib.lists.Node = [names(12).map((x) => makeGpuNode(x)), null];
    lib.lists.Pod = [[], null];
    const fake = prom({ data: hot(12) });
    lib.api.handler = (p) => {
      if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [] });
      if (p.indexOf('/proxy/api/v1/') >= 0) return fake(p);
      return Promise.reject(Object.assign(new Error('503'), { status: 503 }));
    };
    const plugin = createPlugin({ React: React, lib: lib, CommonComponents: CC });
    const r = render(h(plugin.routeComponent('metrics')));
    await r.settle();
    const before = fake.mock.calls.length;
    r.change(r.getByLabelText('Sort GPU nodes'), 'power');
    await r.settle();
    const sent = decoded(fake).slice(before);
    expect(sent.filter((q) => q.indexOf('topk(8,') >= 0)).toHaveLength(1);
    const range = sent.filter((q) => q.indexOf('/query_range') >= 0);
    expect(range).toHaveLength(1);
    expect(range[0]).toContain('hostname=~"mi355x-004|mi355x-009|');
    expect(r.text()).toContain('Showing 1–8 of 12 GPU nodes reporting');
    const titles = r.byTag('h2').map((n) => textOfNode(n)).filter((t) => /^mi355x-/.test(t));
    expect(titles[0]).toBe('mi355x-004 — 8 × MI355X');
    r.unmount();
  });
});

describe('telemetryScope', () => {
  it('small-cluster mode while the node list loads and while it fits one page; then the page; cluster-wide when the node list failed', () => {
    expect(telemetryScope(makeContext({ loading: true }), {})).toEqual({ enabled: true, scope: [], small: true });
    expect(telemetryScope(ctxOf(8), {})).toEqual({ enabled: true, scope: names(8), small: true });
    expect(telemetryScope(ctxOf(8), { filter: '003' })).toEqual({ enabled: true, scope: ['mi355x-003'], small: true });
    expect(telemetryScope(ctxOf(12), { page: 1 })).toEqual({ enabled: true, scope: names(12).slice(8) });
    const denied = Object.assign(makeContext({ nodes: [] }), { error: 'nodes is forbidden' });
    expect(telemetryScope(denied, {})).toEqual({ enabled: true, scope: undefined });
  });
});

describe('nodesView: one page of nodes', () => {
  it('renders at most NODES_PER_PAGE rows and cards, with a pager, whatever the node count', () => {
    const small = nodesView(ctxOf(8), {});
    const big = nodesView(ctxOf(200), {});
    const last = nodesView(ctxOf(200), { pager: { page: 24 } });
    expect(cards(big)).toEqual(names(8));
    expect(cards(last)).toEqual(names(200).slice(192));
    expect(countRows(big)).toEqual(countRows(small));
    const p = pagerOf(big);
    expect([p.total, p.pages, p.noun]).toEqual([200, 25, 'GPU nodes']);
    expect(findSection(big, 'GPU Node Summary').blocks[0].rows).toHaveLength(8);
    expect(renderPage(big)).toContain('data-testid="pager"');
  });
  it('a filter narrows rows and cards; no match leaves the pager saying so', () => {
    const vm = nodesView(ctxOf(30), { pager: { filter: '02' } });
    expect(cards(vm)).toEqual(['mi355x-002', 'mi355x-020', 'mi355x-021', 'mi355x-022', 'mi355x-023', 'mi355x-024', 'mi355x-025', 'mi355x-026']);
    const none = nodesView(ctxOf(30), { pager: { filter: 'gpu-z' } });
    expect(findSection(none, 'GPU Node Summary')).toBe(null);
    expect(pagerText(pagerOf(none))).toBe('No GPU nodes match "gpu-z"');
  });
  it('no pager without GPU nodes (the empty state stands alone)', () => {
    const vm = nodesView(makeContext({ nodes: [] }), {});
    expect(pagerOf(vm)).toBe(null);
    expect(sectionTitles(vm)).toContain('No GPU Nodes Found');
  });
});

describe('scoped queries', () => {
  it('hostname matcher escapes regex metacharacters; an empty scope matches no node', () => {
    expect(regexLiteral('a.b+c')).toBe('a\\.b\\+c');
    expect(hostnameMatcher(['n.0', 'n1'])).toBe('hostname=~"n\\\\.0|n1"');
    expect(hostnameMatcher([])).toBe('hostname="."');
  });
  it('the summary query tags each aggregate so `or` keeps them apart', () => {
    const q = summaryQuery();
    expect(q.split(' or ')).toHaveLength(3);
    ['"agg", "sum"', '"agg", "count"', '"agg", "nodes"'].forEach((t) => expect(q).toContain(t));
  });
  it('totals from aggregates equal the totals summed over every GPU', () => {
    const data = exporterData(['n0', 'n1', 'n2']);
    data[SERIES.exporter.powerCap] = [];
    const fake = prom({ data: data });
    return fake(BASE0 + '/api/v1/query?query=' + encodeURIComponent(summaryQuery())).then((r) => {
      const t = totalsFromRows(r.data.result);
      const m = joinExporterResults(splitByName(flatten(data)));
      const s = summarizeMetrics(m);
      ['gpus', 'powerWatts', 'powerCapWatts', 'vramUsedBytes', 'vramTotalBytes', 'avgGfxActivityPct', 'powerCapAssumed'].forEach((k) => {
        expect(t[k]).toBe(s[k]);
      });
      expect(t.nodes).toBe(3);
    });
  });
  it('aggregate rows never join as GPUs', () => {
    const rows = splitByName([{ metric: { __name__: SERIES.exporter.power, agg: 'sum' }, value: [0, '9'] }]);
    expect(rows.__agg).toHaveLength(1);
    expect(joinExporterResults(rows).gpus).toHaveLength(0);
  });
  it('scoped series ask for the page nodes and the cluster line', () => {
    const q = scopedSeriesQuery(['n0']);
    expect(q).toContain('hostname=~"n0"');
    expect(q).toContain('"scope", "cluster"');
  });
});

describe('metrics client: scoped snapshots', () => {
  function source(fake) {
    return createMetricsSource({ request: fake });
  }
  it('fetches only the GPUs of the scope, plus cluster totals on request, in one query', async () => {
    const fake = prom({ data: exporterData(names(12)) });
    const s = source(fake);
    const m = await s.fetchGpuMetrics('gauges', { scope: ['mi355x-003', 'mi355x-007'], summary: true });
    expect(fake.mock.calls).toHaveLength(1);
    expect(decoded(fake)[0]).toContain('hostname=~"mi355x-003|mi355x-007"');
    expect(Array.from(new Set(m.gpus.map((g) => g.nodeName)))).toEqual(['mi355x-003', 'mi355x-007']);
    expect(m.scope).toEqual(['mi355x-003', 'mi355x-007']);
    expect([m.totals.gpus, m.totals.nodes]).toEqual([96, 12]);
    expect(m.source).toBe('amd-exporter');
  });
  it('later fetches of the same scope are live-only (statics cached per node) and share unchanged GPUs', async () => {
    const fake = prom({ data: exporterData(names(3)) });
    const s = source(fake);
    const a = await s.fetchGpuMetrics('topology', { scope: ['mi355x-001'] });
    const b = await s.fetchGpuMetrics('topology', { scope: ['mi355x-001'] });
    const qs = decoded(fake);
    expect(qs[0]).toContain(SERIES.exporter.vramTotal);
    expect(qs[1]).not.toContain(SERIES.exporter.vramTotal);
    expect(b.gpus).toBe(a.gpus);
    // a new page of nodes needs their statics: asked for again
    await s.fetchGpuMetrics('topology', { scope: ['mi355x-002'] });
    expect(decoded(fake)[2]).toContain(SERIES.exporter.vramTotal);
  });
  it('an empty scope with a summary asks for the totals only', async () => {
    const fake = prom({ data: exporterData(names(2)) });
    const m = await source(fake).fetchGpuMetrics('gauges', { scope: [], summary: true });
    expect(decoded(fake)[0]).not.toContain('hostname=');
    expect(m.gpus).toHaveLength(0);
    expect(m.totals.gpus).toBe(16);
  });
  it('scoped series keep the cluster line apart', async () => {
    const fake = prom({ data: exporterData(names(2)) });
    const sr = await source(fake).fetchSeries(1800, 30, ['n0']);
    expect(Object.keys(sr.power)).toEqual(['n0']);
    expect(sr.total.power.length).toBe(2);
    expect(sr.power[TOTAL_SERIES]).toBe(undefined);
  });
});

describe('metricsView: one page of per-node cards', () => {
  async function state(n, scope) {
    const fake = prom({ data: exporterData(names(n).filter((x) => x !== 'mi355x-001')) });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuMetrics('gauges', { scope: scope, summary: true });
    const series = await s.fetchSeries(1800, 30, scope);
    return { metrics: m, series: series, fetchError: null, fetching: false };
  }
  it('summary from the cluster totals; cards for the page; a node without series gets a no-telemetry card', async () => {
    const ctx = ctxOf(20);
    const st = await state(20, names(20).slice(0, 8));
    const vm = metricsView(ctx, st, {});
    expect(rowValue(vm, 'GPUs Monitored')).toBe('152');
    expect(rowValue(vm, 'Nodes Reporting').text).toBe('19 / 20 GPU nodes (1 without telemetry)');
    expect(cards(vm)).toEqual(['mi355x-000 — 8 × MI355X', 'mi355x-001 — no telemetry'].concat(names(8).slice(2).map((x) => x + ' — 8 × MI355X')));
    const series = findSection(vm, 'Power & HBM (last 30 min)').blocks.filter((b) => b.t === 'series')[0];
    expect(Object.keys(series.power)[0]).toBe(ALL_NODES_SERIES);
    expect(pagerOf(vm).total).toBe(20);
  });
  it('cards of nodes not yet covered by the snapshot say telemetry is on its way', async () => {
    const st = await state(20, names(8));
    const vm = metricsView(ctxOf(20), st, { pager: { page: 1 } });
    expect(cards(vm)[0]).toBe('mi355x-008 — fetching telemetry…');
  });
  it('warns when the exporter hostnames match no node on the page', async () => {
    const fake = prom({ data: exporterData(['10.0.0.1', '10.0.0.2']) });
    const s = createMetricsSource({ request: fake });
    const m = await s.fetchGpuMetrics('gauges', { scope: names(2), summary: true });
    const vm = metricsView(ctxOf(2), { metrics: m, series: null, fetchError: null, fetching: false }, {});
    expect(sectionTitles(vm)).toContain('Telemetry Not Matched To Nodes');
  });
  it('a cluster-wide snapshot (terminal client) is paged over the nodes reporting', async () => {
    const fake = prom({ data: exporterData(names(12)) });
    const m = await createMetricsSource({ request: fake }).fetchGpuMetrics('gauges');
    const vm = metricsView(ctxOf(12), { metrics: m, series: null, fetchError: null, fetching: false }, { pager: { page: 1 } });
    expect(cards(vm)).toEqual(names(12).slice(8).map((x) => x + ' — 8 × MI355X'));
    expect(pagerOf(vm).noun).toBe('GPU nodes reporting');
  });
});

describe('plugin pages: pager state drives the scoped queries', () => {
  function setup(n) {
    lib.resetHeadlamp();
    const nodes = names(n).map((x) => makeGpuNode(x));
    lib.lists.Node = [nodes, null];
    lib.lists.Pod = [[makeGpuPod('train-a', { node: 'mi355x-000' })], null];
    const fake = prom({ data: exporterData(names(n)) });
    lib.api.handler = (p) => {
      if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
      if (p.indexOf('/proxy/api/v1/') >= 0) return fake(p);
      return Promise.reject(Object.assign(new Error('503'), { status: 503 }));
    };
    const plugin = createPlugin({ React: React, lib: lib, CommonComponents: CC });
    return { fake: fake, plugin: plugin };
  }
  const scoped = (fake) => decoded(fake).filter((p) => p.indexOf('/query?') >= 0 && p.indexOf('hostname=~') >= 0);

  it('GPU Nodes: the first query covers page 1; Next page asks for page 2; the filter narrows it', async () => {
    const { fake, plugin } = setup(20);
    const r = render(h(plugin.routeComponent('nodes')));
    await r.settle();
    expect(scoped(fake)).toHaveLength(1);
    expect(scoped(fake)[0]).toContain('hostname=~"' + names(8).join('|') + '"');
    expect(r.text()).toContain('Showing 1–8 of 20 GPU nodes');
    r.click(r.getByLabelText('Next page'));
    await r.settle();
    expect(scoped(fake)[1]).toContain('hostname=~"' + names(16).slice(8).join('|') + '"');
    expect(r.text()).toContain('mi355x-015');
    expect(r.text()).not.toContain('mi355x-007');
    r.change(r.getByLabelText('Filter GPU nodes by name'), 'x-019');
    await r.settle();
    expect(scoped(fake).pop()).toContain('hostname=~"mi355x-019"');
    expect(r.getByLabelText('Next page').props.disabled).toBe(true);
    r.unmount();
  });
  it('Metrics: cluster totals and the page scope in one live query', async () => {
    const { fake, plugin } = setup(12);
    const r = render(h(plugin.routeComponent('metrics')));
    await r.settle();
    const live = scoped(fake);
    expect(live).toHaveLength(1);
    expect(live[0]).toContain('"agg", "sum"');
    expect(r.text()).toContain('12 / 12 GPU nodes');
    expect(r.byTag('section').length).toBeLessThan(8 + 6);
    r.unmount();
  });
});

describe('GPU Pods / Device Plugins / Overview tables are bounded too', () => {
  const pods = (n) => Array.from({ length: n }, (_, i) => makeGpuPod('train-' + String(i).padStart(4, '0'), { node: 'mi355x-' + String(i % 50).padStart(3, '0') }));
  const withPods = (list) => makeContext({ nodes: names(50).map((x) => makeGpuNode(x)), pods: list });
  it('GPU Pods: PODS_PER_PAGE rows per page, filter on namespace/name and node', () => {
    const vm = podsView(withPods(pods(120)), {});
    expect(PODS_PER_PAGE).toBe(25);
    expect(findSection(vm, 'All GPU Pods').blocks[0].rows).toHaveLength(25);
    expect(pagerText(pagerOf(vm))).toBe('Showing 1–25 of 120 GPU pods · page 1 of 5');
    const byNode = podsView(withPods(pods(120)), { pager: { filter: 'mi355x-007' } });
    expect(findSection(byNode, 'All GPU Pods').blocks[0].rows.map((r) => r[0])).toEqual(['train-0007', 'train-0057', 'train-0107']);
    expect(rowValue(vm, 'Total GPU Pods')).toBe('120'); // the summary still counts every pod
  });
  it('pending pods: the oldest PODS_PER_PAGE, the rest counted', () => {
    const list = Array.from({ length: 40 }, (_, i) => makeGpuPod('wait-' + i, { phase: 'Pending', node: null, waiting: 'Unschedulable' }));
    const sec = findSection(podsView(withPods(list), {}), 'Attention: Pending GPU Pods');
    expect(sec.blocks[0].rows).toHaveLength(25);
    expect(rowValue(sec, 'Not shown')).toBe('15 more pending GPU pods (filter the table above by name)');
  });
  it('owners are asked for the pods of the page only', async () => {
    const fake = prom({ data: exporterData(['n0']) });
    const s = createMetricsSource({ request: fake });
    await s.fetchGpuOwners({ pods: ['ml/train-0', 'ml/train-1'] });
    expect(decoded(fake)[0]).toContain('pod=~"train-0|train-1", namespace=~"ml"');
    const none = await s.fetchGpuOwners({ pods: [] });
    expect(none.gpus).toHaveLength(0);
    expect(fake.mock.calls).toHaveLength(1);
    expect(ownersScope(withPods(pods(30)), { page: 1 }).pods).toEqual(pods(30).slice(25).map((p) => 'ml/' + p.metadata.name));
  });
  it('Overview lists at most OVERVIEW_PLUGIN_PODS operator pods, not-ready first; Device Plugins pages through them', () => {
    const ops = Array.from({ length: 30 }, (_, i) => makePluginPod('amd-dp-' + i, { ready: i !== 17 }));
    const ctx = makeContext({ nodes: [makeGpuNode('mi355x-000')], pluginPods: ops });
    const ov = findSection(overviewView(ctx), 'Plugin Daemon Pods');
    expect(ov.blocks[0].rows).toHaveLength(OVERVIEW_PLUGIN_PODS);
    expect(ov.blocks[0].rows[0][0]).toBe('amd-dp-17');
    expect(rowValue(ov, 'Readiness').text).toBe('1 not ready');
    const dp = devicePluginsView(ctx, { pager: { page: 1 } });
    expect(findSection(dp, 'Plugin Daemon Pods').blocks[0].rows.map((r) => r[0])).toEqual(ops.slice(25).map((p) => p.metadata.name));
    expect(pagerOf(dp).noun).toBe('operator pods');
  });
});
