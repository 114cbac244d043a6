/**
 * Malformed cluster objects all the way to the screen: the view-models are
 * fuzzed for exceptions in tests/js/properties.test.js; here what they build
 * from the same seeded, mutated nodes / pods / DeviceConfigs is mounted
 * through the shipped renderer on the tier's React — the harness React, real
 * React 18.3.1 (offline, where any React warning also fails the run:
 * tests/test_js_real_react.py) and react-dom in jsdom (networked CI). A
 * label or status field holding an object, an array or NaN must come out as
 * text, never as a React child React refuses.
 */
import { React, render, tier } from 'amd-test-harness';
import * as CC from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { createRenderer } from '../../../src/view/react.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { nodeColumns, nodeDetailView, podDetailView } from '../../../src/view/pages/details.js';
import { devicePluginsView } from '../../../src/view/pages/devicePlugins.js';
import { metricsView } from '../../../src/view/pages/metricsPage.js';
import { nodesView } from '../../../src/view/pages/nodes.js';
import { overviewView } from '../../../src/view/pages/overview.js';
import { podsView } from '../../../src/view/pages/pods.js';

const pages = {
  clearViewMemo, devicePluginsView, metricsView, nodeColumns, nodeDetailView, nodesView, overviewView, podDetailView, podsView,
};
import { createClusterStore } from '../../../src/api/clusterStore.js';
import { createMetricsSource } from '../../../src/api/metrics.js';
import { makeContext, makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../fixtures.js';
import { exporterData, flatten, ok } from '../promFake.js';
import { mutate, pick, rng } from '../fuzzlib.js';

const h = React.createElement;
const env = (k) => (typeof process !== 'undefined' && process.env[k]) || null;
const ROUNDS = Number(env('FUZZ_RENDER_ROUNDS') || 40);
const SEED = Number(env('FUZZ_SEED') || 9001);
// Mutations applied to each mutated object (FUZZ_MUTATIONS widens the search).
const PASSES = Number(env('FUZZ_MUTATIONS') || 1);
const mutateN = (r, o) => {
  let x = o;
  for (let i = 0; i < PASSES; i++) x = mutate(r, x, 0);
  return x;
};

/** Mount every view-model and section; a failure names the round and the view. */
function mountAll(view, round, vms, sections) {
  let mounted = 0;
  const fail = (what, e) => {
    e.message = 'round ' + round + ', ' + what + ': ' + e.message;
    throw e;
  };
  vms.forEach((vm, i) => {
    try {
      const m = render(h(view.Page, { vm, onRefresh: () => {} }));
      expect(typeof m.text()).toBe('string');
      m.unmount();
    } catch (e) {
      fail('page ' + i + ' ' + JSON.stringify(vm.title), e);
    }
    mounted++;
  });
  sections.forEach((s, i) => {
    if (!s) return;
    try {
      render(h(view.Section, { s })).unmount();
    } catch (e) {
      fail('section ' + i + ' ' + JSON.stringify(s.title), e);
    }
    mounted++;
  });
  return mounted;
}

describe('shared: malformed clusters render (' + tier + ')', () => {
  it('every page, detail section and Nodes-table cell of a mutated cluster mounts and unmounts', async () => {
    const view = createRenderer(React, CC);
    const r = rng(SEED);
    const now = Date.parse('2026-10-16T00:00:00Z');
    let mounted = 0;
    for (let round = 0; round < ROUNDS; round++) {
      const nodes = [makeGpuNode('g0'), makeGpuNode('g1', { partition: 'CPX/NPS4' }), makeNode('c0')]
        .map((n) => (r() < 0.6 ? mutateN(r, n) : n));
      const pods = [makeGpuPod('a', { node: 'g0', gpus: 2 }), makeGpuPod('b', { node: 'g1' }), makePlainPod('w', 'c0'), makePluginPod('dp')]
        .map((p) => (r() < 0.6 ? mutateN(r, p) : p));
      const dcs = [makeDeviceConfig()].map((d) => (r() < 0.6 ? mutateN(r, d) : d));
      const store = createClusterStore({
        request: (path) => Promise.resolve({ kind: 'List', items: path.indexOf('deviceconfigs') >= 0 ? dcs : [] }),
      });
      store.setNodes(nodes, null);
      store.setPods(pods, null);
      await store.refresh();
      const ctx = store.getSnapshot();
      const opts = { now };
      const vms = [pages.overviewView(ctx, opts), pages.devicePluginsView(ctx, opts), pages.nodesView(ctx, opts),
        pages.podsView(ctx, opts), pages.metricsView(ctx, { metrics: null, fetchError: null, fetching: false }, opts)];
      const sections = nodes.map((n) => pages.nodeDetailView(n, ctx, opts)).concat(pods.map((p) => pages.podDetailView(p, opts)));
      mounted += mountAll(view, round, vms, sections);
      // Nodes-table cells, as the column processor hands them to Headlamp's table (plugin.js).
      const cols = pages.nodeColumns();
      const cells = [];
      nodes.forEach((n) => cols.forEach((c) => cells.push(h('td', { key: cells.length }, h(view.Value, { v: c.getter(n) })))));
      const t = render(h('table', null, h('tbody', null, h('tr', null, cells))));
      expect(t.byTag('td')).toHaveLength(nodes.length * cols.length);
      t.unmount();
      pages.clearViewMemo();
    }
    expect(mounted).toBeGreaterThan(ROUNDS * 5);
  });

  it('telemetry from wrong-shaped Prometheus rows renders on every page that shows it', async () => {
    const view = createRenderer(React, CC);
    const r = rng(SEED + 1);
    const WRONG = [null, undefined, 0, '', 'NaN', '+Inf', '-1', [], {}, [1], { x: 1 }, 'abc'];
    const ctx = makeContext({ nodes: [makeGpuNode('n0'), makeGpuNode('n1')], pods: [makeGpuPod('train-0', { node: 'n0' })] });
    let mounted = 0;
    for (let round = 0; round < ROUNDS; round++) {
      const rows = flatten(exporterData(['n0', 'n1'])).map((row) => {
        if (r() > 0.2) return row;
        const k = pick(r, ['metric', 'value', 'metric.gpu_id', 'metric.hostname', 'value.1', 'metric.__name__', 'metric.pod',
          'metric.namespace', 'metric.card_model', 'metric.serial_number']);
        const out = JSON.parse(JSON.stringify(row));
        const path = k.split('.');
        let o = out;
        for (let i = 0; i < path.length - 1; i++) o = o[path[i]];
        o[path[path.length - 1]] = pick(r, WRONG);
        return out;
      });
      for (let i = 0, n = Math.floor(r() * 4); i < n; i++) {
        const metric = { agg: pick(r, ['rank', 'ranked', 'gpu_nodes', 'sum', 'count', pick(r, WRONG)]) };
        if (r() < 0.7) metric.hostname = pick(r, ['n0', 'n1', 'ghost', pick(r, WRONG)]);
        rows.push({ metric: metric, value: [0, pick(r, ['12', '0', '9e99'].concat(WRONG))] });
      }
      const request = (path) => Promise.resolve(/query=1$/.test(path) ? ok([{ metric: {}, value: [0, '1'] }]) : ok(rows));
      const src = createMetricsSource({ request: request });
      const m = await src.fetchGpuMetrics(pick(r, ['gauges', 'topology']), { summary: r() < 0.5, small: r() < 0.5 });
      const power = { n0: [[0, pick(r, [1, NaN, null, '3', { x: 1 }])], [30, 2]] };
      const st = { metrics: m, series: { power, vram: {} }, fetchError: null, fetching: false };
      const ro = await src.fetchGpuOwners({ rank: { by: 'power', page: 0, per: 25, filter: '' } });
      const vms = [pages.metricsView(ctx, st, { now: 0 }), pages.nodesView(ctx, { metrics: m, now: 0 }),
        pages.podsView(ctx, { metrics: m, now: 0 }), pages.podsView(ctx, { metrics: ro, now: 0, pager: { sort: 'power' } })];
      const sections = [pages.nodeDetailView(ctx.gpuNodes[0], ctx, { metrics: m, series: { power: power.n0 } }),
        pages.podDetailView(ctx.gpuPods[0], { metrics: m, series: { power: power.n0 } })];
      mounted += mountAll(view, round, vms, sections);
      pages.clearViewMemo();
    }
    expect(mounted).toBeGreaterThan(ROUNDS * 4);
  });
});
