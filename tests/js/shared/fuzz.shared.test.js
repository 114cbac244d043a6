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
import * as pages from '../../../src/view/pages.js';
import { createClusterStore } from '../../../src/api/clusterStore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../fixtures.js';
import { mutate, rng } from '../fuzzlib.js';

const h = React.createElement;
const ROUNDS = Number((typeof process !== 'undefined' && process.env.FUZZ_RENDER_ROUNDS) || 40);

describe('shared: malformed clusters render (' + tier + ')', () => {
  it('every page, detail section and Nodes-table cell of a mutated cluster mounts and unmounts', async () => {
    const view = createRenderer(React, CC);
    const r = rng(Number((typeof process !== 'undefined' && process.env.FUZZ_SEED) || 9001));
    const now = Date.parse('2026-10-16T00:00:00Z');
    let mounted = 0;
    for (let round = 0; round < ROUNDS; round++) {
      const nodes = [makeGpuNode('g0'), makeGpuNode('g1', { partition: 'CPX/NPS4' }), makeNode('c0')]
        .map((n) => (r() < 0.6 ? mutate(r, n, 0) : n));
      const pods = [makeGpuPod('a', { node: 'g0', gpus: 2 }), makeGpuPod('b', { node: 'g1' }), makePlainPod('w', 'c0'), makePluginPod('dp')]
        .map((p) => (r() < 0.6 ? mutate(r, p, 0) : p));
      const dcs = [makeDeviceConfig()].map((d) => (r() < 0.6 ? mutate(r, d, 0) : d));
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
      const where = (what) => (e) => {
        e.message = 'round ' + round + ', ' + what + ': ' + e.message;
        throw e;
      };
      vms.forEach((vm, i) => {
        try {
          const m = render(h(view.Page, { vm, onRefresh: () => {} }));
          expect(typeof m.text()).toBe('string');
          m.unmount();
        } catch (e) {
          where('page ' + i + ' ' + JSON.stringify(vm.title))(e);
        }
        mounted++;
      });
      const sections = nodes.map((n) => pages.nodeDetailView(n, ctx, opts)).concat(pods.map((p) => pages.podDetailView(p, opts)));
      sections.forEach((s, i) => {
        if (!s) return;
        try {
          render(h(view.Section, { s })).unmount();
        } catch (e) {
          where('section ' + i + ' ' + JSON.stringify(s.title))(e);
        }
        mounted++;
      });
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
});
