/**
 * Randomised check of the paged pages' first wave (metrics.js sizeGuard /
 * smallClusterQuery, pages.js telemetryScope, providerCore.js smallKey):
 * whatever the cluster — 0 to 20 listed GPU nodes, some without exporter
 * series, stale exporter hostnames the node list lacks, any order and filter
 * — a cold Metrics page settles with telemetry for every node of its page
 * that reports, "no telemetry" for the others, nothing still "fetching", and
 * at most three live queries (the guarded first wave, the page once the list
 * names a larger cluster, the names once an answer found more than a page).
 * Seeded, so a failure reproduces.
 */
import React, { render } from './stubs/react.js';
import * as lib from './stubs/headlamp-lib.js';
import * as CC from './stubs/CommonComponents.js';
import { createPlugin } from '../../src/plugin.js';
import { resetSharedStores } from '../../src/api/clusterStore.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../src/api/k8sCore.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { NODE_SORTS, nodePage } from '../../src/view/pages/paging.js';
import { makeContext, makeGpuNode, makeGpuPod } from './fixtures.js';
import { exporterData, prom } from './promFake.js';

const h = React.createElement;

function rng(seed) {
  let a = seed >>> 0;
  return function () {
    a = (a + 0x6d2b79f5) >>> 0;
    let t = a;
    t = Math.imul(t ^ (t >>> 15), t | 1);
    t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}
const int = (r, lo, hi) => lo + Math.floor(r() * (hi - lo + 1));

describe('cold Metrics page, random clusters', () => {
  for (let seed = 1; seed <= 40; seed++) {
    it('seed ' + seed, async () => {
      const r = rng(seed);
      lib.resetHeadlamp();
      resetSharedStores();
      clearViewMemo();
      const listed = Array.from({ length: int(r, 0, 20) }, (_, i) => 'mi355x-' + String(i).padStart(3, '0'));
      const reporting = listed.filter(() => r() < 0.8);
      const stale = Array.from({ length: int(r, 0, 10) }, (_, i) => 'gone-' + i);
      const nodes = listed.map((n) => makeGpuNode(n, { ready: r() < 0.9 }));
      const pods = listed.filter(() => r() < 0.5).map((n, i) => makeGpuPod('w' + i, { gpus: int(r, 1, 8), node: n }));
      const pager = { page: 0, filter: r() < 0.3 ? 'x-0' + int(r, 0, 1) : '', sort: NODE_SORTS[int(r, 0, NODE_SORTS.length - 1)].value };
      const fake = prom({ data: exporterData(reporting.concat(stale)) });
      lib.lists.Node = [null, null];
      lib.lists.Pod = [null, null];
      lib.api.handler = (p) => {
        if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [] });
        if (p.indexOf('/proxy/api/v1/') >= 0) return fake(p);
        return Promise.reject(Object.assign(new Error('503'), { status: 503 }));
      };
      // The page opens on a stored pager state (plugin.js usePager / settings.js loadViewState).
      const mem = {};
      const storage = { getItem: (k) => (k in mem ? mem[k] : null), setItem: (k, v) => { mem[k] = v; } };
      const plugin = createPlugin({ React, lib, CommonComponents: CC, viewStorage: storage });
      storage.setItem('headlamp-amd-gpu-plugin.view.__default__|metrics', JSON.stringify(pager));
      const Page = plugin.routeComponent('metrics');
      const view = render(h(Page));
      await view.settle();
      lib.lists.Node = [nodes, null];
      lib.lists.Pod = [pods, null];
      view.rerender(h(Page));
      await view.settle(40);
      const live = fake.mock.calls.map((c) => decodeURIComponent(c[0])).filter((q) => /\/query\?query=(?!1$)/.test(q));
      expect(live.length).toBeLessThanOrEqual(3);
      const text = view.text();
      expect(text).not.toContain('fetching telemetry');
      if (listed.length === 0) return;
      const ctx = makeContext({ nodes, pods });
      const shown = nodePage(ctx.gpuNodes, pager, ctx.index).names;
      shown.forEach((n) => {
        expect(text).toContain(reporting.indexOf(n) >= 0 ? n + ' — 8 × MI355X' : n + ' — no telemetry');
      });
      view.unmount();
    });
  }
});
