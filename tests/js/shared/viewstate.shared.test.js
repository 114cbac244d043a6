/**
 * A page keeps its place (pager page, filter, order) for the browser tab:
 * leave GPU Nodes and come back, and it reopens where it was (plugin.js
 * usePager → settings.js saveViewState / loadViewState), per page and per
 * cluster. Driven through the controls on the harness React and on real
 * React 18.3.1; the storage is injected (`viewStorage`), as a tab's
 * sessionStorage would be.
 */
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import * as CC from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { createPlugin } from '../../../src/plugin.js';
import { resetSharedStores } from '../../../src/api/clusterStore.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { makeGpuNode } from '../fixtures.js';

const h = React.createElement;

function memStorage() {
  const m = {};
  return { getItem: (k) => (k in m ? m[k] : null), setItem: (k, v) => { m[k] = String(v); }, m };
}

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  clearViewMemo();
});

describe('shared: a page keeps its place for the tab (' + tier + ')', () => {
  it('GPU Nodes reopens on the same order, filter and page; Metrics keeps its own', async () => {
    const names = Array.from({ length: 20 }, (_, i) => 'mi355x-' + String(i).padStart(3, '0'));
    lib.lists.Node = [names.map((n) => makeGpuNode(n)), null];
    lib.lists.Pod = [[], null];
    lib.api.handler = () => Promise.reject(Object.assign(new Error('503'), { status: 503 }));
    const storage = memStorage();
    const plugin = createPlugin({ React, lib, CommonComponents: CC, viewStorage: storage });
    const a = render(h(plugin.routeComponent('nodes')));
    await a.settle();
    a.change(a.byLabel('Sort GPU nodes'), 'attention');
    a.change(a.byLabel('Filter GPU nodes by name'), 'x-01');
    await a.settle();
    a.click(a.byLabel('Next page'));
    await a.settle();
    expect(a.text()).toContain('Showing 9–10 of 10 matching "x-01" (20 GPU nodes)');
    a.unmount();
    const b = render(h(plugin.routeComponent('nodes')));
    await b.settle();
    expect(b.text()).toContain('Showing 9–10 of 10 matching "x-01" (20 GPU nodes)');
    expect(b.value(b.byLabel('Sort GPU nodes'))).toBe('attention');
    expect(b.value(b.byLabel('Filter GPU nodes by name'))).toBe('x-01');
    b.unmount();
    const m = render(h(plugin.routeComponent('metrics')));
    await m.settle();
    m.unmount();
    const keys = Object.keys(storage.m);
    expect(keys.every((k) => k.indexOf('headlamp-amd-gpu-plugin.view.') === 0)).toBe(true);
    const metricsKey = keys.filter((k) => /\|metrics$/.test(k))[0];
    expect(JSON.parse(storage.m[metricsKey])).toEqual({ page: 0, filter: '', sort: 'name' });
  });
});
