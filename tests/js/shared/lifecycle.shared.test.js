/**
 * Nothing outlives a view: with auto-refresh on, every route and both detail
 * sections start pollers (setInterval), tab-visibility listeners (in a DOM)
 * and a subscription to the shared cluster store; leaving them must release
 * all of it, however many times the user switches. The reference clears
 * nothing of the kind (its request timeouts stay armed: SURVEY Q6); here a
 * route switch loop leaves the process exactly as it found it. Runs on the
 * harness React and on real React 18.3.1 (both offline) and on react-dom in
 * jsdom (networked CI).
 */
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import '../../../src/index.tsx';
import { resetSharedStores, sharedStores } from '../../../src/api/clusterStore.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { DEFAULT_SETTINGS, invalidateSettings, saveSettings } from '../../../src/api/settings.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../../src/api/k8sCore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../fixtures.js';
import { exporterData, prom } from '../promFake.js';

const h = React.createElement;
const reg = { routes: lib.registry.routes.slice(), details: lib.registry.details.slice() };
const NODES = ['mi355x-000', 'mi355x-001'];

function cluster() {
  const pods = [makeGpuPod('train-a', { gpus: 4, node: NODES[0] }), makeGpuPod('train-b', { gpus: 2, node: NODES[1] }),
    makePlainPod('web-0'), makePluginPod('amdgpu-dp-0')];
  lib.lists.Node = [NODES.map((n) => makeGpuNode(n)).concat([makeNode('cpu-0')]), null];
  lib.lists.Pod = [pods, null];
  const fake = prom({ data: exporterData(NODES) });
  lib.api.handler = (path) => {
    if (path === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
    if (path.indexOf('/proxy/api/v1/') >= 0) return fake(path);
    if (path.indexOf('/api/v1/pods?fieldSelector=') === 0) return Promise.resolve({ kind: 'List', metadata: {}, items: pods.slice(0, 1) });
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
}

/** Live setInterval handles and visibilitychange listeners, counted through wrappers. */
function track() {
  const g = globalThis;
  const saved = { setInterval: g.setInterval, clearInterval: g.clearInterval };
  const live = new Set();
  g.setInterval = function () {
    const id = saved.setInterval.apply(g, arguments);
    live.add(id);
    return id;
  };
  g.clearInterval = function (id) {
    live.delete(id);
    return saved.clearInterval.call(g, id);
  };
  const doc = typeof document !== 'undefined' && document && typeof document.addEventListener === 'function' ? document : null;
  const listeners = new Set();
  let docSaved = null;
  if (doc) {
    docSaved = { add: doc.addEventListener, remove: doc.removeEventListener };
    doc.addEventListener = function (type, fn) {
      if (type === 'visibilitychange') listeners.add(fn);
      return docSaved.add.apply(doc, arguments);
    };
    doc.removeEventListener = function (type, fn) {
      if (type === 'visibilitychange') listeners.delete(fn);
      return docSaved.remove.apply(doc, arguments);
    };
  }
  return {
    intervals: () => live.size,
    visibility: () => listeners.size,
    hasDocument: !!doc,
    restore: () => {
      g.setInterval = saved.setInterval;
      g.clearInterval = saved.clearInterval;
      if (doc) {
        doc.addEventListener = docSaved.add;
        doc.removeEventListener = docSaved.remove;
      }
    },
  };
}

let t = null;

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  clearViewMemo();
  if (typeof sessionStorage !== 'undefined' && sessionStorage) sessionStorage.clear();
  saveSettings(Object.assign({}, DEFAULT_SETTINGS, { refreshIntervalSec: 30 }));
  t = track();
});

afterEach(() => {
  t.restore();
  saveSettings(DEFAULT_SETTINGS);
  invalidateSettings();
});

describe('shared: nothing outlives a view (' + tier + ')', () => {
  it('switching through every route 8 times leaves no poller, listener or store subscription behind', async () => {
    cluster();
    const views = reg.routes.map((r) => () => h(r.component))
      .concat([() => reg.details[0]({ resource: { kind: 'Node', jsonData: makeGpuNode(NODES[1]) } }),
        () => reg.details[1]({ resource: { kind: 'Pod', jsonData: makeGpuPod('train-a', { gpus: 4, node: NODES[0] }) } })]);
    expect(views).toHaveLength(7);
    for (let round = 0; round < 8; round++) {
      for (let v = 0; v < views.length; v++) {
        const r = render(views[v]());
        await r.settle(4);
        // auto-refresh is on: the view polls while it is shown
        expect(t.intervals()).toBeGreaterThan(0);
        if (t.hasDocument) expect(t.visibility()).toBe(t.intervals());
        r.unmount();
        expect(t.intervals()).toBe(0);
        expect(t.visibility()).toBe(0);
      }
    }
    expect(sharedStores()).toHaveLength(1);
    expect(sharedStores()[0].counters().subscribers).toBe(0);
  });

  it('two views of the same store subscribe and release independently', async () => {
    cluster();
    const a = render(h(reg.routes[0].component));
    await a.settle(4);
    expect(sharedStores()).toHaveLength(1);
    const store = sharedStores()[0];
    const one = store.counters().subscribers;
    expect(one).toBeGreaterThan(0);
    const b = render(h(reg.routes[2].component));
    await b.settle(4);
    expect(store.counters().subscribers).toBeGreaterThan(one);
    a.unmount();
    expect(store.counters().subscribers).toBeGreaterThan(0);
    expect(t.intervals()).toBeGreaterThan(0);
    b.unmount();
    expect(store.counters().subscribers).toBe(0);
    expect(t.intervals()).toBe(0);
  });
});
