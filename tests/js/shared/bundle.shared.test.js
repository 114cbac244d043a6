/**
 * The built plugin bundle (tools/bundle.js → the single script Headlamp
 * loads) evaluated with a host `pluginLib` whose React is the tier's React:
 * the harness React offline, and REAL React 18.3.1 + react-dom — offline via
 * the UMD builds (tests/test_js_real_react.py) and under jsdom in networked
 * CI. So the shipped file, not only its source modules, registers and renders
 * on the React Headlamp provides. tests/js/bundle.test.js holds the
 * harness-only checks of the bundle (module order, externals, every shim).
 */
import path from 'path';
import { fileURLToPath } from 'url';
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import * as CC from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { bundle } from '../../../tools/bundle.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../../src/api/k8sCore.js';
import { resetSharedStores } from '../../../src/api/clusterStore.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../fixtures.js';

const ROOT = path.resolve(path.dirname(fileURLToPath(import.meta.url)), '..', '..', '..');
const h = React.createElement;
const built = bundle(path.join(ROOT, 'src', 'index.tsx'));

/** Evaluate the bundle as Headlamp does: one script, the host library as `pluginLib`. */
function loadBundle() {
  const pluginLib = Object.assign({}, lib, { React: React, CommonComponents: Object.assign({}, CC) });
  // eslint-disable-next-line no-new-func
  return new Function('pluginLib', 'return (' + built.code.trim().replace(/;$/, '') + '\n);')(pluginLib);
}

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  clearViewMemo();
  lib.lists.Node = [[makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1'), makeNode('cpu-0')], null];
  lib.lists.Pod = [[makeGpuPod('train-a', { gpus: 4 }), makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' }), makePlainPod('web-0'),
    makePluginPod('amdgpu-dp-0')], null];
  lib.api.handler = (p) => {
    if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
});

describe('shared: the built bundle on the host React (' + tier + ')', () => {
  it('registers every extension point and its Overview renders and refreshes', async () => {
    const mod = loadBundle();
    expect(mod.registered).toEqual({ sidebar: 6, routes: 5, detailSections: 2, columnProcessors: 1, settings: true });
    const overview = lib.registry.routes.find((r) => r.path === '/amd-gpu').component;
    const r = render(h(overview));
    await r.settle();
    expect(r.text()).toContain('AMD GPU — Overview');
    expect(r.text()).toContain('mi355x-1');
    const crd = () => lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH).length;
    const before = crd();
    r.click(r.byLabel('Refresh AMD GPU data'));
    await r.settle();
    expect(crd()).toBe(before + 1);
    r.unmount();
  });

  it('its GPU Nodes page and Node detail section render', async () => {
    loadBundle();
    const nodes = lib.registry.routes.find((r) => r.path === '/amd-gpu/nodes').component;
    const a = render(h(nodes));
    await a.settle();
    expect(a.text()).toContain('GPU Node Summary');
    // one page of nodes: the pager is its count line until asked for its controls
    a.click(a.byLabel('Filter or sort GPU nodes'));
    await a.settle();
    expect(a.byLabel('Sort GPU nodes')).toBeTruthy();
    a.unmount();
    const b = render(lib.registry.details[0]({ resource: { kind: 'Node', jsonData: makeGpuNode('mi355x-1') } }));
    await b.settle();
    expect(b.text()).toContain('AMD GPU');
    b.unmount();
  });
});
