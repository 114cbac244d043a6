/**
 * The plugin bundle (tools/bundle.js → dist-offline/main.js), executed the way
 * Headlamp executes a plugin script: one self-contained file evaluated with
 * the host's `pluginLib` (here: the harness stand-ins for React, the
 * Headlamp library and CommonComponents). The reference's CI builds its
 * bundle (`headlamp-plugin build`, /root/reference/.github/workflows/ci.yaml:169-170)
 * but never loads it; here the built file registers every extension point
 * and its pages render and fetch.
 */
import path from 'path';
import { fileURLToPath } from 'url';
import React, { render } from './stubs/react.js';
import * as lib from './stubs/headlamp-lib.js';
import * as CC from './stubs/CommonComponents.js';
import { bundle, transformModule, EXTERNALS } from '../../tools/bundle.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../src/api/k8sCore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from './fixtures.js';

const ROOT = path.resolve(path.dirname(fileURLToPath(import.meta.url)), '..', '..');
const h = React.createElement;
const built = bundle(path.join(ROOT, 'src', 'index.tsx'));

function pluginLib() {
  return Object.assign({}, lib, { React: React, CommonComponents: Object.assign({}, CC) });
}

/** Evaluate the bundle as a plugin script; returns the entry module's exports. */
function load(libObj) {
  // eslint-disable-next-line no-new-func
  return new Function('pluginLib', 'return (' + built.code.trim().replace(/;$/, '') + '\n);')(libObj);
}

function load2(code) {
  // eslint-disable-next-line no-new-func
  return new Function('pluginLib', 'return (' + code.trim().replace(/;$/, '') + '\n);')(pluginLib());
}

function cluster() {
  lib.lists.Node = [[makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1'), makeNode('cpu-0')], null];
  lib.lists.Pod = [[makeGpuPod('train-a', { gpus: 4 }), makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' }), makePlainPod('web-0'), makePluginPod('amdgpu-dp-0')], null];
  lib.api.handler = (p) => {
    if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
}

beforeEach(() => {
  lib.resetHeadlamp();
});

describe('tools/bundle.js', () => {
  it('bundles the entry and the modules it imports, nothing from the harness', () => {
    expect(built.modules[built.modules.length - 1]).toBe('src/index.tsx');
    ['src/headlamp.ts', 'src/plugin.js', 'src/api/providerCore.js', 'src/api/clusterStore.js', 'src/api/metrics.js', 'src/view/pages/overview.js', 'src/view/react.js'].forEach((m) => {
      expect(built.modules).toContain(m);
    });
    built.modules.forEach((m) => expect(m.indexOf('tests/')).toBe(-1));
    // dependencies before dependants
    expect(built.modules.indexOf('src/api/amdNodes.js')).toBeLessThan(built.modules.indexOf('src/api/clusterStore.js'));
  });

  it('leaves no module syntax and only host modules outside', () => {
    expect(/^\s*(import|export)\s/m.test(built.code)).toBe(false);
    expect(built.code).not.toContain("from '");
    expect(Object.keys(EXTERNALS).sort()).toEqual(['@kinvolk/headlamp-plugin/lib', '@kinvolk/headlamp-plugin/lib/CommonComponents', 'react']);
  });

  it('fails loudly without the host library', () => {
    expect(() => load(undefined)).toThrow('pluginLib');
    const noCC = pluginLib();
    delete noCC.CommonComponents;
    expect(() => load(noCC)).toThrow('CommonComponents');
  });

  it('registers every extension point at load, like src/index.tsx', () => {
    const mod = load(pluginLib());
    expect(mod.registered).toEqual({ sidebar: 6, routes: 5, detailSections: 2, columnProcessors: 1, settings: true });
    expect(lib.registry.sidebar.map((e) => e.label)).toEqual(['AMD GPU', 'Overview', 'Device Plugins', 'GPU Nodes', 'GPU Pods', 'Metrics']);
    expect(lib.registry.routes.map((r) => r.path)).toEqual(['/amd-gpu', '/amd-gpu/device-plugins', '/amd-gpu/nodes', '/amd-gpu/pods', '/amd-gpu/metrics']);
  });

  it('a bundled route renders and its Refresh issues one CRD request', async () => {
    load(pluginLib());
    cluster();
    const overview = lib.registry.routes[0].component;
    const r = render(h(overview));
    await r.settle();
    expect(r.instances(CC.SectionHeader)[0].props.title).toBe('AMD GPU — Overview');
    const n = lib.api.calls.length;
    r.click(r.getByLabelText('Refresh AMD GPU data'));
    await r.settle();
    expect(lib.api.calls.slice(n)).toEqual([DEVICE_CONFIG_LIST_PATH]);
    r.unmount();
  });

  it('the bundled Nodes page, detail section and table columns see the GPU nodes', async () => {
    load(pluginLib());
    cluster();
    const r = render(h(lib.registry.routes[2].component));
    await r.settle();
    expect(r.html()).toContain('mi355x-1');
    expect(r.html()).not.toContain('cpu-0');
    r.unmount();
    const cols = lib.registry.columns[0]({ id: 'headlamp-nodes', columns: [{ label: 'Name' }] });
    expect(cols.map((c) => c.label)).toEqual(['Name', 'GPU Model', 'GPU Devices', 'GPU HBM']);
    const node = lib.registry.details[0]({ resource: { kind: 'Node', jsonData: makeGpuNode('mi355x-0') } });
    expect(node).not.toBe(null);
    expect(lib.registry.details[0]({ resource: { kind: 'Pod', jsonData: makePlainPod('web-0') } })).toBe(null);
  });
});

describe('transformModule', () => {
  const file = path.join(ROOT, 'src', 'x.js');
  const dep = (from, spec) => 'src/' + spec.replace('./', '');

  it('turns imports into module-table lookups and exports into live getters', () => {
    const t = transformModule(
      "import { a, b as c } from './y.js';\nimport D from './z.js';\nexport let n = 1;\nexport function f() { return a + c + D; }\nexport { n as m };\nexport default f;\n",
      file,
      dep,
    );
    expect(t.deps).toEqual(['src/y.js', 'src/z.js']);
    const mods = { 'src/y.js': { a: 1, b: 2 }, 'src/z.js': { default: 3 } };
    const exportsObj = {};
    // eslint-disable-next-line no-new-func
    new Function('__exports', '__req', '__ext', '__export', '__default', '__missing', t.code)(
      exportsObj,
      (id) => mods[id],
      null,
      (o, k, g) => Object.defineProperty(o, k, { enumerable: true, get: g }),
      (m) => (m.default !== undefined ? m.default : m),
      (name) => { throw new Error('missing ' + name); },
    );
    expect(exportsObj.f()).toBe(6);
    expect(exportsObj.default).toBe(exportsObj.f);
    expect(exportsObj.m).toBe(1);
  });

  it('exports every name a destructuring declaration binds (src/headlamp.ts)', () => {
    const t = transformModule("import { plugin } from './y.js';\nexport const { Page, Section: S, ...rest } = plugin.view;\n", file, dep);
    const exportsObj = {};
    // eslint-disable-next-line no-new-func
    new Function('__exports', '__req', '__ext', '__export', '__default', '__missing', t.code)(
      exportsObj,
      () => ({ plugin: { view: { Page: 1, Section: 2, Value: 3 } } }),
      null,
      (o, k, g) => Object.defineProperty(o, k, { enumerable: true, get: g }),
      (m) => m,
      (name) => { throw new Error('missing ' + name); },
    );
    expect(Object.keys(exportsObj).sort()).toEqual(['Page', 'S', 'rest']);
    expect(exportsObj.S).toBe(2);
    expect(exportsObj.rest).toEqual({ Value: 3 });
  });

  it('bundles every TypeScript module under src/ (the binding, not only through the entry)', () => {
    const shims = ['src/headlamp.ts', 'src/index.tsx'];
    shims.forEach((f) => {
      const b = bundle(path.join(ROOT, f));
      expect(b.modules[b.modules.length - 1]).toBe(f);
      const mod = load2(b.code);
      expect(Object.keys(mod).length).toBeGreaterThan(0);
    });
  });

  it('rejects what it does not understand instead of passing it through', () => {
    expect(() => transformModule("export * from './y.js';\n", file, dep)).toThrow('unsupported statement');
    expect(() => transformModule("import x from 'lodash';\n", file, dep)).toThrow('not a host module');
    expect(() => transformModule("const m = import('./y.js');\n", file, dep)).toThrow('dynamic import');
  });
});
