/**
 * The shipped entry point, executed: `src/index.tsx` (and through it
 * `src/headlamp.ts` and `src/plugin.js`) is imported exactly as Headlamp's
 * bundler would, with 'react' and '@kinvolk/headlamp-plugin/lib[/CommonComponents]'
 * resolved to the harness stand-ins (tools/plugin-loader.js under Node;
 * vitest.config.mts aliases under vitest). Registration runs at module load
 * like the reference (src/index.tsx:35-182); every registered component is
 * then mounted and driven. The reference's registration is untested
 * (SURVEY.md §4 gaps); its page specs mock CommonComponents the same way
 * (src/components/OverviewPage.test.tsx:8-61).
 */
import React, { render } from './stubs/react.js';
import * as lib from './stubs/headlamp-lib.js';
import * as CC from './stubs/CommonComponents.js';
import { registered } from '../../src/index.tsx';
import { plugin } from '../../src/headlamp.ts';
import {
  AmdGpuDataProvider, buildNodeGpuColumns, MetricsPage as MetricsTsx, OverviewPage as OverviewTsx, Page, Section, useAmdGpuContext,
} from '../../src/headlamp.ts';
import { PLUGIN_NAME, createPlugin, registerPlugin } from '../../src/plugin.js';
import { resetSharedStores } from '../../src/api/clusterStore.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { isAmdGpuPluginPod } from '../../src/api/amdPods.js';
import { DEVICE_CONFIG_LIST_PATH, PLUGIN_POD_QUERIES } from '../../src/api/k8sCore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from './fixtures.js';
import { exporterData, prom } from './promFake.js';
import { SERIES } from '../../src/api/series.js';

const h = React.createElement;

// Registration happened at import time; keep a copy before any reset.
const reg = {
  sidebar: lib.registry.sidebar.slice(),
  routes: lib.registry.routes.slice(),
  details: lib.registry.details.slice(),
  columns: lib.registry.columns.slice(),
  settings: lib.registry.settings.slice(),
};

function kubeList(items) {
  return { kind: 'List', metadata: {}, items: items };
}

function cluster(o) {
  const opt = Object.assign({ nodes: true, pods: true }, o || {});
  lib.lists.Node = opt.nodes === true ? [[makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1'), makeNode('cpu-0')], null] : opt.nodes;
  lib.lists.Pod = opt.pods === true
    ? [[makeGpuPod('train-a', { gpus: 4 }), makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' }), makePlainPod('web-0'), makePluginPod('amdgpu-dp-0')], null]
    : opt.pods;
  lib.api.handler = (path) => {
    if (path === DEVICE_CONFIG_LIST_PATH) return Promise.resolve(kubeList([makeDeviceConfig()]));
    // One node's pods (the cold Node detail section's field-selected list).
    const fs = /^\/api\/v1\/pods\?fieldSelector=(.*)$/.exec(path);
    if (fs) {
      const node = decodeURIComponent(fs[1]).replace(/^spec\.nodeName=/, '');
      const list = lib.lists.Pod;
      if (!list || !list[0]) return Promise.reject(Object.assign(new Error(list && list[1] ? list[1] : 'pods is forbidden'), { status: 403 }));
      return Promise.resolve(kubeList(list[0].filter((p) => p.spec && p.spec.nodeName === node)));
    }
    // The plugin-pod requests (label selector across namespaces, the operator
    // namespace), answered from the same pod list as an apiserver would.
    const q = PLUGIN_POD_QUERIES.indexOf(path);
    if (q >= 0) {
      const list = lib.lists.Pod;
      const all = list && list[0] ? list[0] : [];
      return Promise.resolve(kubeList(all.filter((p) => (q === 0 ? isAmdGpuPluginPod(p) && p.metadata.namespace !== 'kube-amd-gpu' : p.metadata.namespace === 'kube-amd-gpu'))));
    }
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
}

function route(path) {
  const r = reg.routes.find((x) => x.path === path);
  expect(r).toBeTruthy();
  return r.component;
}

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  clearViewMemo();
});

describe('registration at module load (src/index.tsx)', () => {
  it('reports what it registered', () => {
    expect(registered).toEqual({ sidebar: 6, routes: 5, detailSections: 2, columnProcessors: 1, settings: true });
  });

  it('registers the sidebar root and five children', () => {
    expect(reg.sidebar.map((e) => e.label)).toEqual(['AMD GPU', 'Overview', 'Device Plugins', 'GPU Nodes', 'GPU Pods', 'Metrics']);
  });

  it('registers five exact routes with components', () => {
    expect(reg.routes.map((r) => r.path)).toEqual(['/amd-gpu', '/amd-gpu/device-plugins', '/amd-gpu/nodes', '/amd-gpu/pods', '/amd-gpu/metrics']);
    reg.routes.forEach((r) => {
      expect(r.exact).toBe(true);
      expect(typeof r.component).toBe('function');
    });
  });

  it('registers the settings page under the plugin name without a save button', () => {
    expect(reg.settings).toHaveLength(1);
    expect(reg.settings[0].name).toBe(PLUGIN_NAME);
    expect(reg.settings[0].component).toBe(plugin.SettingsPage);
    expect(reg.settings[0].showSave).toBe(false);
  });

  it('skips plugin settings on hosts without registerPluginSettings', () => {
    const calls = [];
    const old = Object.assign({}, lib, { registerPluginSettings: undefined });
    ['registerSidebarEntry', 'registerRoute', 'registerDetailsViewSection', 'registerResourceTableColumnsProcessor'].forEach((k) => {
      old[k] = (x) => calls.push(k);
    });
    const res = registerPlugin(old, plugin);
    expect(res.settings).toBe(false);
    expect(calls.length).toBe(6 + 5 + 2 + 1);
  });

  it('the TSX shims re-export the plugin built from the real modules', () => {
    expect(OverviewTsx).toBe(plugin.OverviewPage);
    expect(MetricsTsx).toBe(plugin.MetricsPage);
    expect(AmdGpuDataProvider).toBe(plugin.AmdGpuDataProvider);
    expect(useAmdGpuContext).toBe(plugin.useAmdGpuContext);
    expect(Page).toBe(plugin.view.Page);
    expect(Section).toBe(plugin.view.Section);
    expect(buildNodeGpuColumns).toBe(plugin.buildNodeGpuColumns);
  });

  it('createPlugin refuses an incomplete environment', () => {
    expect(() => createPlugin({ React, lib })).toThrow('CommonComponents');
  });
});

describe('route components', () => {
  const pages = [
    ['/amd-gpu', 'AMD GPU — Overview', 'Refresh AMD GPU data'],
    ['/amd-gpu/device-plugins', 'AMD GPU — Device Plugins', 'Refresh device plugin data'],
    ['/amd-gpu/nodes', 'AMD GPU — Nodes', 'Refresh node data'],
    ['/amd-gpu/pods', 'AMD GPU — Pods', 'Refresh pod data'],
    ['/amd-gpu/metrics', 'AMD GPU — Metrics', 'Refresh metrics'],
  ];

  it.each(pages)('%s renders its header and refresh button', async (path, title, aria) => {
    cluster();
    const r = render(h(route(path)));
    await r.settle();
    expect(r.instances(CC.SectionHeader)[0].props.title).toBe(title);
    const btn = r.getByLabelText(aria);
    expect(btn.props.disabled).toBe(false);
  });

  it('shows the loader until the lists arrive', async () => {
    cluster({ nodes: [null, null], pods: [null, null] });
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    expect(r.instances(CC.Loader)[0].props.title).toBe('Loading AMD GPU data...');
    expect(r.instances(CC.SectionHeader)).toHaveLength(0);
  });

  it('Overview: clicking Refresh issues one CRD request', async () => {
    cluster();
    const r = render(h(route('/amd-gpu')));
    await r.settle();
    const n = lib.api.calls.length;
    r.click(r.getByLabelText('Refresh AMD GPU data'));
    await r.settle();
    expect(lib.api.calls.slice(n)).toEqual([DEVICE_CONFIG_LIST_PATH]);
  });

  it('switching routes reuses the shared store: no second CRD request', async () => {
    cluster();
    const r1 = render(h(route('/amd-gpu')));
    await r1.settle();
    r1.unmount();
    const r2 = render(h(route('/amd-gpu/device-plugins')));
    expect(r2.instances(CC.Loader)).toHaveLength(0);
    await r2.settle();
    expect(lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH)).toHaveLength(1);
  });

  it('Nodes page draws a SimpleTable row per GPU node and one xGMI matrix per node', async () => {
    cluster();
    const r = render(h(route('/amd-gpu/nodes')));
    await r.settle();
    const html = r.html();
    expect(html).toContain('mi355x-0');
    expect(html).toContain('mi355x-1');
    expect(html).not.toContain('cpu-0');
    // one slot strip and one (closed) xGMI matrix per node
    expect(r.queryAll((n) => n.props['data-slots'] !== undefined)).toHaveLength(2);
    expect(r.queryAll((n) => n.props['data-matrix'] === 'closed')).toHaveLength(2);
  });

  it('Pods page lists GPU pods only', async () => {
    cluster();
    const r = render(h(route('/amd-gpu/pods')));
    await r.settle();
    const html = r.html();
    expect(html).toContain('train-a');
    expect(html).toContain('train-b');
    expect(html).not.toContain('web-0');
  });

  it('Device Plugins page shows the DeviceConfig and the operand pod', async () => {
    cluster();
    const r = render(h(route('/amd-gpu/device-plugins')));
    await r.settle();
    const titles = r.instances(CC.SectionBox).map((i) => i.props.title);
    expect(titles).toContain('DeviceConfig: gpu-operator');
    expect(r.html()).toContain('amdgpu-dp-0');
  });

  it('Metrics page: Prometheus unreachable section, Refresh enabled', async () => {
    cluster();
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    const titles = r.instances(CC.SectionBox).map((i) => i.props.title);
    expect(titles).toContain('Prometheus Unreachable');
    expect(r.getByLabelText('Refresh metrics').props.disabled).toBe(false);
  });

  it.each([
    ['pods forbidden', true, [null, 'pods is forbidden']],
    ['nodes forbidden', [null, 'nodes is forbidden'], true],
    ['both forbidden', [null, 'nodes is forbidden'], [null, 'pods is forbidden']],
  ])('Metrics Refresh is enabled and nothing spins when %s', async (_, nodes, pods) => {
    cluster({ nodes, pods });
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    expect(r.getByLabelText('Refresh metrics').props.disabled).toBe(false);
    expect(r.instances(CC.Loader)).toHaveLength(0);
  });
});

describe('detail sections', () => {
  function nodeSection(resource) {
    return reg.details[0]({ resource });
  }
  function podSection(resource) {
    return reg.details[1]({ resource });
  }

  it('Node detail: AMD node renders the AMD GPU section with its workload pods', async () => {
    cluster();
    const el = nodeSection(makeGpuNode('mi355x-0'));
    const r = render(el);
    await r.settle();
    expect(r.instances(CC.SectionBox)[0].props.title).toBe('AMD GPU');
    const rows = r.instances(CC.NameValueTable)[0].props.rows;
    const wl = rows.find((x) => x.name === 'GPU Workload Pods');
    expect(r.html()).toContain('train-a');
    expect(wl).toBeTruthy();
  });

  it('Node detail: nothing for a CPU node, nothing for non-Node resources', async () => {
    cluster();
    const r = render(nodeSection(makeNode('cpu-0')));
    await r.settle();
    expect(r.instances(CC.SectionBox)).toHaveLength(0);
    expect(nodeSection(makeGpuPod('x'))).toBeNull();
    expect(nodeSection(undefined)).toBeNull();
  });

  it('Node detail with pods forbidden says the pod list is unavailable, not Loading…', async () => {
    cluster({ pods: [null, 'pods is forbidden'] });
    const r = render(nodeSection(makeGpuNode('mi355x-0')));
    await r.settle();
    expect(r.text()).not.toContain('Loading…');
    expect(r.text()).toContain('Unavailable — the pod list could not be read');
  });

  it('cold Node detail (no plugin page yet) reads its own pods: a list + watch scoped to the node, no cluster-wide watch', async () => {
    cluster();
    const r = render(nodeSection(makeGpuNode('mi355x-1')));
    await r.settle();
    expect(lib.lists.calls.Node).toHaveLength(0);
    expect(lib.lists.calls.Pod.length).toBeGreaterThan(0);
    expect(lib.lists.calls.Pod.every((o) => o && o.fieldSelector === 'spec.nodeName=mi355x-1' && o.namespace === '')).toBe(true);
    expect(lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH)).toHaveLength(0);
    expect(lib.api.calls.filter((p) => p.indexOf('/api/v1/pods') === 0)).toHaveLength(0); // the list is the hook's
    expect(r.html()).toContain('train-b');
    expect(r.html()).not.toContain('train-a'); // mi355x-0's pod
    r.unmount();
  });

  it('warm Node detail (a plugin page fed the store) reads the store and sends no pod request', async () => {
    cluster();
    const page = render(h(route('/amd-gpu/nodes')));
    await page.settle();
    const before = lib.api.calls.length;
    const r = render(nodeSection(makeGpuNode('mi355x-0')));
    await r.settle();
    expect(lib.api.calls.slice(before).filter((p) => p.indexOf('/api/v1/pods') === 0)).toHaveLength(0);
    expect(r.html()).toContain('train-a');
    r.unmount();
    page.unmount();
  });

  it('Node detail opened next to a page adds no CRD request', async () => {
    cluster();
    const r = render(h('div', null, h(route('/amd-gpu/nodes')), nodeSection(makeGpuNode('mi355x-0'))));
    await r.settle();
    // GPU Nodes draws no DeviceConfig, and the section next to it reads the store.
    expect(lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH)).toHaveLength(0);
    expect(r.html()).toContain('train-a');
  });

  it.each(['/amd-gpu', '/amd-gpu/nodes', '/amd-gpu/pods', '/amd-gpu/metrics', '/amd-gpu/device-plugins'])(
    'Node detail after %s unmounted mounts no cluster-wide watch and no DeviceConfig request', async (path) => {
      cluster();
      const page = render(h(route(path)));
      await page.settle();
      page.unmount();
      lib.lists.calls.Node.length = 0;
      lib.lists.calls.Pod.length = 0;
      const before = lib.api.calls.length;
      const r = render(nodeSection(makeGpuNode('mi355x-1')));
      await r.settle();
      expect(lib.lists.calls.Node).toHaveLength(0);
      expect(lib.lists.calls.Pod.length).toBeGreaterThan(0);
      lib.lists.calls.Pod.forEach((o) => expect(o && o.fieldSelector).toBe('spec.nodeName=mi355x-1'));
      expect(lib.api.calls.slice(before).filter((p) => p === DEVICE_CONFIG_LIST_PATH)).toHaveLength(0);
      expect(r.html()).toContain('train-b');
      expect(r.html()).not.toContain('train-a');
      r.unmount();
    });

  it('Node detail next to a mounted page reads the store; when the page unmounts it moves to its node-scoped watch', async () => {
    cluster();
    const page = render(h(route('/amd-gpu/nodes')));
    await page.settle();
    lib.lists.calls.Node.length = 0;
    lib.lists.calls.Pod.length = 0;
    const r = render(nodeSection(makeGpuNode('mi355x-0')));
    await r.settle();
    expect(lib.lists.calls.Pod.filter((o) => o && o.fieldSelector)).toHaveLength(0); // the store, no list of its own
    page.unmount();
    await r.settle();
    lib.lists.calls.Node.length = 0;
    lib.lists.calls.Pod.length = 0;
    r.rerender(nodeSection(makeGpuNode('mi355x-0')));
    await r.settle();
    expect(lib.lists.calls.Node).toHaveLength(0);
    lib.lists.calls.Pod.forEach((o) => expect(o && o.fieldSelector).toBe('spec.nodeName=mi355x-0'));
    expect(lib.lists.calls.Pod.length).toBeGreaterThan(0);
    expect(r.html()).toContain('train-a');
    r.unmount();
  });

  it('Pod detail: GPU pod renders without a provider or a cluster request', async () => {
    const el = podSection(makeGpuPod('train-a', { gpus: 2 }));
    expect(el.type).toBe(plugin.PodDetailSection);
    const r = render(el);
    await r.settle();
    expect(r.instances(CC.SectionBox)[0].props.title).toBe('AMD GPU Resources');
    expect(lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH)).toHaveLength(0);
    expect(lib.lists.calls.Pod).toHaveLength(0);
  });

  it('Pod detail: nothing for a non-GPU pod or a Node', async () => {
    const r = render(podSection(makePlainPod('web-0')));
    await r.settle();
    expect(r.instances(CC.SectionBox)).toHaveLength(0);
    expect(podSection(makeGpuNode('mi355x-0'))).toBeNull();
  });
});

describe('Nodes table columns', () => {
  it('appends GPU Model / GPU Devices / GPU HBM to headlamp-nodes only', () => {
    const base = [{ label: 'Name' }];
    const out = reg.columns[0]({ id: 'headlamp-nodes', columns: base });
    expect(out.map((c) => c.label)).toEqual(['Name', 'GPU Model', 'GPU Devices', 'GPU HBM']);
    expect(reg.columns[0]({ id: 'headlamp-pods', columns: base })).toBe(base);
  });

  it('getters render through the IR cell renderer', () => {
    const cols = reg.columns[0]({ id: 'headlamp-nodes', columns: [] });
    const r = render(h('div', null, cols.map((c, i) => h('span', { key: i }, c.getter(makeGpuNode('mi355x-0'))))));
    expect(r.text()).toContain('MI355X');
    const cpu = render(h('div', null, cols.map((c, i) => h('span', { key: i }, c.getter(makeNode('cpu-0'))))));
    expect(cpu.text()).not.toContain('MI355X');
  });
});

describe('settings page', () => {
  function memoryStorage() {
    let v = null;
    const saved = [];
    return {
      saved,
      load: () => v || { prometheus: null, refreshIntervalSec: 0, requestTimeoutMs: 2000, seriesMinutes: 30 },
      save: (x) => {
        v = x;
        saved.push(x);
        return x;
      },
    };
  }

  it('changing auto-refresh saves validated settings and notifies Headlamp', () => {
    const storage = memoryStorage();
    const p = createPlugin({ React, lib, CommonComponents: CC, settingsStorage: storage });
    const onDataChange = vi.fn();
    const r = render(h(p.SettingsPage, { onDataChange }));
    expect(r.instances(CC.SectionBox)[0].props.title).toBe('AMD GPU plugin settings');
    r.change(r.getByLabelText('Auto-refresh interval'), '30');
    expect(storage.saved[0].refreshIntervalSec).toBe(30);
    expect(onDataChange).toHaveBeenCalledTimes(1);
    expect(r.getByLabelText('Auto-refresh interval').props.value).toBe(30);
  });

  it('an invalid timeout is clamped; an incomplete Prometheus service is dropped', () => {
    const storage = memoryStorage();
    const p = createPlugin({ React, lib, CommonComponents: CC, settingsStorage: storage });
    const r = render(h(p.SettingsPage));
    r.blur(r.getByLabelText('Request timeout'), '5');
    expect(storage.saved[0].requestTimeoutMs).toBe(250);
    r.change(r.getByLabelText('Prometheus namespace'), 'monitoring');
    r.blur(r.getByLabelText('Prometheus namespace'));
    expect(storage.saved[1].prometheus).toBeNull();
    r.change(r.getByLabelText('Prometheus service'), 'prom');
    r.change(r.getByLabelText('Prometheus port'), '9090');
    r.blur(r.getByLabelText('Prometheus port'));
    expect(storage.saved[2].prometheus).toEqual({ namespace: 'monitoring', service: 'prom', port: '9090' });
  });
});

describe('page-scoped telemetry', () => {
  function withPrometheus() {
    cluster();
    const fake = prom({ data: exporterData(['mi355x-0', 'mi355x-1']) });
    const crd = lib.api.handler;
    lib.api.handler = (p) => (p.indexOf('/proxy/api/v1/') >= 0 ? fake(p) : crd(p));
    return fake;
  }
  const liveQueries = (fake) => fake.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => /\/query\?query=(?!1$)/.test(p));

  it('Metrics page: per-GPU gauges, no xGMI links', async () => {
    const fake = withPrometheus();
    const r = render(h(route('/amd-gpu/metrics')));
    await r.settle();
    const qs = liveQueries(fake);
    expect(qs.length).toBeGreaterThan(0);
    qs.forEach((q) => {
      expect(q).toContain(SERIES.exporter.gfx);
      expect(q).not.toContain(SERIES.exporter.xgmiRe);
    });
    expect(r.html()).toContain('GPU Power Summary');
    r.unmount();
  });

  it('GPU Nodes page: owners and xGMI links, none of the Metrics gauges', async () => {
    const fake = withPrometheus();
    const r = render(h(route('/amd-gpu/nodes')));
    await r.settle();
    const qs = liveQueries(fake);
    expect(qs.length).toBeGreaterThan(0);
    qs.forEach((q) => {
      expect(q).toContain(SERIES.exporter.xgmiRe);
      expect(q).not.toContain(SERIES.exporter.gfx);
    });
    r.unmount();
  });
});

describe('React StrictMode (effects mounted, cleaned up and mounted again)', () => {
  function withPrometheus() {
    cluster();
    const fake = prom({ data: exporterData(['mi355x-0', 'mi355x-1']) });
    const crd = lib.api.handler;
    lib.api.handler = (p) => (p.indexOf('/proxy/api/v1/') >= 0 ? fake(p) : crd(p));
    return fake;
  }
  const liveQueries = (fake) => fake.mock.calls.filter((c) => /\/query\?query=(?!1$)/.test(decodeURIComponent(c[0]))).length;

  it('Overview mounts with one CRD request', async () => {
    cluster();
    const r = render(h(route('/amd-gpu')), { strict: true });
    await r.settle();
    expect(lib.api.calls.filter((p) => p === DEVICE_CONFIG_LIST_PATH)).toHaveLength(1);
    expect(r.instances(CC.SectionHeader)[0].props.title).toBe('AMD GPU — Overview');
    r.unmount();
  });

  it('Metrics page mounts with one live query and renders its data', async () => {
    const fake = withPrometheus();
    const r = render(h(route('/amd-gpu/metrics')), { strict: true });
    await r.settle();
    expect(liveQueries(fake)).toBe(1);
    // at most one range query (none when the shared source's window is current)
    expect(fake.mock.calls.filter((c) => c[0].indexOf('/query_range') >= 0).length).toBeLessThanOrEqual(1);
    expect(r.html()).toContain('GPU Power Summary');
    r.unmount();
  });

  it('Node detail section mounts with one node-scoped query', async () => {
    const fake = withPrometheus();
    const Detail = reg.details[0];
    const r = render(h(() => Detail({ resource: { kind: 'Node', jsonData: makeGpuNode('mi355x-0') } })), { strict: true });
    await r.settle();
    const scoped = fake.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('hostname="mi355x-0"') >= 0);
    // one node-scoped instant query (live telemetry) and one node-scoped range query (power history)
    expect(scoped.filter((p) => p.indexOf('/query?') >= 0)).toHaveLength(1);
    expect(scoped.filter((p) => p.indexOf('/query_range?') >= 0)).toHaveLength(1);
    r.unmount();
  });
});

// Pod detail power history and Metrics without Prometheus RBAC: tests/js/shared/telemetry.shared.test.js (both React tiers).

describe('pager state survives leaving and reopening a page (this tab)', () => {
  function memStorage() {
    const m = {};
    return { getItem: (k) => (k in m ? m[k] : null), setItem: (k, v) => { m[k] = String(v); }, m };
  }
  // Leaving and reopening GPU Nodes through the controls: tests/js/shared/viewstate.shared.test.js (both React tiers).
  it('unreadable or hostile stored state falls back to the first page', async () => {
    const { loadViewState } = await import('../../src/api/settings.js');
    const st = memStorage();
    st.setItem('headlamp-amd-gpu-plugin.view.c|nodes', '{"page":-3,"filter":7,"sort":{}}');
    expect(loadViewState('c|nodes', st)).toEqual({ page: 0, filter: '', sort: 'name' });
    st.setItem('headlamp-amd-gpu-plugin.view.c|pods', 'not json');
    expect(loadViewState('c|pods', st)).toBe(null);
    expect(loadViewState('c|none', st)).toBe(null);
    expect(loadViewState('c|nodes', null)).toBe(null);
  });
});
