/**
 * The plugin, assembled: every page, detail section, table column and the
 * settings page, built from the pure view-models (./view/pages/*.js), the IR
 * renderer (./view/react.js) and the provider core (./api/providerCore.js)
 * against an INJECTED React + Headlamp library. `registerPlugin` performs the
 * registration the reference does at module load (src/index.tsx:35-182,
 * SURVEY.md C1): sidebar root + 5 children, 5 exact routes, the Node and Pod
 * detail sections and the `headlamp-nodes` column processor, plus the plugin
 * settings page when the host offers `registerPluginSettings`.
 *
 * src/index.tsx is a shim that calls these two functions with the real React
 * and '@kinvolk/headlamp-plugin/lib'; the Node-12 harness calls them with
 * its stand-ins (tests/js/stubs/), so what the tests execute is the shipped
 * code, not a copy.
 *
 * Unlike the reference, routes do not each mount a cold provider: the
 * provider is a view onto one shared per-cluster store, so switching pages
 * or opening a Node detail view renders cached data at once and revalidates
 * in the background (reference quirk Q7).
 */

import { createProviderCore, READ_ONLY_NEEDS } from './api/providerCore.js';
import { isAmdGpuNode } from './api/amdNodes.js';
import { isGpuRequestingPod } from './api/amdPods.js';
import { get, unwrapKubeObject } from './api/k8sCore.js';
import { nodeColumns, nodeDetailView, podDetailView } from './view/pages/details.js';
import { devicePluginsView } from './view/pages/devicePlugins.js';
import { metricsView } from './view/pages/metricsPage.js';
import { nodesView, telemetryScope } from './view/pages/nodes.js';
import { overviewOwnersScope, overviewView } from './view/pages/overview.js';
import { nodeSortOf, RANKED_NODE_SORTS } from './view/pages/paging.js';
import { ownersScope, podsView } from './view/pages/pods.js';
import { createRenderer } from './view/react.js';
import { createSettingsPage } from './view/settingsPage.js';
import { loadViewState, saveViewState } from './api/settings.js';
import { processColumns, ROUTES, SIDEBAR } from './routes.js';

/** Plugin name used for `registerPluginSettings`. */
export const PLUGIN_NAME = 'amd-gpu';

/**
 * What each page draws, hence what its route mounts (providerCore.js
 * AmdGpuDataProvider): Metrics needs the node list only (names of the page,
 * nodes reporting); GPU Nodes and GPU Pods need both lists but not the
 * DeviceConfigs; Device Plugins the DeviceConfigs and the operator pods'
 * own lists + watches (providerCore.js OperatorPodFeed: the operator
 * namespace and the plugin labels), not the all-namespaces pod list;
 * Overview everything.
 * The reference mounts all of it on every route (src/index.tsx:87-145).
 */
export const PAGE_NEEDS = Object.freeze({
  overview: Object.freeze({ nodes: true, pods: true, crd: true }),
  'device-plugins': Object.freeze({ nodes: false, pods: false, crd: true, operatorPods: true }),
  nodes: Object.freeze({ nodes: true, pods: true, crd: false }),
  pods: Object.freeze({ nodes: true, pods: true, crd: false }),
  metrics: Object.freeze({ nodes: true, pods: false, crd: false }),
});

/**
 * @param {{React: any, lib: any, CommonComponents: Record<string, Function>,
 *          deps?: Parameters<typeof createProviderCore>[2], settingsStorage?: {load: Function, save: Function},
 *          viewStorage?: {getItem: Function, setItem: Function} | null}} env
 */
export function createPlugin(env) {
  if (!env || !env.React || !env.lib || !env.CommonComponents) throw new Error('createPlugin: React, lib and CommonComponents are required');
  const React = env.React;
  const h = React.createElement;
  const core = createProviderCore(React, env.lib, env.deps);
  const view = createRenderer(React, env.CommonComponents);
  const Page = view.Page;
  const Section = view.Section;
  const Value = view.Value;

  // -------------------------------------------------------------------------
  // Pages (reference src/components/*Page.tsx, SURVEY.md C5–C9)
  // -------------------------------------------------------------------------

  /**
   * Cluster-level MI355X dashboard (reference OverviewPage.tsx, C5). On a
   * cluster of more than one page of GPU nodes, the exporter's owner answer
   * stands in for the pod-derived sections while the pod list loads
   * (overviewOwnersScope); no Prometheus request otherwise.
   */
  function OverviewPage() {
    const ctx = core.useAmdGpuContext();
    const o = overviewOwnersScope(ctx);
    const m = core.useGpuOwners(o.enabled, o.pods, o.small, undefined, o.preview);
    return h(Page, { vm: overviewView(ctx, { metrics: o.enabled ? m.metrics : null }), onRefresh: ctx.refresh });
  }

  /** AMD GPU Operator DeviceConfigs and operand pods (reference DevicePluginsPage.tsx, C6). */
  function DevicePluginsPage() {
    const ctx = core.useAmdGpuContext();
    const pager = usePager('device-plugins');
    return h(Page, {
      vm: devicePluginsView(ctx, { pager: pager.state }), onRefresh: ctx.refresh,
      onPage: pager.onPage, onFilter: pager.onFilter, onSort: pager.onSort,
    });
  }

  /**
   * Pager state of a paged page: {page, filter, sort}. A new filter or order
   * starts again at the first page. It is kept per cluster and page for this
   * browser tab (settings.js loadViewState), so leaving the page and coming
   * back — Headlamp unmounts it — returns to the same place.
   */
  function usePager(name) {
    const key = core.clusterKey() + '|' + name;
    const st = React.useState(function () {
      return loadViewState(key, env.viewStorage) || { page: 0, filter: '', sort: 'name' };
    });
    const pg = st[0];
    const setPg = st[1];
    React.useEffect(function () {
      saveViewState(key, pg, env.viewStorage);
    }, [key, pg]);
    return {
      state: pg,
      onPage: function (p) { setPg(function (s) { return { page: p, filter: s.filter, sort: s.sort }; }); },
      onFilter: function (f) { setPg(function (s) { return { page: 0, filter: f, sort: s.sort }; }); },
      onSort: function (o) { setPg(function (s) { return { page: 0, filter: s.filter, sort: o }; }); },
    };
  }

  /**
   * A power-ranked answer past the last page (the ranked count shrank while
   * the user was on a later page): move to the last page, which asks again.
   */
  function useRankedPageClamp(metrics, pager) {
    const r = metrics && metrics.rank;
    const last = r && r.per > 0 ? Math.max(0, Math.ceil(r.count / r.per) - 1) : 0;
    const beyond = !!r && r.page > last && r.page === pager.state.page;
    React.useEffect(function () {
      if (beyond) pager.onPage(last);
    }, [beyond, last]);
  }

  /**
   * MI355X nodes: summary table, per-node cards with the per-GPU allocation
   * strip and the xGMI matrix (reference NodesPage.tsx, C7), one page of
   * nodes at a time. Exporter telemetry of the nodes on the page (no time
   * series: this page draws none) upgrades the strip to exact pod→GPU
   * ownership and overlays measured xGMI throughput.
   */
  function NodesPage() {
    const ctx = core.useAmdGpuContext();
    const pager = usePager('nodes');
    const t = telemetryScope(ctx, pager.state, true);
    const m = core.useGpuMetrics(t.enabled, false, 'topology', t.scope, t.small, t.rank);
    useRankedPageClamp(m.metrics, pager);
    // The node and pod lists are live watches; what Refresh can renew here is
    // the telemetry (the DeviceConfigs are not on this page).
    return h(Page, {
      vm: nodesView(ctx, { metrics: m.metrics, pager: pager.state, fetching: m.fetching }), onRefresh: m.refresh,
      onPage: pager.onPage, onFilter: pager.onFilter, onSort: pager.onSort,
    });
  }

  /**
   * Pods requesting amd.com/* (reference PodsPage.tsx, C8), one page of the
   * table at a time. Exporter pod labels add the physical GPUs each pod on
   * the page holds — fetched as attribution only, one series per allocated
   * GPU of those pods.
   */
  function PodsPage() {
    const ctx = core.useAmdGpuContext();
    const pager = usePager('pods');
    const o = ownersScope(ctx, pager.state);
    const m = core.useGpuOwners(o.enabled, o.pods, o.small, o.rank, o.preview);
    useRankedPageClamp(m.metrics, pager);
    // As on GPU Nodes: the lists are watches; Refresh renews the attribution.
    return h(Page, {
      vm: podsView(ctx, { metrics: m.metrics, pager: pager.state, fetching: m.fetching }), onRefresh: m.refresh,
      onPage: pager.onPage, onFilter: pager.onFilter, onSort: pager.onSort,
    });
  }

  /**
   * Power, HBM, activity, temperature, RAS and xGMI telemetry from Prometheus
   * (reference MetricsPage.tsx, C9): cluster totals as server-side
   * aggregates, per-node cards and series for one page of GPU nodes.
   */
  function MetricsPage() {
    const ctx = core.useAmdGpuContext();
    const pager = usePager('metrics');
    const t = telemetryScope(ctx, pager.state, true);
    const m = core.useGpuMetrics(t.enabled, true, 'gauges', t.scope, t.small, t.rank);
    useRankedPageClamp(m.metrics, pager);
    // The route feeds the node list only (PAGE_NEEDS); the allocation orders
    // rank nodes by the GPUs pods hold, so they mount the pod list too.
    const sort = nodeSortOf(pager.state, RANKED_NODE_SORTS);
    const needPods = sort === 'in-use' || sort === 'free';
    return h(React.Fragment, null, needPods ? h(core.PodListHere, null) : null, h(Page, {
      vm: metricsView(ctx, m, { pager: pager.state }), onRefresh: m.refresh,
      onPage: pager.onPage, onFilter: pager.onFilter, onSort: pager.onSort,
    }));
  }

  // -------------------------------------------------------------------------
  // Native-view integrations (reference C10–C12)
  // -------------------------------------------------------------------------

  /**
   * Section on Headlamp's Node detail page (reference NodeDetailSection.tsx,
   * C10). Nothing for non-AMD nodes. Reads the shared store, so it costs no
   * fetch when a plugin page already loaded the cluster; the node's own
   * telemetry comes from one `hostname`-scoped query.
   */
  function NodeDetailSection(props) {
    const ctx = core.useAmdGpuContext();
    const raw = unwrapKubeObject(props.resource);
    const gpuNode = isAmdGpuNode(raw);
    const m = core.useNodeGpuMetrics(gpuNode ? raw.metadata.name : null, gpuNode);
    const ps = core.useNodeGpuSeries(gpuNode ? raw.metadata.name : null, gpuNode);
    const section = nodeDetailView(props.resource, ctx, { metrics: m.metrics, series: ps.series });
    return section ? h(Section, { s: section }) : null;
  }

  /**
   * The Node detail section when no mounted page feeds the store — the usual
   * case: Headlamp reaches a Node's page from its own Nodes list, after any
   * plugin page unmounted. The node's own pods by a list + watch scoped to
   * the node (live, like the reference's section; seeded by the store's last
   * pod list for the first paint), with its telemetry and power history in
   * the same wave — no cluster-wide watch and no DeviceConfig request.
   * Mounted for AMD GPU nodes only.
   */
  function NodeDetailCold(props) {
    const name = unwrapKubeObject(props.resource).metadata.name;
    const np = core.useNodePods(name);
    const m = core.useNodeGpuMetrics(name, true);
    const ps = core.useNodeGpuSeries(name, true);
    const section = nodeDetailView(props.resource, np[0], { metrics: m.metrics, series: ps.series });
    return h(React.Fragment, null, np[1], section ? h(Section, { s: section }) : null);
  }

  /**
   * Nothing for a node without AMD GPUs. While a plugin page that draws pods
   * is mounted next to it (its pod feed keeps the store current), the section
   * reads the store under a provider that mounts nothing (READ_ONLY_NEEDS);
   * otherwise NodeDetailCold, O(one node). The reference mounts a full
   * provider — both cluster-wide lists and the CRD + 3 serial requests — on
   * every Node detail page (src/index.tsx:152-160).
   */
  function NodeDetailHost(props) {
    const live = core.usePodsLive();
    if (!isAmdGpuNode(unwrapKubeObject(props.resource))) return null;
    if (live) return h(core.AmdGpuDataProvider, { needs: READ_ONLY_NEEDS }, h(NodeDetailSection, props));
    return h(NodeDetailCold, props);
  }

  /**
   * Section on Headlamp's Pod detail page (reference PodDetailSection.tsx,
   * C11). Needs no cluster data, so it mounts no provider; for a scheduled GPU
   * pod it reads the telemetry of the pod's node only (live power / GFX / HBM
   * of the GPUs the pod holds).
   */
  function PodDetailSection(props) {
    const raw = unwrapKubeObject(props.resource);
    const gpuPod = isGpuRequestingPod(raw);
    const nodeName = gpuPod ? get(raw, ['spec', 'nodeName'], null) : null;
    const m = core.useNodeGpuMetrics(nodeName, gpuPod);
    // Power history of the pod's GPUs, fetched next to (not after) the node's telemetry.
    const md = gpuPod && raw.metadata ? raw.metadata : null;
    const ps = core.usePodGpuSeries(md ? md.namespace || '' : null, md ? md.name : null, !!nodeName);
    const section = podDetailView(props.resource, { metrics: m.metrics, series: ps.series });
    return section ? h(Section, { s: section }) : null;
  }

  /** GPU Model / GPU Devices / GPU HBM columns for the native Nodes table (reference NodeColumns.tsx, C12). */
  function buildNodeGpuColumns() {
    return nodeColumns().map(function (c) {
      return { label: c.label, getter: function (resource) { return h(Value, { v: c.getter(resource) }); } };
    });
  }

  const pages = {
    overview: OverviewPage,
    'device-plugins': DevicePluginsPage,
    nodes: NodesPage,
    pods: PodsPage,
    metrics: MetricsPage,
  };

  /** Route component: the page under the (shared-store) provider, mounting what the page draws. */
  function routeComponent(page) {
    const P = pages[page];
    if (!P) throw new Error('createPlugin: unknown page ' + page);
    const needs = PAGE_NEEDS[page];
    function Route() {
      return h(core.AmdGpuDataProvider, { needs: needs }, h(P, null));
    }
    Route.displayName = 'AmdGpuRoute(' + page + ')';
    return Route;
  }

  /**
   * Detail-view section callback for Nodes (reference src/index.tsx:152-160,
   * which mounts a full provider — both cluster-wide lists and the CRD /
   * operator-pod requests — on every Node detail page).
   */
  function nodeDetailSectionFor(args) {
    const resource = args && args.resource;
    if (!resource || resource.kind !== 'Node') return null;
    return h(NodeDetailHost, { resource: resource });
  }

  /** Detail-view section callback for Pods: no provider (reference src/index.tsx:167-170). */
  function podDetailSectionFor(args) {
    const resource = args && args.resource;
    if (!resource || resource.kind !== 'Pod') return null;
    return h(PodDetailSection, { resource: resource });
  }

  return {
    core: core,
    view: view,
    AmdGpuDataProvider: core.AmdGpuDataProvider,
    useAmdGpuContext: core.useAmdGpuContext,
    OverviewPage: OverviewPage,
    DevicePluginsPage: DevicePluginsPage,
    NodesPage: NodesPage,
    PodsPage: PodsPage,
    MetricsPage: MetricsPage,
    NodeDetailSection: NodeDetailSection,
    NodeDetailCold: NodeDetailCold,
    PodDetailSection: PodDetailSection,
    SettingsPage: createSettingsPage(React, env.CommonComponents, env.settingsStorage),
    buildNodeGpuColumns: buildNodeGpuColumns,
    pages: pages,
    routeComponent: routeComponent,
    nodeDetailSectionFor: nodeDetailSectionFor,
    podDetailSectionFor: podDetailSectionFor,
  };
}

/**
 * Register every extension point with Headlamp (reference src/index.tsx:35-182).
 * @param {any} lib  '@kinvolk/headlamp-plugin/lib'
 * @param {ReturnType<typeof createPlugin>} plugin
 * @returns {{sidebar: number, routes: number, detailSections: number, columnProcessors: number, settings: boolean}}
 */
export function registerPlugin(lib, plugin) {
  for (let i = 0; i < SIDEBAR.length; i++) lib.registerSidebarEntry(SIDEBAR[i]);
  for (let i = 0; i < ROUTES.length; i++) {
    const r = ROUTES[i];
    lib.registerRoute({ path: r.path, sidebar: r.sidebar, name: r.name, exact: true, component: plugin.routeComponent(r.page) });
  }
  lib.registerDetailsViewSection(plugin.nodeDetailSectionFor);
  lib.registerDetailsViewSection(plugin.podDetailSectionFor);
  lib.registerResourceTableColumnsProcessor(function (args) { return processColumns(args, plugin.buildNodeGpuColumns); });
  // Headlamp >= 0.22 offers plugin settings; older hosts run with the
  // defaults of src/api/settings.js.
  const settings = typeof lib.registerPluginSettings === 'function';
  if (settings) lib.registerPluginSettings(PLUGIN_NAME, plugin.SettingsPage, false);
  return { sidebar: SIDEBAR.length, routes: ROUTES.length, detailSections: 2, columnProcessors: 1, settings: settings };
}
