/**
 * The two request schedules the benchmark runs over the same HTTP client:
 * `amdSchedule` drives the SHIPPED data layer (src/api/clusterStore.js,
 * src/api/metrics.js) as src/plugin.js wires it per page; `referenceSchedule`
 * is the reference's provider + pages request pattern
 * (./referenceSchedule.js). Both expose the same surface to the driver:
 * coldOpen, refresh, refreshPage, coldOpenPage, switchRoute, ctx, mstate,
 * pageMstate, pageMetrics.
 */
import { createClusterStore } from '../src/api/clusterStore.js';
import { createMetricsSource } from '../src/api/metrics.js';
import { telemetryScope } from '../src/view/pages/nodes.js';
import { ownersScope } from '../src/view/pages/pods.js';
import { overviewOwnersScope } from '../src/view/pages/overview.js';
import { renderPage } from '../src/view/html.js';
import { PAGE_NEEDS } from '../src/plugin.js';
import { createReferenceSchedule } from './referenceSchedule.js';
import { hiResClock } from './common.js';
import { PAGER, hasContent, pageVm } from './pageRender.js';

export function amdSchedule(request, clock, timeoutMs) {
  // Request spans from the data layer's tracing hook (clusterStore/metrics onTrace).
  const spans = [];
  function onTrace(span) {
    spans.push(span);
  }
  const clk = clock || hiResClock;
  const store = createClusterStore({ request: request, onTrace: onTrace, clock: clk, timeoutMs: timeoutMs });
  // The feeds a route mounts (providerCore.js PodListFeed / OperatorPodFeed,
  // plugin.js PAGE_NEEDS): the all-namespaces pod list is attached while a
  // page that draws pods is shown; Device Plugins mounts the operator pods'
  // own lists instead. A page's refresh runs with its route's feeds, so it
  // asks what the shipped route asks (Device Plugins: the DeviceConfigs alone,
  // its operator pods being watched).
  let detachFeed = store.attachPodFeed();
  function needsOf(page) {
    return PAGE_NEEDS[page === 'devicePlugins' ? 'device-plugins' : page];
  }
  /** Switch the attached feeds to `page`'s route; returns a function restoring the pod list feed. */
  function mountFeeds(page) {
    const needs = needsOf(page);
    if (needs.pods || !detachFeed) return function () {};
    detachFeed();
    detachFeed = null;
    const detachOps = needs.operatorPods ? store.attachOperatorFeed() : null;
    return function () {
      if (detachOps) detachOps();
      detachFeed = store.attachPodFeed();
    };
  }
  function onRoute(page, run) {
    const restore = mountFeeds(page);
    return run().then(function (v) {
      restore();
      return v;
    });
  }
  const metrics = createMetricsSource({ request: request, onTrace: onTrace, clock: clk, timeoutMs: timeoutMs });
  const mstate = { metrics: null, fetchError: null, fetching: false, series: null };
  // Per-page metrics state, as each page's own hook holds it (plugin.js):
  // GPU Nodes → owners + xGMI links of the nodes on its first page
  // ('topology', scoped), GPU Pods → pod→GPU attribution only, Metrics →
  // cluster totals + per-GPU gauges + series of the nodes on its first page
  // ('gauges', scoped). Cold open / route switch / the all-pages composite
  // fetch every live series in one query ('all').
  const pageMetrics = { nodes: null, pods: null, overview: null };
  const metricsPage = { metrics: null, fetchError: null, fetching: false, series: null };
  function fetchMetrics(view) {
    return Promise.all([metrics.fetchGpuMetrics(view), metrics.fetchSeries(1800, 30)]).then(function (r) {
      mstate.metrics = r[0];
      mstate.series = r[1];
      mstate.fetchError = r[0] ? null : 'Could not reach Prometheus';
    });
  }
  /**
   * What the page's hook asks for now (pages.js telemetryScope): its query
   * key (null = disabled) and fetch options. While the node list loads, and
   * while every GPU node fits on one page, that is the size-guarded
   * small-cluster query under one key.
   */
  function scoped(summary) {
    const t = telemetryScope(store.getSnapshot(), PAGER);
    const key = !t.enabled ? null : t.scope === undefined ? 'all' : t.small ? 'small' : 'scope:' + t.scope.join(',');
    return t.scope === undefined ? { key: key, opts: undefined, scope: undefined, small: false }
      : { key: key, opts: { scope: t.scope, summary: summary, small: !!t.small }, scope: t.scope, small: !!t.small };
  }
  function ownersKey() {
    const o = ownersScope(store.getSnapshot(), PAGER);
    return !o.enabled ? null : o.pods === undefined ? 'all' : o.small ? 'small' : 'pods:' + o.pods.join(',');
  }
  /**
   * A page's metrics hook from mount to the lists: it fetches under the key
   * of its first render and again only if the lists change that key (a
   * larger cluster's first page), as useMetricsFetch does.
   */
  function pageOpen(page, onData) {
    const keyOf = page === 'pods' ? ownersKey : function () { return scoped(false).key; };
    const fetch0 = page === 'pods' ? fetchPodsPage : page === 'nodes' ? fetchNodesPage : fetchMetricsPage;
    const fetch = onData ? function () { return fetch0(onData).then(onData); } : fetch0;
    const k0 = keyOf();
    const first = k0 === null ? Promise.resolve() : fetch();
    const second = listed(page === 'pods' ? 'podsState' : 'nodesState').then(function () {
      const k1 = keyOf();
      return k1 !== null && k1 !== k0 ? fetch() : first;
    });
    return Promise.all([first, second]);
  }
  function listed(which) {
    return new Promise(function (resolve) {
      function done() {
        const st = store.getSnapshot()[which];
        return st === 'ready' || st === 'error';
      }
      if (done()) return resolve();
      const off = store.subscribe(function () {
        if (done()) {
          off();
          resolve();
        }
      });
    });
  }
  function pageMetricsOf(page) {
    if (page === 'overview') return pageMetrics.overview;
    return page in pageMetrics && pageMetrics[page] ? pageMetrics[page] : mstate.metrics;
  }
  /**
   * Overview's owner hook (plugin.js OverviewPage): once the node list says the
   * cluster is larger than one page and while its pod list is still loading
   * (overview.js overviewOwnersScope), the exporter's owners with a preview.
   */
  function overviewOpen(onData) {
    pageMetrics.overview = null;
    return listed('nodesState').then(function () {
      const o = overviewOwnersScope(store.getSnapshot());
      if (!o.enabled) return undefined;
      return metrics.fetchGpuOwners({ pods: o.pods, small: o.small, preview: o.preview }).then(function (m) {
        pageMetrics.overview = m;
        if (onData) onData();
      });
    });
  }
  function fetchPodsPage() {
    const o = ownersScope(store.getSnapshot(), PAGER);
    const opts = o.pods === undefined ? undefined : { pods: o.pods, small: !!o.small, preview: o.preview };
    return metrics.fetchGpuOwners(opts).then(function (m) { pageMetrics.pods = m; });
  }
  function fetchNodesPage() {
    return metrics.fetchGpuMetrics('topology', scoped(false).opts).then(function (m) { pageMetrics.nodes = m; });
  }
  /** The Metrics page's hook (providerCore.js useGpuMetrics): telemetry shown as it comes (`early`), then the series. */
  function fetchMetricsPage(early) {
    const sc = scoped(true);
    const mp = metrics.fetchGpuMetrics('gauges', sc.opts);
    mp.then(function (m) {
      if (!m || !early) return;
      metricsPage.metrics = m;
      metricsPage.fetchError = null;
      early();
    });
    return Promise.all([mp, metrics.fetchSeries(1800, 30, sc.scope, sc.small)]).then(function (r) {
      metricsPage.metrics = r[0];
      metricsPage.series = r[1];
      metricsPage.fetchError = r[0] ? null : 'Could not reach Prometheus';
    });
  }
  return {
    /**
     * Every page's data at once, as each page fetches it: the lists, the
     * DeviceConfig and the pages' size-guarded telemetry in one wave; on a
     * cluster larger than one page, GPU Nodes / Metrics / GPU Pods telemetry
     * of their first pages once the node (pod) list is in.
     */
    coldOpen: function () {
      return Promise.all([store.loadLists(), store.refresh(), pageOpen('nodes'), pageOpen('metrics'), pageOpen('pods')]);
    },
    /** Composite refresh: every page's Refresh in one wave (5 requests, within the 6 browser sockets). */
    refresh: function () {
      return Promise.all([store.refresh(), fetchNodesPage(), fetchPodsPage(), fetchMetricsPage()]);
    },
    /** Every live series of every GPU (the terminal client's and the screenshots' snapshot). */
    fetchAll: function () {
      return fetchMetrics();
    },
    /** One page's Refresh button, as src/plugin.js wires it. */
    refreshPage: function (page) {
      // GPU Nodes / GPU Pods renew their telemetry only (plugin.js: the lists are watches).
      if (page === 'nodes') return fetchNodesPage();
      if (page === 'pods') return fetchPodsPage();
      if (page === 'metrics') return fetchMetricsPage();
      return onRoute(page, function () { return store.refresh(); });
    },
    /**
     * One page opened on an empty cache, as src/plugin.js mounts it: the
     * provider's lists + DeviceConfig request and the page's size-guarded
     * telemetry in one wave — all of it on a cluster of one page; a larger
     * cluster's GPU Nodes / Metrics (GPU Pods) ask for their first page of
     * nodes (pods) once the node (pod) list is there (a second wave).
     *
     * `marks` (all optional) are called as the page fills in:
     *   first     the page's view-model first shows content (pages.js decides:
     *             its full-page loader gone; on Metrics, telemetry or a state
     *             saying there is none) — built and rendered on every store
     *             commit and telemetry answer, as the mounted page re-renders;
     *   content   the lists + DeviceConfig committed (the reference's content);
     *   complete  everything THIS page draws is in (Metrics: the node list and
     *             its telemetry, not the pod list; Device Plugins: the
     *             DeviceConfigs and the pod list; the others: both lists, the
     *             DeviceConfigs where shown, their telemetry).
     * Resolves when every request has finished (the next open starts drained).
     */
    coldOpenPage: function (page, marks) {
      const mk = marks || {};
      // What the page's route mounts (src/plugin.js PAGE_NEEDS).
      const needs = needsOf(page);
      mountFeeds(page); // a fresh schedule per open: nothing to restore
      let shown = !mk.first;
      function check() {
        if (shown) return;
        const vm = pageVm(page, store.getSnapshot(), page === 'metrics' ? metricsPage : mstate, pageMetricsOf(page));
        if (!hasContent(page, vm)) return;
        shown = true;
        renderPage(vm);
        mk.first();
      }
      const off = store.subscribe(check);
      // The list requests of the watches the route mounts.
      const lists = Promise.all([store.loadLists({ nodes: needs.nodes, pods: needs.pods }),
        needs.operatorPods && !needs.pods ? store.loadOperatorPods() : null]);
      const crd = needs.crd ? store.refresh() : Promise.resolve();
      // The page's metrics hook runs from the first render (pages.js
      // telemetryScope) and once more if the node list changes its key.
      const telemetry = page === 'nodes' || page === 'metrics' || page === 'pods' ? pageOpen(page, check) : Promise.resolve();
      // Overview's stand-in for its pod sections while a large cluster's pod
      // list loads: shown as it comes, not part of what the page draws when complete.
      const interim = page === 'overview' ? overviewOpen(check) : Promise.resolve();
      const content = Promise.all([lists, crd]).then(function () { if (mk.content) mk.content(); });
      // Everything the page draws: what its route mounts, and its telemetry.
      const complete = Promise.all([lists, crd, telemetry]).then(function () { if (mk.complete) mk.complete(); });
      return Promise.all([lists, crd, telemetry, interim, content, complete]).then(function () { off(); });
    },
    pageMetrics: pageMetricsOf,
    /** The Metrics page's own state (its hook), for rendering that page. */
    pageMstate: function () { return metricsPage; },
    /** Route switch: render from the shared store now, revalidate in the background. */
    switchRoute: function () {
      const bg = Promise.all([store.refresh(), fetchNodesPage(), fetchPodsPage(), fetchMetricsPage()]);
      return { rendered: Promise.resolve(), background: bg };
    },
    ctx: function () { return store.getSnapshot(); },
    mstate: function () { return mstate; },
    source: metrics,
    spans: spans,
  };
}

export function referenceSchedule(request) {
  const r = createReferenceSchedule(request);
  return {
    coldOpen: r.coldOpen,
    refresh: r.refresh,
    switchRoute: function () {
      const p = r.coldOpen();
      return { rendered: p, background: p };
    },
    refreshPage: r.refreshPage,
    coldOpenPage: r.coldOpenPage,
    pageMetrics: function () { return r.metrics(); },
    pageMstate: function () { return { metrics: r.metrics(), fetchError: r.metrics() ? null : 'unreachable', fetching: false }; },
    ctx: r.snapshot,
    mstate: function () { return { metrics: r.metrics(), fetchError: r.metrics() ? null : 'unreachable', fetching: false }; },
  };
}
