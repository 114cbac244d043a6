/**
 * Provider core — the React binding of the shared ClusterStore and of the
 * Prometheus client, written against INJECTED React hooks and an injected
 * Headlamp library, so the exact code Headlamp runs also runs under the
 * Node-12 harness's React stand-in (tests/js/stubs/react.js).
 *
 * Reference analog: src/api/IntelGpuDataContext.tsx (SURVEY.md C3) and the
 * MetricsPage state/effect (src/components/MetricsPage.tsx:191-231). Same
 * public contract — `useAmdGpuContext()` returns {deviceConfigs,
 * pluginInstalled, gpuNodes, gpuPods, pluginPods, crdAvailable, loading,
 * error, refresh} and throws outside a provider (reference :60-66) — but
 * the provider is a thin view onto one store per cluster
 * (src/api/clusterStore.js):
 *
 *   * Headlamp's reactive `useList()` hooks feed nodes and pods into the
 *     store (two-track design, reference ADR 002 / :98-99); an errored list
 *     is fed as an error, which the store treats as settled;
 *   * the imperative track (DeviceConfig CRD, operator pods only when the
 *     pod list is unavailable) runs in parallel inside the store, with
 *     timeouts and a sequence guard (reference: serial, :122-165);
 *   * a mounting provider calls `revalidate(STALE_MS)`: if another view
 *     fetched moments ago (route switch, Node detail section next to a page)
 *     nothing is re-fetched and the cached snapshot renders at once
 *     (reference quirk Q7: every route mounted a cold provider).
 */

import { createClusterStore, getSharedStore } from './clusterStore.js';
import { dedupePods, filterAmdGpuPluginPods } from './amdPods.js';
import { OPERATOR_POD_LISTS, unwrapAll } from './k8sCore.js';
import { createMetricsSource } from './metrics.js';
import { countOutside } from './selectors.js';
import { createNodePodHooks } from './nodePodHooks.js';
import { clusterKey as defaultClusterKey } from './cluster.js';
import { POLL_MISS, createPoller, loadSettings as defaultLoadSettings, prometheusCandidates, seriesStepSec } from './settings.js';

/** Data younger than this is served from the shared store on mount without re-fetching. */
export const STALE_MS = 5000;

/** What a provider feeds by default: both lists and the DeviceConfigs (the reference's provider). */
const ALL_NEEDS = Object.freeze({ nodes: true, pods: true, crd: true, operatorPods: false });

/** A provider that reads the store and mounts nothing (a Node detail section next to a page that feeds it). */
export const READ_ONLY_NEEDS = Object.freeze({ nodes: false, pods: false, crd: false, operatorPods: false });

/**
 * Period (s) of a scoped request that stands in for a list + watch the host
 * would not scope (ADR 012) when auto-refresh is off: a watch is live, so
 * its stand-in is re-read rather than read once.
 */
export const SCOPED_POLL_SEC = 30;

export const PROMETHEUS_UNREACHABLE =
  'Could not reach Prometheus. Ensure kube-prometheus-stack is installed in the monitoring namespace.';

export const PROMETHEUS_FORBIDDEN =
  'Access to Prometheus was denied (HTTP 403): your user needs "get" on services/proxy for the Prometheus service in the monitoring namespace (deploy/rbac/headlamp-amd-gpu-viewer.yaml).';

export const OUTSIDE_PROVIDER = 'useAmdGpuContext must be used within an AmdGpuDataProvider';

const HOOKS = ['createContext', 'createElement', 'useContext', 'useEffect', 'useMemo', 'useRef', 'useState', 'useSyncExternalStore'];

function errorText(e) {
  return e instanceof Error ? e.message : String(e);
}

/**
 * [items, error] from either shape of a Headlamp list-hook result (see
 * useListOf). `items` null means "not listed yet" (or failed).
 * @param {any} res
 * @returns {[any[]|null, any]}
 */
export function listResult(res) {
  if (!res) return [null, null];
  if (Array.isArray(res)) return [res[0] !== undefined ? res[0] : null, res[1] !== undefined ? res[1] : null];
  let err = res.error !== undefined ? res.error : null;
  if (!err && res.errors) err = Array.isArray(res.errors) ? (res.errors.length ? res.errors[0] : null) : res.errors;
  const items = res.isLoading || res.items === undefined ? null : res.items;
  return [items, err || null];
}

/**
 * @param {any} React  React 18 (or the harness stand-in)
 * @param {{K8s: any, ApiProxy: any}} lib  '@kinvolk/headlamp-plugin/lib'
 * @param {{request?: (path: string) => Promise<any>, clusterKey?: () => string,
 *          loadSettings?: () => ReturnType<typeof defaultLoadSettings>}} [deps]
 */
export function createProviderCore(React, lib, deps) {
  for (let i = 0; i < HOOKS.length; i++) {
    if (!React || typeof React[HOOKS[i]] !== 'function') throw new Error('createProviderCore: React.' + HOOKS[i] + ' is required');
  }
  const d = deps || {};
  const request = d.request || function (path) { return lib.ApiProxy.request(path); };
  const clusterKey = d.clusterKey || defaultClusterKey;
  const loadSettings = d.loadSettings || function () { return defaultLoadSettings(); };
  const h = React.createElement;
  const useEffect = React.useEffect;
  const useMemo = React.useMemo;
  const useState = React.useState;

  const Context = React.createContext(null);

  /** The shared store of a cluster (created on first use; keyed by the settings that shape it). */
  function storeFor(cluster) {
    const settings = loadSettings();
    return getSharedStore(cluster + '|' + settings.requestTimeoutMs, function () {
      return createClusterStore({ request: request, timeoutMs: settings.requestTimeoutMs });
    });
  }

  const metricsSources = {};

  function sourceKey(cluster, settings) {
    return cluster + '|' + JSON.stringify(settings.prometheus) + '|' + settings.requestTimeoutMs;
  }

  /**
   * The shared Prometheus client of a cluster (its discovery cache lives
   * here). Keyed by the settings that shape it, so saving new settings takes
   * effect on the next mount.
   */
  function metricsSourceFor(cluster) {
    const settings = loadSettings();
    const key = sourceKey(cluster, settings);
    if (!metricsSources[key]) {
      metricsSources[key] = createMetricsSource({
        request: request,
        services: prometheusCandidates(settings),
        timeoutMs: settings.requestTimeoutMs,
      });
    }
    return metricsSources[key];
  }

  function useAmdGpuContext() {
    const ctx = React.useContext(Context);
    if (!ctx) throw new Error(OUTSIDE_PROVIDER);
    return ctx;
  }

  /**
   * [items, error] of a Headlamp list hook. Headlamp's `useList()` returns
   * `[items, error, ...]` (the reference destructures it, :98-99; items null
   * while the first list is in flight and when it failed); later Headlamp
   * releases return a result object `{items, error | errors, isLoading}`.
   * Both shapes are read, so a host upgrade does not leave pages loading.
   */
  function useListOf(cls, opts) {
    const res = opts ? cls.useList(opts) : cls.useList();
    return listResult(res);
  }

  /** Feeds Headlamp's node list + watch into the store (its own component: the hook runs only where mounted). */
  function NodeListFeed(props) {
    const store = props.store;
    const nodes = useListOf(lib.K8s.ResourceClasses.Node);
    const allNodes = nodes[0];
    const nodeError = nodes[1];
    useEffect(function () {
      store.setNodes(allNodes === undefined ? null : allNodes, nodeError ? errorText(nodeError) : null);
    }, [store, allNodes, nodeError]);
    return null;
  }

  /**
   * Feeds Headlamp's all-namespaces pod list + watch into the store. While
   * one is mounted the store derives operator pods from it; after the last
   * unmounts they come from the plugin-pod requests (clusterStore.js
   * attachPodFeed).
   */
  function PodListFeed(props) {
    const store = props.store;
    useEffect(function () { return store.attachPodFeed(); }, [store]);
    const pods = useListOf(lib.K8s.ResourceClasses.Pod, { namespace: '' });
    const allPods = pods[0];
    const podError = pods[1];
    useEffect(function () {
      store.setPods(allPods === undefined ? null : allPods, podError ? errorText(podError) : null);
    }, [store, allPods, podError]);
    return null;
  }

  /**
   * The operator pods by their own lists + watches (k8sCore.js
   * OPERATOR_POD_LISTS: the plugin labels outside the operator namespace,
   * and the operator namespace) — what a page that draws operator pods but
   * no other pod mounts (Device Plugins), instead of the all-namespaces list.
   * Live like the reference's provider lists (IntelGpuDataContext.tsx:98-99),
   * whose operator pods only changed on a Refresh click (:142-165). A
   * failing list contributes nothing, as a failing selector request does in
   * the reference (:162-164); both failing hand over to the plugin-pod
   * requests (clusterStore.js setOperatorPods).
   */
  function OperatorPodFeed(props) {
    const store = props.store;
    useEffect(function () { return store.attachOperatorFeed(); }, [store]);
    const a = useListOf(lib.K8s.ResourceClasses.Pod, OPERATOR_POD_LISTS[0]);
    const b = useListOf(lib.K8s.ResourceClasses.Pod, OPERATOR_POD_LISTS[1]);
    const fed = useMemo(function () {
      const lists = [a, b];
      let pending = false;
      let failed = 0;
      let found = [];
      let outside = 0;
      for (let i = 0; i < lists.length; i++) {
        if (lists[i][1]) failed++;
        else if (!lists[i][0]) pending = true;
        else {
          const raw = unwrapAll(lists[i][0]);
          outside += countOutside(raw, OPERATOR_POD_LISTS[i]);
          found = found.concat(filterAmdGpuPluginPods(raw));
        }
      }
      if (failed === lists.length) return { items: null, error: errorText(a[1]), outside: outside };
      // A host that dropped the list options delivered every pod: the answer
      // is still right (the plugin-pod filter), but the provider swaps this
      // feed for the scoped requests (OperatorPodPoll).
      return { items: pending ? null : dedupePods(found), error: null, outside: outside };
    }, [a[0], a[1], b[0], b[1]]);
    useEffect(function () {
      store.setOperatorPods(fed.items, fed.error);
      if (fed.outside > 0) store.noteSelectorIgnored('operatorPods', fed.outside, fed);
    }, [store, fed]);
    return null;
  }

  /** How often a scoped request standing in for a watch is re-read: the refresh period, else SCOPED_POLL_SEC. */
  function scopedPollSec() {
    const sec = loadSettings().refreshIntervalSec;
    return sec > 0 ? sec : SCOPED_POLL_SEC;
  }

  /**
   * The operator pods by the plugin-pod requests (PLUGIN_POD_QUERIES: the
   * same two selections, applied by the apiserver as query parameters),
   * re-read every scopedPollSec(): what the provider mounts instead of
   * OperatorPodFeed on a host that ignores useList() options, so Device
   * Plugins never mounts the unscoped lists such a host would deliver.
   */
  function OperatorPodPoll(props) {
    const store = props.store;
    const period = scopedPollSec();
    useEffect(function () { return store.attachOperatorFeed(); }, [store]);
    useEffect(function () {
      store.loadOperatorPods();
      const poller = createPoller(period);
      poller.start(function () { return store.loadOperatorPods(); });
      return function () { poller.stop(); };
    }, [store, period]);
    return null;
  }

  /**
   * The pod list + watch fed into the current cluster's store, mounted by a
   * page whose provider does not feed pods when one of its views needs them
   * after all (the Metrics page in an allocation order).
   */
  function PodListHere() {
    return h(PodListFeed, { store: storeFor(clusterKey()) });
  }

  /**
   * The cluster context of a page. `props.needs` says what the page draws
   * ({nodes, pods, crd}, each default true; `operatorPods`, default false:
   * the operator pods' own lists where the pod list is not mounted): only those are subscribed to
   * and fetched — the Metrics page mounts the node list alone, never the
   * all-namespaces pod list (tens of MB, parsed on the browser's main thread
   * on a large cluster) nor the DeviceConfig request; the reference mounts
   * both lists and its CRD + 3 serial requests on every route
   * (src/index.tsx:87-145, IntelGpuDataContext.tsx:98-165). What one page
   * fed stays in the shared store for the next. `loading` is the reference's
   * rule over what this provider feeds.
   */
  function AmdGpuDataProvider(props) {
    const store = storeFor(clusterKey());
    const needs = props.needs || ALL_NEEDS;
    const wantNodes = needs.nodes !== false;
    const wantPods = needs.pods !== false;
    const wantCrd = needs.crd !== false;
    const wantOps = needs.operatorPods === true && !wantPods;

    // Track 2 — imperative CRD / operator-pod fetch, shared and deduplicated.
    useEffect(function () {
      if (wantCrd) store.revalidate(STALE_MS);
    }, [store, wantCrd]);

    // Optional auto-refresh (settings; the reference only refreshes on click).
    const refreshIntervalSec = loadSettings().refreshIntervalSec;
    useEffect(function () {
      if (!wantCrd) return undefined;
      const poller = createPoller(refreshIntervalSec);
      poller.start(function () { return store.revalidate(STALE_MS); });
      return function () { poller.stop(); };
    }, [store, refreshIntervalSec, wantCrd]);

    const snapshot = React.useSyncExternalStore(store.subscribe, store.getSnapshot);
    const value = useMemo(function () {
      const loading = (wantCrd && snapshot.crdLoading) || (wantNodes && snapshot.nodesLoading) ||
        (wantPods && snapshot.podsLoading) || (wantOps && snapshot.pluginPodsLoading);
      return Object.assign({}, snapshot, { loading: !!loading, refresh: function () { store.refresh(); } });
    }, [snapshot, store, wantCrd, wantNodes, wantPods, wantOps]);

    // Track 1 — reactive lists from Headlamp (all namespaces for pods), as
    // feed components next to the page, so a page mounts only the watches it draws.
    return h(Context.Provider, { value: value },
      wantNodes ? h(NodeListFeed, { store: store }) : null,
      wantPods ? h(PodListFeed, { store: store }) : null,
      wantOps ? h(store.selectorsIgnored('operatorPods') ? OperatorPodPoll : OperatorPodFeed, { store: store }) : null,
      props.children);
  }

  const IDLE = { metrics: null, series: null, fetchError: null, fetching: false };

  /**
   * One metrics fetch bound to component state, re-run by `refresh()` and by
   * the auto-refresh poller. `key` null fetches nothing; a new key (or an
   * unmount) drops the previous key's in-flight answer (the reference's
   * `cancelled` flag, MetricsPage.tsx:206-230).
   * @param {string|null} key
   * @param {(early: (metrics: any) => void) => Promise<[any, any]>} fetchPair  resolves [metrics, series];
   *   may call `early(metrics)` when the telemetry is in before the series (the page shows it at once)
   * @param {boolean} [seriesOnly]  the fetch returns series only: unreachable = no series
   * @param {{failureReason?: () => string}} [source]  says whether a failure was RBAC (403) or an outage
   */
  function useMetricsFetch(key, fetchPair, seriesOnly, source) {
    const refreshIntervalSec = loadSettings().refreshIntervalSec;
    const st = useState(IDLE);
    const state = st[0];
    const setState = st[1];
    const sq = useState(0);
    const seq = sq[0];
    const setSeq = sq[1];

    useEffect(function () {
      if (key === null) return undefined;
      let cancelled = false;
      setState(function (s) { return Object.assign({}, s, { fetching: true, fetchError: null }); });
      fetchPair(function early(metrics) {
        if (cancelled || !metrics) return;
        // Telemetry ahead of its range series: shown now, the series (and
        // `fetching`) follow with the pair.
        setState(function (s) { return Object.assign({}, s, { metrics: metrics, fetchError: null }); });
      }).then(
        function (pair) {
          if (cancelled) return;
          const metrics = pair[0];
          const reached = seriesOnly ? !!pair[1] : !!metrics;
          const why = !reached && source && source.failureReason ? source.failureReason() : 'unreachable';
          setState({
            metrics: metrics, series: pair[1], fetching: false,
            fetchError: reached ? null : why === 'forbidden' ? PROMETHEUS_FORBIDDEN : PROMETHEUS_UNREACHABLE,
          });
        },
        function (e) {
          if (cancelled) return;
          setState(function (s) { return Object.assign({}, s, { fetching: false, fetchError: errorText(e) }); });
        }
      );
      return function () { cancelled = true; };
      // `fetchPair` is rebuilt every render; `key` names what it fetches.
    }, [key, seq]);

    // The poller backs off while Prometheus does not answer or refuses the
    // proxy (each tick would otherwise re-run discovery: a query plus one
    // probe per candidate); a manual refresh is never delayed.
    const unreachable = React.useRef(false);
    useEffect(function () {
      unreachable.current = state.fetchError === PROMETHEUS_UNREACHABLE || state.fetchError === PROMETHEUS_FORBIDDEN;
    }, [state.fetchError]);
    useEffect(function () {
      if (key === null) return undefined;
      const poller = createPoller(refreshIntervalSec);
      poller.start(function () {
        const miss = unreachable.current;
        setSeq(function (s) { return s + 1; });
        return miss ? POLL_MISS : undefined;
      });
      return function () { poller.stop(); };
    }, [key, refreshIntervalSec]);

    return useMemo(function () {
      return Object.assign({}, state, { refresh: function () { setSeq(function (s) { return s + 1; }); } });
    }, [state]);
  }

  /**
   * GPU telemetry (+ power/HBM series when `withSeries`) of the series `view`
   * draws (metrics.js METRIC_VIEWS: 'gauges' for the Metrics page, 'topology'
   * for GPU Nodes, default 'all').
   *
   * `scope` (optional) is the list of GPU node names the page shows (a paged
   * view, pages.js nodePage): telemetry and series are then fetched for those
   * nodes only, and on the 'gauges' view with the cluster totals as
   * server-side aggregates — O(page) bytes on any cluster. Without `scope`
   * the whole cluster is fetched (terminal client, small clusters).
   *
   * `rank` (pages.js telemetryScope, Metrics in power order): Prometheus
   * picks the page (metrics.js rankedClusterQuery); the page's series are
   * asked for once its names are in, a second round trip.
   *
   * `small` (pages.js telemetryScope): the page may be the whole cluster —
   * every GPU when the cluster is small, else `scope`'s nodes, decided by
   * Prometheus (metrics.js smallClusterQuery). The query key then leaves out
   * the names, so the node list arriving does not refetch; a refresh asks
   * with the names of that render.
   *
   * Unlike the reference it does not wait for the cluster context to finish
   * loading (MetricsPage.tsx:203-205): the two are independent and fetched in
   * parallel.
   */
  function useGpuMetrics(enabled, withSeries, view, scope, small, rank) {
    const on = enabled === undefined ? true : enabled;
    const series = withSeries === undefined ? true : withSeries;
    const v = view || 'all';
    const cluster = clusterKey();
    const source = metricsSourceFor(cluster);
    const settings = loadSettings();
    const scoped = Array.isArray(scope);
    const names = scoped ? scope.slice() : null;
    const sm = scoped && !!small;
    const ex = useState(false);
    const rk = rank ? rank.by + ':' + rank.page + ':' + rank.per + ':' + rank.filter : null;
    const key = 'gpus|' + sourceKey(cluster, settings) + '|' + v + '|' + series + '|' + settings.seriesMinutes +
      (rk ? '|rank:' + rk : sm ? smallKey(ex[0], names) : scoped ? '|scope:' + names.join(',') : '');
    const res = useMetricsFetch(on ? key : null, function (early) {
      if (rk) {
        // The ranked page's names come with the answer: its series follow it.
        return source.fetchGpuMetrics(v, { rank: rank, summary: v === 'gauges' }).then(function (m) {
          if (!series || !m) return [m, null];
          early(m);
          return source.fetchSeries(settings.seriesMinutes * 60, seriesStepSec(settings), m.scope || [])
            .then(function (sr) { return [m, sr]; });
        });
      }
      const opts = scoped ? { scope: names, summary: v === 'gauges', small: sm } : undefined;
      const mp = source.fetchGpuMetrics(v, opts);
      // The range series usually answer after the instant telemetry: the page shows the telemetry first.
      if (series) mp.then(early, function () {});
      return Promise.all([
        mp,
        series ? source.fetchSeries(settings.seriesMinutes * 60, seriesStepSec(settings), names || undefined, sm) : Promise.resolve(null),
      ]);
    }, false, source);
    useExceeded(sm, res, ex);
    return res;
  }

  /**
   * Key suffix of a small-cluster fetch: one key while the answer held the
   * whole cluster, so the node list arriving refetches nothing. An answer
   * that found more than one page (stale series of a removed node, exporter
   * hostnames the node list lacks) held only the names known when it was
   * asked: then the key follows the names, and new names are fetched.
   */
  function smallKey(exceeded, names) {
    return '|small' + (exceeded && names.length ? ':' + names.join(',') : '');
  }

  /** Track `res.metrics.small.exceeded` in the state pair `ex` (see smallKey). */
  function useExceeded(sm, res, ex) {
    const now = !!(sm && res.metrics && res.metrics.small && res.metrics.small.exceeded);
    const was = ex[0];
    const set = ex[1];
    useEffect(function () {
      if (now !== was) set(now);
    }, [now, was]);
  }

  /**
   * Telemetry of one node's GPUs for the native Node / Pod detail pages: a
   * `hostname`-scoped query through the shared client (metrics.js
   * fetchNodeMetrics), so a detail page costs the same few KB on a 500-node
   * cluster as on one node. `nodeName` null (or `enabled` false) fetches
   * nothing.
   */
  function useNodeGpuMetrics(nodeName, enabled) {
    const cluster = clusterKey();
    const source = metricsSourceFor(cluster);
    const active = (enabled === undefined ? true : enabled) && !!nodeName;
    return useMetricsFetch(active ? 'node|' + sourceKey(cluster, loadSettings()) + '|' + nodeName : null, function () {
      return source.fetchNodeMetrics(nodeName).then(function (m) { return [m, null]; });
    }, false, source);
  }

  /**
   * One pod's GPU power history for the native Pod detail page
   * (metrics.js fetchPodSeries): one pod-scoped range query, next to the
   * node-scoped telemetry query.
   */
  function usePodGpuSeries(namespace, pod, enabled) {
    const cluster = clusterKey();
    const source = metricsSourceFor(cluster);
    const settings = loadSettings();
    const active = (enabled === undefined ? true : enabled) && !!namespace && !!pod;
    const key = 'podseries|' + sourceKey(cluster, settings) + '|' + namespace + '/' + pod + '|' + settings.seriesMinutes;
    return useMetricsFetch(active ? key : null, function () {
      return source.fetchPodSeries(namespace, pod, settings.seriesMinutes * 60, seriesStepSec(settings))
        .then(function (sr) { return [null, sr]; });
    }, true);
  }

  /** One node's GPU power history for the native Node detail page (metrics.js fetchNodeSeries). */
  function useNodeGpuSeries(nodeName, enabled) {
    const cluster = clusterKey();
    const source = metricsSourceFor(cluster);
    const settings = loadSettings();
    const active = (enabled === undefined ? true : enabled) && !!nodeName;
    const key = 'nodeseries|' + sourceKey(cluster, settings) + '|' + nodeName + '|' + settings.seriesMinutes;
    return useMetricsFetch(active ? key : null, function () {
      return source.fetchNodeSeries(nodeName, settings.seriesMinutes * 60, seriesStepSec(settings))
        .then(function (sr) { return [null, sr]; });
    }, true);
  }

  /**
   * Pod → GPU attribution for the Pods page (metrics.js fetchGpuOwners): one
   * series per allocated GPU — of the pods on the page when `pods` (their
   * "namespace/name" keys) is given, else of every pod; `small` as in
   * useGpuMetrics (pages.js ownersScope); `preview` (small, no page yet): on a
   * larger cluster the `preview` pods drawing the most power (a partial page
   * before the pod list is in).
   */
  function useGpuOwners(enabled, pods, small, rank, preview) {
    const cluster = clusterKey();
    const source = metricsSourceFor(cluster);
    const on = enabled === undefined ? true : enabled;
    const scoped = !rank && Array.isArray(pods);
    const keys = scoped ? pods.slice() : null;
    const sm = scoped && !!small;
    const ex = useState(false);
    // Power order (ownersScope rank): Prometheus picks the page's pods.
    const rk = rank ? rank.by + ':' + rank.page + ':' + rank.per + ':' + rank.filter : null;
    // The preview is asked with the first small query but is not part of its
    // key: on a small cluster the pod list arriving keeps the key (no refetch).
    const pre = sm && !keys.length && preview > 0 ? preview : 0;
    const key = 'owners|' + sourceKey(cluster, loadSettings()) +
      (rk ? '|rank:' + rk : sm ? smallKey(ex[0], keys) : scoped ? '|pods:' + keys.join(',') : '');
    const res = useMetricsFetch(on ? key : null, function () {
      const opts = rank ? { rank: rank } : scoped ? { pods: keys, small: sm, preview: pre } : undefined;
      return source.fetchGpuOwners(opts).then(function (m) { return [m, null]; });
    }, false, source);
    useExceeded(sm, res, ex);
    return res;
  }

  // The Node detail section's pods (nodePodHooks.js).
  const nodePods = createNodePodHooks(React, lib, {
    storeFor: storeFor, clusterKey: clusterKey, request: request, loadSettings: loadSettings,
    scopedPollSec: scopedPollSec, useListOf: useListOf, errorText: errorText,
  });

  return {
    Context: Context,
    AmdGpuDataProvider: AmdGpuDataProvider,
    PodListHere: PodListHere,
    useAmdGpuContext: useAmdGpuContext,
    useGpuMetrics: useGpuMetrics,
    useNodeGpuMetrics: useNodeGpuMetrics,
    useGpuOwners: useGpuOwners,
    usePodGpuSeries: usePodGpuSeries,
    useNodeGpuSeries: useNodeGpuSeries,
    useNodePods: nodePods.useNodePods,
    usePodsLive: nodePods.usePodsLive,
    storeFor: storeFor,
    metricsSourceFor: metricsSourceFor,
    /** The current cluster's key (per-cluster state: stores, view state). */
    clusterKey: clusterKey,
  };
}
