/**
 * ClusterStore — framework-agnostic data layer for the AMD GPU plugin.
 *
 * Replaces the reference's per-route React provider state
 * (src/api/IntelGpuDataContext.tsx:96-254, SURVEY.md C3) with a store that:
 *
 *   * refreshes with ONE request (the DeviceConfig list): operator pods are
 *     derived from the watched pod list (or the operator pods' own watched
 *     lists on a route that draws no other pod), and the plugin-pod requests run —
 *     in parallel, each time-boxed — only when that list is unavailable
 *     (reference: CRD + 3 selectors, serial, :122-165) — refresh latency is
 *     one RTT instead of Σ RTT;
 *   * keeps its last CRD state through transient failures and clears it on
 *     404 / 403 (reference: any failure = absent, :133-138);
 *   * keeps the last good data visible while a refresh is in flight
 *     (stale-while-revalidate) instead of swapping the page for a Loader;
 *   * is shared across routes and detail views through `getSharedStore`, so
 *     a route switch or a Node detail view reuses the cluster snapshot instead
 *     of starting cold (reference Q7);
 *   * clears its timeout timers (reference Q6) and drops responses from a
 *     superseded refresh via a sequence number (the analog of the
 *     reference's `cancelled` flag, :114/:187);
 *   * classifies only the objects a watch event changed (./listCache.js) and
 *     rebuilds the cluster index only when a GPU node / pod changed, with
 *     structural sharing per node (reference: every pod re-filtered per
 *     event, every aggregate recomputed per render).
 *
 * Nodes and pods arrive from Headlamp's `useList` watch through
 * `setNodes` / `setPods` (same two-track design as reference ADR 002);
 * `loadLists()` fetches them directly for harnesses without Headlamp.
 *
 * The store exposes `subscribe` / `getSnapshot` for React 18's
 * `useSyncExternalStore`; snapshots are immutable objects.
 */

import { isAmdGpuNode, isDeviceConfig } from './amdNodes.js';
import { dedupePods, filterAmdGpuPluginPods, isAmdGpuPluginPod, isGpuRequestingPod } from './amdPods.js';
import { buildClusterIndex, patchClusterIndex } from './clusterIndex.js';
import { DEVICE_CONFIG_LIST_PATH, isKubeList, PLUGIN_POD_QUERIES } from './k8sCore.js';
import { createListTracker } from './listCache.js';
import { primeOperatorFacts } from './operatorFacts.js';
import { DEFAULT_REQUEST_TIMEOUT_MS, defaultClock, isAbsent, sameObjects, withTimeout } from './requests.js';

export { DEFAULT_REQUEST_TIMEOUT_MS, fetchNodePods, isAbsent, nodePodsPath, nodePodsSelector, sameObjects, withTimeout } from './requests.js';

/** Time limit of a whole-cluster node / pod list (loadLists). */
export const LIST_TIMEOUT_MS = 60000;

/**
 * @typedef {Object} ClusterSnapshot
 * @property {any[]} deviceConfigs
 * @property {boolean} pluginInstalled
 * @property {any[]} gpuNodes
 * @property {any[]} gpuPods
 * @property {any[]} pluginPods
 * @property {boolean} crdAvailable
 * @property {boolean} crdForbidden  the DeviceConfig list was refused (401 / 403) rather than absent (404)
 * @property {boolean} loading      true until the node and pod lists have settled (arrived or
 *                                  failed) and the first CRD/pod fetch is in (the reference's
 *                                  rule, IntelGpuDataContext.tsx:214)
 * @property {boolean} nodesLoading the node list has not settled yet
 * @property {boolean} podsLoading  the pod list has not settled yet
 * @property {boolean} crdLoading   the first DeviceConfig / operator-pod fetch is not in yet
 *                                  (pages render what they can as each of the three settles:
 *                                  a page waits only for the lists it draws)
 * @property {boolean} pluginPodsLoading  the operator pods are not known yet: from the pod list
 *                                  while a pod feed is mounted, else from the plugin-pod
 *                                  requests (the Device Plugins route mounts no pod list)
 * @property {'unknown'|'pending'|'ready'|'error'} nodesState
 * @property {'unknown'|'pending'|'ready'|'error'} podsState
 * @property {boolean} refreshing   a refresh is in flight (data above is still valid)
 * @property {string|null} error
 * @property {ReturnType<typeof buildClusterIndex>} index
 * @property {number|null} lastUpdated  ms epoch of the last committed refresh
 * @property {number} version
 */

/**
 * @param {{ request: (path: string) => Promise<any>, timeoutMs?: number,
 *           clock?: {setTimeout: Function, clearTimeout: Function, now: Function},
 *           crdPath?: string, pluginPodQueries?: string[],
 *           onTrace?: (span: {name: string, path: string, start: number, end: number, ok: boolean}) => void }} opts
 */
export function createClusterStore(opts) {
  if (!opts || typeof opts.request !== 'function') throw new Error('createClusterStore: request(path) is required');
  const request = opts.request;
  const timeoutMs = opts.timeoutMs || DEFAULT_REQUEST_TIMEOUT_MS;
  const clock = opts.clock || defaultClock;
  const crdPath = opts.crdPath || DEVICE_CONFIG_LIST_PATH;
  const podQueries = opts.pluginPodQueries || PLUGIN_POD_QUERIES;
  const onTrace = opts.onTrace || null;

  const s = {
    nodes: null,
    nodeError: null,
    pods: null,
    podError: null,
    deviceConfigs: [],
    crdAvailable: false,
    crdForbidden: false, // the CRD list answered 401 / 403: RBAC, not a missing operator
    pluginPods: [], // from the plugin-pod queries (used when the pod list is not available or not watched)
    pluginPodsKnown: false, // s.pluginPods holds an answer (queried, or the watched list's last word)
    // The operator pods by their own scoped lists + watches (providerCore.js
    // OperatorPodFeed: the operator namespace, the plugin labels elsewhere) —
    // what the Device Plugins route mounts instead of the all-namespaces list.
    opPods: null,
    opPodsState: 'unknown',
    // Where each list stands: 'unknown' (never fed: harness/tests),
    // 'pending' (a list/watch is in flight), 'ready', or 'error'. An errored
    // list (e.g. pods forbidden cluster-wide) is settled: the page leaves its
    // loading state and shows the error, instead of waiting forever for a
    // list that will not come (reference quirk Q11 inferred loading from
    // `items === null`, IntelGpuDataContext.tsx:214).
    nodesState: 'unknown',
    podsState: 'unknown',
    asyncLoaded: false,
    refreshing: false,
    asyncError: null,
    lastUpdated: null,
  };
  let seq = 0;
  let inflight = null;
  let podsQueried = false; // the in-flight refresh includes the plugin-pod requests
  // Pod list feeds mounted right now (providerCore.js PodListFeed). A store
  // no feed ever attached to (harness, terminal client, tests feeding
  // setPods / loadLists themselves) treats its pod list as current; once
  // feeds attach, the list is current only while one is mounted — after the
  // last unmounts nothing keeps it up to date, so operator pods come from the
  // plugin-pod requests again.
  let podFeeds = 0;
  let feedsAttached = false;
  let opFeeds = 0; // operator pod feeds mounted right now
  // Objects a scoped list + watch delivered OUTSIDE the selection it asked
  // for (nodePodHooks.js NodePodsWatch, providerCore.js OperatorPodFeed): a host whose
  // useList() drops the list options. Once seen, those views read their
  // scoped requests instead (ADR 012).
  const ignored = { nodePods: 0, operatorPods: 0 };
  const noted = typeof WeakSet === 'function' ? new WeakSet() : null; // deliveries already counted
  let opLoad = null; // loadOperatorPods in flight
  let version = 0;
  const listeners = [];

  // GPU nodes, GPU pods and operator pods are kept incrementally
  // (./listCache.js): the watch delivers a new list on every event anywhere
  // in the cluster, but only objects that changed are classified again, and
  // each subset keeps its identity unless one of its members was added,
  // changed or removed — churn of unrelated pods costs one pass of identity
  // compares and invalidates no memoised view downstream.
  const nodeTracker = createListTracker([isAmdGpuNode]);
  const podTracker = createListTracker([isGpuRequestingPod, isAmdGpuPluginPod]);
  let memoGpuNodes = [];
  let memoGpuPods = [];
  let memoPluginPods = [];
  const counters = { indexBuilds: 0, indexPatches: 0 };
  let memoIndexKey = [null, null];
  let memoIndex = buildClusterIndex([], []);
  let snapshot = null;

  function trackNodes(items) {
    const r = nodeTracker.update(items || []);
    if (r.changed[0] && !sameObjects(memoGpuNodes, r.subsets[0])) memoGpuNodes = r.subsets[0];
    if (!items) memoGpuNodes = [];
  }
  function trackPods(items) {
    const r = podTracker.update(items || []);
    if (r.changed[0] && !sameObjects(memoGpuPods, r.subsets[0])) {
      // A delta of the GPU pods (status updates, pods added / removed):
      // patch the index of the current nodes + previous pods instead of
      // rebuilding it from every GPU node and pod.
      const delta = r.deltas[0];
      if (delta && memoIndexKey[0] === memoGpuNodes && memoIndexKey[1] === memoGpuPods) {
        const patched = patchClusterIndex(memoIndex, delta, podTracker.positionOf);
        if (patched) {
          counters.indexPatches++;
          memoIndex = patched;
          memoIndexKey = [memoGpuNodes, r.subsets[0]];
        }
      }
      memoGpuPods = r.subsets[0];
    }
    if (r.changed[1] && !sameObjects(memoPluginPods, r.subsets[1])) memoPluginPods = r.subsets[1];
    if (!items) {
      memoGpuPods = [];
      memoPluginPods = [];
    }
  }
  function gpuNodes() {
    return memoGpuNodes;
  }
  function gpuPods() {
    return memoGpuPods;
  }
  /**
   * Operator pods, from whichever watch delivers them. While Headlamp's pod
   * list (all namespaces) is watched they are derived from it: it already
   * holds every pod the reference's three plugin-pod requests return, so a
   * refresh needs only the CRD request. A route that watches the operator
   * pods' own lists instead (Device Plugins: attachOperatorFeed) reads those.
   * With neither (forbidden, failed, unmounted, or no watch at all) they come
   * from the PLUGIN_POD_QUERIES requests.
   */
  function pluginPods() {
    if (s.podsState === 'ready' && s.pods && podsLive()) return memoPluginPods;
    if (opFeeds > 0 && s.opPodsState === 'ready') return s.opPods;
    return s.pluginPods;
  }
  /** The pod list is kept current (a feed is mounted, or no feed ever was: see podFeeds). */
  function podsLive() {
    return podFeeds > 0 || !feedsAttached;
  }
  /** The all-namespaces pod list is there or on its way, and kept current. */
  function listLive() {
    return s.podsState !== 'unknown' && s.podsState !== 'error' && podsLive();
  }
  /** An operator pod feed is mounted and has not failed: its watches keep the operator pods current. */
  function opLive() {
    return opFeeds > 0 && s.opPodsState !== 'error';
  }
  function pluginPodsLoading() {
    if (podsLive() && s.podsState !== 'unknown') return !settled(s.podsState);
    // While the operator feed's first lists are in flight, a known answer stays shown.
    if (opLive() && s.opPodsState !== 'unknown') return s.opPodsState === 'pending' && !s.pluginPodsKnown;
    return !s.pluginPodsKnown;
  }
  function index(n, p) {
    if (memoIndexKey[0] !== n || memoIndexKey[1] !== p) {
      memoIndexKey = [n, p];
      memoIndex = buildClusterIndex(n, p, memoIndex);
      counters.indexBuilds++;
    }
    return memoIndex;
  }

  let primedConfigs = null;

  function build() {
    const n = gpuNodes();
    const p = gpuPods();
    const errors = [];
    if (s.nodeError) errors.push(String(s.nodeError));
    if (s.podError) errors.push(String(s.podError));
    if (s.asyncError) errors.push(s.asyncError);
    const pp = pluginPods();
    // The DeviceConfigs' facts, once per list (operatorFacts.js); operator
    // pods' when a page shows their row.
    if (s.deviceConfigs !== primedConfigs) {
      primeOperatorFacts(s.deviceConfigs);
      primedConfigs = s.deviceConfigs;
    }
    version++;
    return Object.freeze({
      deviceConfigs: s.deviceConfigs,
      pluginInstalled: s.deviceConfigs.length > 0 || pp.length > 0,
      gpuNodes: n,
      gpuPods: p,
      pluginPods: pp,
      crdAvailable: s.crdAvailable,
      crdForbidden: s.crdForbidden,
      loading: !s.asyncLoaded || !settled(s.nodesState) || !settled(s.podsState),
      nodesLoading: !settled(s.nodesState),
      podsLoading: !settled(s.podsState),
      crdLoading: !s.asyncLoaded,
      pluginPodsLoading: pluginPodsLoading(),
      nodesState: s.nodesState,
      podsState: s.podsState,
      refreshing: s.refreshing,
      error: errors.length ? errors.join('; ') : null,
      index: index(n, p),
      lastUpdated: s.lastUpdated,
      version: version,
    });
  }

  function settled(state) {
    return state === 'ready' || state === 'error';
  }

  function emit() {
    snapshot = build();
    const ls = listeners.slice();
    for (let i = 0; i < ls.length; i++) ls[i]();
  }

  function traced(name, path, ms) {
    const start = clock.now();
    const p = withTimeout(request(path), ms || timeoutMs, clock);
    if (!onTrace) return p;
    return p.then(
      function (v) {
        onTrace({ name: name, path: path, start: start, end: clock.now(), ok: true });
        return v;
      },
      function (e) {
        onTrace({ name: name, path: path, start: start, end: clock.now(), ok: false });
        throw e;
      }
    );
  }

  /** Run the plugin-pod requests; resolves to the deduplicated operator pods. */
  function queryPluginPods() {
    const pods = podQueries.map(function (path, i) {
      return traced('plugin-pods-' + i, path).then(
        function (list) { return isKubeList(list) ? filterAmdGpuPluginPods(list.items) : []; },
        function () { return []; }
      );
    });
    return Promise.all(pods).then(function (results) {
      let found = [];
      for (let i = 0; i < results.length; i++) found = found.concat(results[i]);
      return dedupePods(found);
    });
  }

  function commitQueriedPods(pods) {
    s.pluginPods = sameObjects(s.pluginPods, pods) ? s.pluginPods : pods;
    s.pluginPodsKnown = true;
  }

  /**
   * Re-fetch the DeviceConfig CRD (and, only while no pod list is available,
   * the operator pods). Resolves once the new data is committed (or dropped
   * because a newer refresh superseded it).
   * @returns {Promise<void>}
   */
  function refresh() {
    const my = ++seq;
    s.refreshing = true;
    emit();
    const crd = traced('crd', crdPath).then(
      function (list) {
        return isKubeList(list) ? { ok: true, items: list.items.filter(isDeviceConfig) } : { ok: false, items: [] };
      },
      function (e) {
        // A missing or forbidden CRD degrades silently (reference ADR 003).
        // A timeout or server error says nothing about the CRD: keep the last
        // known state instead of flapping to "CRD Not Available".
        const st = e && (e.status || (e.response && e.response.status));
        return { ok: isAbsent(e) ? false : null, items: [], forbidden: st === 403 || st === 401 };
      }
    );
    // The plugin-pod requests run only when no watch delivers operator pods:
    // neither the all-namespaces pod list nor the operator pod feed.
    const needPods = !listLive() && !opLive();
    podsQueried = needPods;
    const pods = needPods ? queryPluginPods() : Promise.resolve(null);
    const run = Promise.all([crd, pods]).then(
      function (results) {
        if (my !== seq) return;
        podsQueried = false;
        const c = results[0];
        if (c.ok !== null || !s.asyncLoaded) {
          s.crdAvailable = c.ok === true;
          s.crdForbidden = !!c.forbidden;
          // Structural sharing: an unchanged list keeps its identity, so every
          // memoised view (and React.memo'd section) downstream is reused.
          s.deviceConfigs = sameObjects(s.deviceConfigs, c.items) ? s.deviceConfigs : c.items;
        }
        if (results[1]) commitQueriedPods(results[1]);
        s.asyncError = null;
        s.asyncLoaded = true;
        s.refreshing = false;
        s.lastUpdated = clock.now();
        emit();
      },
      function (err) {
        if (my !== seq) return;
        podsQueried = false;
        s.asyncError = err instanceof Error ? err.message : String(err);
        s.asyncLoaded = true;
        s.refreshing = false;
        emit();
      }
    );
    inflight = run;
    return run;
  }

  /** Feed the Headlamp `useList()` result for nodes (wrappers are unwrapped here). */
  function setNodes(items, error) {
    const next = items ? (Array.isArray(items) ? items : []) : null;
    const err = error ? String(error) : null;
    const state = err ? 'error' : next ? 'ready' : 'pending';
    if (items === null && s.nodes === null && err === s.nodeError && state === s.nodesState) return;
    // A view mounting a fresh list hook reports "no items yet" while its
    // watch starts; the list already held stays valid (stale-while-
    // revalidate) instead of blanking every page back to its loader.
    if (state === 'pending' && s.nodesState === 'ready') return;
    s.nodes = next;
    s.nodeError = err;
    s.nodesState = state;
    trackNodes(next);
    emit();
  }

  function setPods(items, error) {
    const next = items ? (Array.isArray(items) ? items : []) : null;
    const err = error ? String(error) : null;
    const state = err ? 'error' : next ? 'ready' : 'pending';
    if (items === null && s.pods === null && err === s.podError && state === s.podsState) return;
    if (state === 'pending' && s.podsState === 'ready') return;
    const wasError = s.podsState === 'error';
    s.pods = next;
    s.podError = err;
    s.podsState = state;
    trackPods(next);
    emit();
    // The pod list failed (e.g. cluster-wide list forbidden): fall back to the
    // plugin-pod requests so operator pods still show.
    if (state === 'error' && !wasError && !(s.refreshing && podsQueried)) {
      queryPluginPods().then(function (pods) {
        if (s.podsState !== 'error') return;
        commitQueriedPods(pods);
        emit();
      });
    }
  }

  /**
   * Fetch nodes and pods directly (harness / cold start without Headlamp
   * hooks); `which` ({nodes, pods}, default both) says which lists, as a
   * route's provider mounts only the lists its page draws. Runs in parallel
   * with nothing else; callers usually do
   * `Promise.all([store.loadLists(), store.refresh()])`.
   */
  function loadLists(which) {
    const w = which || {};
    const wantNodes = w.nodes !== false;
    const wantPods = w.pods !== false;
    if (wantPods && s.podsState === 'unknown') s.podsState = 'pending';
    if (wantNodes && s.nodesState === 'unknown') s.nodesState = 'pending';
    // Whole-cluster lists (what Headlamp's useList() delivers in the plugin;
    // loaded here by the terminal client and the harness) take far longer
    // than a CRD request on a large cluster: tens of MB at 1,000 nodes.
    const nodesP = !wantNodes ? null : traced('nodes', '/api/v1/nodes', LIST_TIMEOUT_MS).then(
      function (l) { setNodes(isKubeList(l) ? l.items : [], null); },
      function (e) { setNodes([], e instanceof Error ? e.message : String(e)); }
    );
    const podsP = !wantPods ? null : traced('pods', '/api/v1/pods', LIST_TIMEOUT_MS).then(
      function (l) { setPods(isKubeList(l) ? l.items : [], null); },
      function (e) { setPods([], e instanceof Error ? e.message : String(e)); }
    );
    return Promise.all([nodesP, podsP]).then(function () {});
  }

  /**
   * A pod list feed mounted (providerCore.js PodListFeed); returns its
   * detach. When the last feed detaches, the watched list's operator pods
   * become the queried answer (the freshest known) until the next refresh
   * asks the plugin-pod requests.
   */
  function attachPodFeed() {
    const wasLive = podsLive();
    podFeeds++;
    feedsAttached = true;
    let attached = true;
    // The watched list is the operator pods' source again (a re-mounted feed).
    if (podFeeds === 1 && !wasLive) emit();
    return function detach() {
      if (!attached) return;
      attached = false;
      podFeeds--;
      if (podFeeds > 0) return;
      if (s.podsState === 'ready' && s.pods) {
        s.pluginPods = memoPluginPods;
        s.pluginPodsKnown = true;
      }
      emit();
    };
  }

  /**
   * An operator pod feed mounted (providerCore.js OperatorPodFeed); returns
   * its detach. While one is mounted its lists + watches are the operator
   * pods' source (unless the all-namespaces list is watched too) and a
   * refresh is the CRD request alone; after the last unmounts its answer is
   * kept as the last known one, as for attachPodFeed.
   */
  function attachOperatorFeed() {
    opFeeds++;
    let attached = true;
    if (opFeeds === 1 && s.opPodsState === 'ready') emit();
    return function detach() {
      if (!attached) return;
      attached = false;
      opFeeds--;
      if (opFeeds > 0) return;
      if (s.opPodsState === 'ready' && s.opPods) commitQueriedPods(s.opPods);
      emit();
    };
  }

  /**
   * Feed the operator pod lists (already unwrapped, filtered to operator
   * pods and deduplicated): `items` null while they are in flight. A list
   * already held stays while a re-mounted feed reports "no items yet".
   */
  function setOperatorPods(items, error) {
    const next = items ? (Array.isArray(items) ? items : []) : null;
    const state = error ? 'error' : next ? 'ready' : 'pending';
    if (state === 'pending' && (s.opPodsState === 'ready' || s.opPodsState === 'pending')) return;
    const wasError = s.opPodsState === 'error';
    s.opPodsState = state;
    if (next) s.opPods = sameObjects(s.opPods, next) ? s.opPods : next;
    emit();
    // Both scoped lists failed: the plugin-pod requests are the fallback.
    if (state === 'error' && !wasError && !listLive() && !(s.refreshing && podsQueried)) {
      queryPluginPods().then(function (pods) {
        if (s.opPodsState !== 'error') return;
        commitQueriedPods(pods);
        emit();
      });
    }
  }

  /**
   * Fetch the operator pod lists directly (the list requests an operator pod
   * feed's watches start with), for clients without Headlamp's hooks (the
   * benchmark): the plugin-pod requests, fed through setOperatorPods.
   */
  function loadOperatorPods() {
    // Callers asking while a load is in flight share it (an effect run twice).
    if (opLoad) return opLoad;
    if (s.opPodsState === 'unknown') s.opPodsState = 'pending';
    const lists = podQueries.map(function (path, i) {
      return traced('operator-pods-' + i, path).then(
        function (list) { return { items: isKubeList(list) ? filterAmdGpuPluginPods(list.items) : [] }; },
        function (e) { return { error: e instanceof Error ? e.message : String(e) }; }
      );
    });
    const run = Promise.all(lists).then(function (rs) {
      opLoad = null;
      let found = [];
      let failed = 0;
      for (let i = 0; i < rs.length; i++) {
        if (rs[i].error) failed++;
        else found = found.concat(rs[i].items);
      }
      if (failed === rs.length) setOperatorPods(null, rs[0].error);
      else setOperatorPods(dedupePods(found), null);
    });
    opLoad = run;
    return run;
  }

  /**
   * A scoped list + watch of `kind` delivered `n` objects outside its
   * selection: the host ignored the list options. Counted (counters()
   * .selectorIgnored); the first report notifies subscribers, so the views
   * switch to their scoped requests.
   */
  function noteSelectorIgnored(kind, n, delivery) {
    if (!(kind in ignored) || !(n > 0)) return;
    // One delivery is counted once, however often its effect runs (StrictMode).
    if (delivery && noted) {
      if (noted.has(delivery)) return;
      noted.add(delivery);
    }
    const first = ignored[kind] === 0;
    ignored[kind] += n;
    if (first) emit();
  }

  function subscribe(fn) {
    listeners.push(fn);
    return function () {
      const i = listeners.indexOf(fn);
      if (i >= 0) listeners.splice(i, 1);
    };
  }

  function getSnapshot() {
    if (!snapshot) snapshot = build();
    return snapshot;
  }

  /**
   * Refresh unless a refresh is already in flight or the data is younger
   * than `maxAgeMs` — what each mounting view calls, so N providers mounted
   * together (a route + a Node detail section) cost one fetch, not N.
   */
  function revalidate(maxAgeMs) {
    // Operator pods nobody knows: no pod list is watched and no refresh asked
    // the plugin-pod requests (a route without the pod list mounted after one
    // whose list never arrived) — fresh DeviceConfigs alone do not do.
    const podsMissing = !podsLive() && !opLive() && !s.pluginPodsKnown;
    if (s.refreshing && inflight && !(podsMissing && !podsQueried)) return inflight;
    const age = s.lastUpdated === null ? Infinity : clock.now() - s.lastUpdated;
    if (age < (maxAgeMs === undefined ? 0 : maxAgeMs) && !podsMissing) return Promise.resolve();
    return refresh();
  }

  return {
    subscribe: subscribe,
    getSnapshot: getSnapshot,
    setNodes: setNodes,
    setPods: setPods,
    attachPodFeed: attachPodFeed,
    attachOperatorFeed: attachOperatorFeed,
    setOperatorPods: setOperatorPods,
    loadOperatorPods: loadOperatorPods,
    refresh: refresh,
    revalidate: revalidate,
    loadLists: loadLists,
    /** Promise of the most recent refresh (or a resolved promise). */
    settled: function () { return inflight || Promise.resolve(); },
    /** True once a CRD/pod fetch has committed at least once. */
    hasLoaded: function () { return s.asyncLoaded; },
    /**
     * Work counters: cluster-index rebuilds vs delta patches, and the list
     * trackers' classification counts (objects classified / reused / skipped),
     * and the views subscribed right now.
     */
    counters: function () {
      return Object.assign({}, counters, {
        pods: podTracker.stats(), nodes: nodeTracker.stats(), subscribers: listeners.length,
        podFeeds: podFeeds, operatorFeeds: opFeeds,
        selectorIgnored: ignored.nodePods || ignored.operatorPods ? Object.assign({}, ignored) : null,
      });
    },
    /** A pod list feed is mounted right now: the store's pod list is being kept current. */
    podFeedMounted: function () { return podFeeds > 0; },
    noteSelectorIgnored: noteSelectorIgnored,
    /** True once a scoped list of `kind` ('nodePods' | 'operatorPods') came back unscoped. */
    selectorsIgnored: function (kind) { return ignored[kind] > 0; },
  };
}

// ---------------------------------------------------------------------------
// Shared stores (one per cluster) — survive route switches and detail views.
// ---------------------------------------------------------------------------

const shared = {};

/**
 * @param {string} key  cluster name
 * @param {() => ReturnType<typeof createClusterStore>} factory
 */
export function getSharedStore(key, factory) {
  const k = key || '__default__';
  if (!shared[k]) shared[k] = factory();
  return shared[k];
}

/** Every shared store alive (diagnostics and lifecycle specs). */
export function sharedStores() {
  return Object.keys(shared).map(function (k) { return shared[k]; });
}

export function resetSharedStores() {
  for (const k in shared) delete shared[k];
}

/**
 * True while a mounted pod feed keeps the store's pod list current and that
 * list is in: a Node detail section can then read the store. A list fed once
 * and no longer watched (every plugin page unmounted, as when the user went
 * to Headlamp's own Node page) is a seed, not a live source.
 */
export function storeIsLive(store) {
  if (!store || !store.podFeedMounted()) return false;
  return store.getSnapshot().podsState === 'ready';
}
