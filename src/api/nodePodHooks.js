/**
 * The pods of ONE node for the native Node detail section (C10), as hooks
 * over the injected React and Headlamp library (providerCore.js builds them
 * with its store and settings). The reference mounts a whole provider there
 * — the cluster-wide Pod list + watch (src/index.tsx:152-160,
 * IntelGpuDataContext.tsx:98-99) — on every detail page; here a section that
 * no plugin page feeds reads its own node's pods only (ADR 011, ADR 012).
 */

import { fetchNodePods, nodePodsSelector, storeIsLive } from './clusterStore.js';
import { filterGpuRequestingPods } from './amdPods.js';
import { get, unwrapAll } from './k8sCore.js';
import { countOutside } from './selectors.js';
import { createPoller } from './settings.js';

/** Raw pods of `items` (list-hook items or raw objects) bound to `nodeName`. */
function onNode(items, nodeName) {
  return unwrapAll(items).filter(function (p) { return get(p, ['spec', 'nodeName'], null) === nodeName; });
}

/** The GPU pods of `nodeName` in the store's last pod list (any age), or null when it holds none. */
function seedPods(store, nodeName) {
  const snap = store.getSnapshot();
  if (snap.podsState !== 'ready') return null;
  const byNode = snap.index && snap.index.podsByNode ? snap.index.podsByNode.get(nodeName) : undefined;
  return byNode || snap.gpuPods.filter(function (p) { return get(p, ['spec', 'nodeName'], null) === nodeName; });
}

/**
 * @param {any} React  React 18 (or the harness stand-in)
 * @param {{K8s: any}} lib  '@kinvolk/headlamp-plugin/lib'
 * @param {{storeFor: (cluster: string) => any, clusterKey: () => string,
 *          request: (path: string) => Promise<any>, loadSettings: () => any,
 *          scopedPollSec: () => number, useListOf: (cls: any, opts?: any) => [any, any],
 *          errorText: (e: any) => string}} env
 */
export function createNodePodHooks(React, lib, env) {
  const h = React.createElement;
  const useEffect = React.useEffect;
  const useMemo = React.useMemo;
  const errorText = env.errorText;

  /**
   * True while a mounted pod feed keeps the cluster's shared store current
   * (clusterStore.js storeIsLive: a plugin page that draws pods is mounted
   * next to the caller). A Node detail section then reads the store;
   * otherwise it reads its own node's pods (useNodePods) and never mounts a
   * cluster-wide watch. Re-renders the caller when that flips (the page
   * unmounts, or its list arrives).
   */
  function usePodsLive() {
    const store = env.storeFor(env.clusterKey());
    return React.useSyncExternalStore(store.subscribe, function () { return storeIsLive(store); });
  }

  /**
   * One node's pods by the host's list + watch hook SCOPED to the node
   * (`fieldSelector spec.nodeName=<node>`, all namespaces), delivered to
   * `props.onList(node, pods | null, error | null)`. The pods are filtered by
   * node here too; objects of other nodes mean the host ignored the field
   * selector (store.noteSelectorIgnored), and useNodePods swaps this feed for
   * NodePodsPoll.
   */
  function NodePodsWatch(props) {
    const node = props.node;
    const opts = useMemo(function () { return { namespace: '', fieldSelector: nodePodsSelector(node) }; }, [node]);
    const res = env.useListOf(lib.K8s.ResourceClasses.Pod, opts);
    const items = res[0];
    const err = res[1];
    const got = useMemo(function () {
      if (!items) return { pods: null, outside: 0 };
      const raw = unwrapAll(items);
      return { pods: onNode(raw, node), outside: countOutside(raw, opts) };
    }, [items, node, opts]);
    useEffect(function () {
      if (got.outside > 0) props.store.noteSelectorIgnored('nodePods', got.outside, got);
      props.onList(node, got.pods, got.pods ? null : err ? errorText(err) : null);
    }, [got, err, node]);
    return null;
  }

  /**
   * One node's pods by the field-selected request (requests.js
   * fetchNodePods: the apiserver applies the selector as a query parameter),
   * re-read every scopedPollSec(): what a Node detail section reads on a host
   * that ignores useList() options, instead of the cluster-wide list such a
   * host would deliver.
   */
  function NodePodsPoll(props) {
    const node = props.node;
    const onList = props.onList;
    const period = env.scopedPollSec();
    useEffect(function () {
      let live = true;
      const timeoutMs = env.loadSettings().requestTimeoutMs;
      function read() {
        return fetchNodePods(env.request, node, timeoutMs).then(
          function (items) { if (live) onList(node, onNode(items, node), null); },
          function (e) { if (live) onList(node, null, errorText(e)); }
        );
      }
      read();
      const poller = createPoller(period);
      poller.start(read);
      return function () {
        live = false;
        poller.stop();
      };
    }, [node, period]);
    return null;
  }

  /**
   * The pods of one node for a Node detail section that no mounted page
   * feeds: a list + watch scoped to the node (NodePodsWatch), live like the
   * reference's section — a pod scheduled onto the node appears without a
   * reload — at O(pods on the node) instead of O(pods in the cluster); on a
   * host that ignores list options, the field-selected request re-read
   * (NodePodsPoll). The list request goes out in the same wave as the node's
   * telemetry and power history.
   *
   * Until the node's own list delivers, the store's last pod list (a plugin
   * page visited earlier, no longer watched) seeds the section, so it paints
   * at once; that list can be of any age, so the context says so
   * (`podsSeeded`) and the section marks its pods as being refreshed. A list
   * that stops answering after it delivered keeps the pods shown; only a
   * first failure says the pods are unreadable.
   *
   * Returns [the slice of the context nodeDetailView reads, the feed element
   * the caller renders].
   */
  function useNodePods(nodeName) {
    const store = env.storeFor(env.clusterKey());
    const ignored = React.useSyncExternalStore(store.subscribe, function () { return store.selectorsIgnored('nodePods'); });
    const seed = useMemo(function () { return seedPods(store, nodeName); }, [store, nodeName]);
    const st = React.useState(null);
    const got = st[0];
    const setGot = st[1];
    const onList = useMemo(function () {
      return function (node, pods, error) {
        setGot(function (prev) {
          const same = prev && prev.node === node;
          if (pods) return { node: node, pods: pods, error: null };
          // A re-list or a failure after a delivery keeps what is shown.
          if (same && prev.pods) return prev;
          return error ? { node: node, pods: null, error: error } : same ? prev : null;
        });
      };
    }, []);
    const cur = got && got.node === nodeName ? got : null;
    const own = cur && cur.pods ? cur.pods : null;
    const pods = own || (cur && cur.error ? null : seed);
    const ctx = useMemo(function () {
      if (pods) return { loading: false, gpuPods: filterGpuRequestingPods(pods), podsState: 'ready', error: null, podsSeeded: !own };
      if (cur && cur.error) return { loading: false, gpuPods: [], podsState: 'error', error: cur.error };
      return { loading: true, gpuPods: [], podsState: 'pending', error: null };
    }, [pods, cur && cur.error]);
    const feed = h(ignored ? NodePodsPoll : NodePodsWatch, { node: nodeName, onList: onList, store: store });
    return [ctx, feed];
  }

  return { usePodsLive: usePodsLive, useNodePods: useNodePods };
}
