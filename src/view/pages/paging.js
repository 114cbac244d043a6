/**
 * Paged lists (ADR 009): which slice of GPU nodes / pods a page shows, in
 * which order, with which filter. The reference renders every GPU node and
 * every GPU pod (src/components/NodesPage.tsx:285-291, PodsPage.tsx:201-236);
 * here a page holds NODES_PER_PAGE nodes or PODS_PER_PAGE pods and fetches
 * the telemetry of those only.
 */

import { isNodeReady } from '../../api/amdNodes.js';
import { podFacts } from '../../api/clusterIndex.js';
import { get } from '../../api/k8sCore.js';
import { memo, NO_PODS } from './common.js';

/** GPU nodes per page on the GPU Nodes and Metrics pages. */
export const NODES_PER_PAGE = 8;

export function nodeNameOf(n) {
  return typeof n === 'string' ? n : n.metadata.name;
}

/**
 * The slice of GPU nodes a paged view shows: `state` = {page, filter,
 * perPage} (page 0-based, clamped; filter a case-insensitive substring of the
 * node name). Memoised on the node list's identity, so the same state over
 * the same list returns the same object (and the same `nodes` array) — the
 * page's memos and the metrics hook's scope key stay put between refreshes.
 *
 * The reference renders one card per GPU node with no cap (NodesPage.tsx:
 * 285-291; its Metrics page one card per chip, MetricsPage.tsx:348-350): at
 * 1,000 nodes that is thousands of cards and every node's telemetry per
 * refresh. Here a page holds NODES_PER_PAGE nodes and fetches their
 * telemetry only.
 * @returns {{nodes: any[], names: string[], page: number, pages: number, from: number, to: number,
 *            total: number, matched: number, filter: string, perPage: number}}
 */
export function nodePage(gpuNodes, state, index) {
  const sort = nodeSortOf(state);
  if (sort === 'name' || !gpuNodes) return listPage('node', gpuNodes, state, nodeNameOf, nodeNameOf, NODES_PER_PAGE);
  // Another order: the list sorted once per node list and cluster index
  // (allocations move with pod churn), then paged like the name order.
  const sorted = memo('node-sort:' + sort, [gpuNodes, index], function () {
    return gpuNodes.slice().sort(nodeComparator(sort, index));
  });
  return listPage('node-' + sort, sorted, state, nodeNameOf, nodeNameOf, NODES_PER_PAGE);
}

/**
 * Orders a paged node view offers (pager `sort`): at 1,000 nodes a page of
 * eight in name order does not show where the free GPUs or the broken nodes
 * are, so the list can be ranked by the allocation the cluster index already
 * holds (no request). Ties keep name order.
 */
export const NODE_SORTS = Object.freeze([
  Object.freeze({ value: 'name', label: 'Name' }),
  Object.freeze({ value: 'in-use', label: 'Most GPUs in use' }),
  Object.freeze({ value: 'free', label: 'Most GPUs free' }),
  Object.freeze({ value: 'attention', label: 'Not ready first' }),
]);

/**
 * GPU Nodes and Metrics add an order only Prometheus knows: total GPU power,
 * highest first. Prometheus ranks and returns that page's nodes in one
 * request (metrics.js rankedClusterQuery); nodes without telemetry are not
 * ranked.
 */
export const RANKED_NODE_SORTS = Object.freeze(NODE_SORTS.concat([Object.freeze({ value: 'power', label: 'Highest GPU power' })]));

/** The pager state's sort if it is one of `sorts` (default NODE_SORTS), else 'name'. */
export function nodeSortOf(state, sorts) {
  const want = state && state.sort;
  const list = sorts || NODE_SORTS;
  for (let i = 0; i < list.length; i++) if (list[i].value === want) return want;
  return 'name';
}

function nodeComparator(sort, index) {
  function stats(n) {
    return index && index.nodeStats ? index.nodeStats.get(nodeNameOf(n)) : undefined;
  }
  function inUse(n) {
    const st = stats(n);
    return st ? st.inUse || 0 : 0;
  }
  function free(n) {
    const st = stats(n);
    return st ? Math.max(0, (st.allocatable || 0) - (st.inUse || 0)) : 0;
  }
  function attention(n) {
    if (typeof n === 'string') return 0;
    if (!isNodeReady(n)) return 2;
    return get(n, ['spec', 'unschedulable'], false) ? 1 : 0;
  }
  const rank = sort === 'in-use' ? inUse : sort === 'free' ? free : attention;
  return function (a, b) {
    const d = rank(b) - rank(a);
    if (d) return d;
    const x = nodeNameOf(a);
    const y = nodeNameOf(b);
    return x < y ? -1 : x > y ? 1 : 0;
  };
}

/** GPU pods per page on the GPU Pods page (and operator pods on Device Plugins). */
export const PODS_PER_PAGE = 25;

export function podKeyOf(p) {
  return (p.metadata.namespace || '') + '/' + p.metadata.name;
}

function podSearchText(p) {
  return podKeyOf(p) + ' ' + get(p, ['spec', 'nodeName'], '');
}

/**
 * The slice of pods a paged table shows (nodePage for pods): the filter is
 * a case-insensitive substring of "namespace/name node". `names` are
 * "namespace/name" keys; `nodes` holds the pod objects.
 */
export function podPage(pods, state, kind) {
  const k = kind || 'pod';
  const sort = k === 'pod' ? podSortOf(state) : 'name';
  if (sort === 'name' || !pods) return listPage(k, pods, state, podKeyOf, podSearchText, PODS_PER_PAGE);
  const sorted = memo('pod-sort:' + sort, [pods], function () { return pods.slice().sort(podComparator(sort)); });
  return listPage(k + '-' + sort, sorted, state, podKeyOf, podSearchText, PODS_PER_PAGE);
}

/**
 * Orders of the GPU Pods table (pager `sort`), from the pod objects alone:
 * namespace / name (the list order), most GPUs held first, newest first,
 * and not running first (pending / failed before running). Ties keep
 * namespace / name order.
 */
export const POD_SORTS = Object.freeze([
  Object.freeze({ value: 'name', label: 'Namespace / name' }),
  Object.freeze({ value: 'gpus', label: 'Most GPUs held' }),
  Object.freeze({ value: 'newest', label: 'Newest first' }),
  Object.freeze({ value: 'attention', label: 'Not running first' }),
]);

/**
 * The GPU Pods table's orders: POD_SORTS plus the power of the GPUs each pod
 * holds, ranked by Prometheus (metrics.js rankedOwnersQuery) from the
 * exporter's pod labels, so one page is asked for whatever the cluster.
 */
export const RANKED_POD_SORTS = Object.freeze(POD_SORTS.concat([Object.freeze({ value: 'power', label: 'Highest GPU power' })]));

/** The pager state's sort if it is one of `sorts` (default POD_SORTS), else 'name'. */
export function podSortOf(state, sorts) {
  const want = state && state.sort;
  const list = sorts || POD_SORTS;
  for (let i = 0; i < list.length; i++) if (list[i].value === want) return want;
  return 'name';
}

function podComparator(sort) {
  function created(p) {
    const t = Date.parse(get(p, ['metadata', 'creationTimestamp'], ''));
    return isNaN(t) ? 0 : t;
  }
  function notRunning(p) {
    const ph = podFacts(p).phase;
    return ph === 'Running' || ph === 'Succeeded' ? 0 : 1;
  }
  const rank = sort === 'gpus' ? function (p) { return podFacts(p).gpus; } : sort === 'newest' ? created : notRunning;
  return function (a, b) {
    const d = rank(b) - rank(a);
    if (d) return d;
    const x = podKeyOf(a);
    const y = podKeyOf(b);
    return x < y ? -1 : x > y ? 1 : 0;
  };
}

/**
 * Slice `all` for a pager `state` ({page, filter, perPage}); memoised per
 * kind + state on the list's identity.
 */
function listPage(kind, all0, state, keyOf, textOf, perDefault) {
  const st = state || {};
  const per = st.perPage > 0 ? Math.min(Math.floor(st.perPage), 200) : perDefault;
  // The raw text is kept for the input box; matching ignores surrounding spaces.
  const filter = typeof st.filter === 'string' ? st.filter : '';
  const all = all0 || NO_PODS;
  const want = Math.max(0, Math.floor(st.page) || 0);
  return memo(kind + '-page:' + per + '|' + want + '|' + filter, [all], function () {
    const f = filter.trim().toLowerCase();
    const list = f ? all.filter(function (n) { return textOf(n).toLowerCase().indexOf(f) >= 0; }) : all;
    const pages = Math.max(1, Math.ceil(list.length / per));
    const pg = Math.min(want, pages - 1);
    const from = pg * per;
    const to = Math.min(list.length, from + per);
    const items = list.slice(from, to);
    return {
      nodes: items, names: items.map(keyOf), page: pg, pages: pages, from: from, to: to,
      total: all.length, matched: list.length, filter: filter, perPage: per,
    };
  });
}

/** The pager page of a power-ranked answer: its nodes, in rank order, out of the nodes ranked. */
export function rankedPage(m, state) {
  return memo('metrics-ranked-page', [m], function () {
    return Object.assign(rankedSlice(m.rank, m.scope.length, state), { nodes: m.scope, names: m.scope });
  });
}

/**
 * Pager fields of a ranked answer holding `shown` items of page `r.page`
 * (`r.count` ranked in all). An answer past the last page (the ranked count
 * shrank while the user was on a later page) is flagged `beyond`, with the
 * last page's numbers; the page component then moves to the last page
 * (plugin.js useRankedPageClamp).
 */
export function rankedSlice(r, shown, state) {
  const count = shown ? Math.max(r.count, r.page * r.per + shown) : r.count;
  const pages = Math.max(1, Math.ceil(count / r.per));
  const beyond = !shown && r.page > pages - 1;
  const page = beyond ? pages - 1 : r.page;
  const from = Math.min(page * r.per, count);
  return {
    page: page, pages: pages, from: from, to: beyond ? from : from + shown, total: count, matched: count,
    filter: (state && state.filter) || '', perPage: r.per, beyond: beyond,
  };
}
