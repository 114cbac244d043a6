/**
 * GPU Nodes page view-model (reference src/components/NodesPage.tsx:145-293,
 * SURVEY C7): summary table and per-node cards with the per-GPU allocation
 * strip and the xGMI neighbour matrix, one page of nodes at a time, and what
 * that page asks Prometheus for (telemetryScope).
 */

import { nodeFacts } from '../../api/clusterIndex.js';
import { nodePowerKeys, nodeTempKeys, nonEmptyMap, ownersByNode } from '../../api/nodeSummaries.js';
import { MI355X } from '../../api/k8sCore.js';
import { SMALL_CLUSTER_NODES } from '../../api/series.js';
import { buildGpuSlots, buildXgmiMatrix, linkFacts } from '../../api/topology.js';
import { bar, kv, loader, page, pager, row, section, status, table } from '../ir.js';
import {
  ageText,
  allocationBar,
  BRAND,
  chunkedRows,
  errorSection,
  memo,
  NO_PODS,
  nodeSummaryRows,
  nowOf,
  podName,
  refreshButton,
  nodesPending,
  PODS_LOADING,
  podsPending,
} from './common.js';
import { nodeNameOf, nodePage, NODES_PER_PAGE, nodeSortOf, RANKED_NODE_SORTS, rankedPage } from './paging.js';

/** Names of the GPU nodes a paged view shows ([] while the node list is loading). */
export function visibleNodeNames(ctx, state) {
  if (!ctx || nodesPending(ctx) || !ctx.gpuNodes) return [];
  return nodePage(ctx.gpuNodes, state, ctx.index).names;
}

/**
 * What a paged page asks Prometheus for:
 *   * while the node list is loading, and while every GPU node fits on one
 *     page: `small` — the whole cluster if it has at most SMALL_CLUSTER_NODES
 *     GPU nodes, else the page's nodes, decided by Prometheus in the same request
 *     (metrics.js smallClusterQuery). A small cluster's page thus needs no
 *     second wave after the node list, and keeps one query key (no refetch)
 *     when the list arrives;
 *   * the names on the page once a larger cluster is listed;
 *   * cluster-wide (`scope` undefined) when the node list failed (e.g. RBAC
 *     denies listing nodes), so telemetry still shows;
 *   * with `ranked` (Metrics) and the power order: `rank`, the page Prometheus
 *     is to pick (metrics.js rankedClusterQuery).
 * @returns {{enabled: boolean, scope?: (string[]|undefined), small?: boolean,
 *            rank?: {by: string, page: number, per: number, filter: string}}}
 */
export function telemetryScope(ctx, state, ranked) {
  if (!ctx) return { enabled: false, scope: [] };
  // Power order (Metrics): Prometheus picks the page — no node list needed.
  if (ranked && nodeSortOf(state, RANKED_NODE_SORTS) === 'power') {
    const st = state || {};
    return {
      enabled: true,
      rank: { by: 'power', page: Math.max(0, Math.floor(st.page) || 0), per: NODES_PER_PAGE, filter: (st.filter || '').trim().toLowerCase() },
    };
  }
  // The node list alone decides the page (the pod list of a large cluster
  // arrives later: tens of MB against the node list's few).
  const nodes = ctx.nodesState;
  if (nodes === 'error') return { enabled: true, scope: undefined };
  if (nodes !== 'ready' && nodesPending(ctx)) return { enabled: true, scope: [], small: true };
  if (ctx.error && (!ctx.gpuNodes || ctx.gpuNodes.length === 0)) return { enabled: true, scope: undefined };
  const names = nodePage(ctx.gpuNodes, state, ctx.index).names;
  return ctx.gpuNodes.length <= SMALL_CLUSTER_NODES ? { enabled: true, scope: names, small: true } : { enabled: true, scope: names };
}

/** Per-GPU allocation strip block. */
export function slotsBlock(node, podsOnNode, owners) {
  const s = buildGpuSlots(node, podsOnNode, owners, nodeFacts(node));
  return { t: 'slots', slots: s.slots, exact: s.exact, partitionsPerGpu: s.partitionsPerGpu };
}

/**
 * xGMI neighbour matrix block; `measuredTopology` when link hops came from
 * the exporter. `open` (default true): the renderers draw the 8 × 8 grid;
 * false: its one-line summary, the grid one click away (a GPU Nodes card:
 * eight grids per page would be most of the page's elements).
 */
export function matrixBlock(gpuCount, measured, probed, open) {
  const n = gpuCount > 0 ? gpuCount : 0;
  // The caption and summary come from the link maps, in one pass; the 8 × 8
  // grid of cells is built on first read (a closed card never reads it).
  return new MatrixBlock(n, measured && typeof measured === 'object' ? measured : null, nonEmptyMap(probed) ? probed : null,
    open === undefined ? true : !!open);
}

/**
 * An xGMI matrix block (IR `matrix`): `fullMesh`, `linksPerGpu`,
 * `ringBusGBs` and the throughput statistics (`linkStats` over throughput
 * placed on links, `gpuStats` over per-GPU totals) read from the maps
 * (topology.js linkFacts, cached on them), as buildXgmiMatrix + isFullMesh
 * would say; `matrix`, the grid itself, built when first read. toJSON gives
 * the plain IR shape (the grid built, the link maps left out), so the JSON
 * a consumer reads (`amd-gpu-dash --json`) renders like the block.
 */
function MatrixBlock(n, measured, probed, open) {
  const f = linkFacts(n, measured, probed);
  this.t = 'matrix';
  this.fullMesh = f.fullMesh;
  // Link types / hops come from the exporter's gpu_xgmi_link_hops (this
  // repo's amdgpu-exporter); without them the matrix is the MI355X
  // platform model. Throughput (stock exporter xgmi_neighbor_*_tx_throughput)
  // sits on a link only where a series pins its peer (topology.js
  // placeThroughput); otherwise only each GPU's total is measured.
  this.measuredTopology = !!probed;
  this.measuredThroughput = !!f.stats;
  this.throughputPerGpu = !!f.gpuStats;
  this.open = open;
  this.size = n;
  this.linksPerGpu = f.linksPerGpu;
  this.linkGBs = MI355X.xgmiLinkGBs;
  this.ringBusGBs = f.linksPerGpu > 0 ? MI355X.xgmiLinkGBs : 0;
  this.linkStats = f.stats;
  this.gpuStats = f.gpuStats;
  this.measured = f.stats || f.gpuStats ? measured : null;
  this.probed = probed;
  this.grid = null;
}

Object.defineProperty(MatrixBlock.prototype, 'matrix', {
  get: function () {
    return this.grid || (this.grid = buildXgmiMatrix(this.size, this.measured || undefined, this.probed || undefined));
  },
});

MatrixBlock.prototype.toJSON = function () {
  return {
    t: 'matrix', matrix: this.matrix, fullMesh: this.fullMesh, measuredTopology: this.measuredTopology,
    measuredThroughput: this.measuredThroughput, throughputPerGpu: this.throughputPerGpu, open: this.open, size: this.size,
    linksPerGpu: this.linksPerGpu, linkGBs: this.linkGBs, ringBusGBs: this.ringBusGBs, linkStats: this.linkStats,
    gpuStats: this.gpuStats,
  };
};

const READY_CELLS = {};

/**
 * Readiness as `kubectl get nodes` words it: "Ready", "Not Ready", and
 * ", SchedulingDisabled" on a cordoned node (spec.unschedulable) — whose free
 * GPUs new pods cannot use, hence a warning (clusterIndex.js nodeFacts). One
 * cell per wording.
 */
export function nodeReadyCell(node) {
  const f = nodeFacts(node);
  return READY_CELLS[f.readyText] || (READY_CELLS[f.readyText] = status(f.readyLevel, f.readyText));
}

/** "key=value:Effect" per taint (clusterIndex.js taintsText, cached per node object). */
export function formatTaints(node) {
  return nodeFacts(node).taints;
}

function nodeCardRows(node, podsOnNode, now, podsPend) {
  // Everything but the pods was derived when the node list arrived
  // (clusterIndex.js nodeFacts `card`), not on this render.
  const card = nodeFacts(node).card;
  return card.before.concat(
    [row('GPU Workload Pods', podsPend ? PODS_LOADING : podsOnNode.length > 0 ? podsOnNode.map(podName).join(', ') : '—')],
    card.after
  );
}

/**
 * Differences: Allocation = GPUs held / allocatable GPUs (reference used the
 * pod count, quirk Q2); each node card adds HBM, the per-GPU allocation
 * strip and the xGMI neighbour matrix. `metrics` (optional) supplies exact
 * per-GPU owners and measured xGMI throughput. The page renders from the
 * node list: while the pod list is still loading, the cells that need pods
 * (allocation, GPU pods, workload pods, the inferred slot strip) say so and
 * fill in when it arrives (reference: a full-page Loader until every list is
 * in, NodesPage.tsx:148-150).
 */
export function nodesView(ctx, opts) {
  const now = nowOf(opts);
  const metrics = opts && opts.metrics ? opts.metrics : null;
  if (nodesPending(ctx)) return page(null, null, [loader('Loading GPU node data...')]);
  const podsPend = podsPending(ctx);
  // One page of nodes (NODES_PER_PAGE, name filter): the summary rows, the
  // cards and the telemetry the page asks for are all O(page), not O(cluster).
  // In power order Prometheus picked the page (metrics.js rankedSnapshot).
  const pagerState = opts && opts.pager;
  const sort = nodeSortOf(pagerState, RANKED_NODE_SORTS);
  const pg = metrics && metrics.rank && sort === 'power' ? rankedNodePage(ctx, metrics, pagerState)
    : nodePage(ctx.gpuNodes, pagerState, ctx.index);
  // Live node power (the GPU Nodes query carries the power gauge for pod
  // attribution anyway): "watts|cap" per node, whole watts, so the head and
  // its rows rebuild only when a shown value changes.
  const power = nodePowerKeys(metrics);
  const temps = nodeTempKeys(metrics);
  const head = memo('nodes-head', [pg, ctx.index, ctx.error, power.sig, temps.sig, podsPend], function () {
    return nodesHeadItems(ctx, now, power, pg, sort, podsPend, temps);
  }, now);
  const owners = ownersByNode(metrics);
  const xgmi = metrics ? metrics.xgmi : undefined;
  const links = metrics ? metrics.links : undefined;
  // The card list as a whole holds while no input changed (most watch events
  // touch no GPU node or pod); otherwise only changed cards are rebuilt.
  const items = memo('nodes-cards', [head, pg, ctx.index, owners, xgmi, links, podsPend], function () {
    const idx = ctx.index;
    function inputs(n) {
      const name = n.metadata.name;
      return [idx.podsByNode.get(name) || NO_PODS, idx.nodeStats.get(name), owners[name],
        xgmi ? xgmi[name] : undefined, links ? links[name] : undefined];
    }
    const cards = chunkedRows('node-cards', pg.nodes, [], function (n) {
      const name = n.metadata.name;
      const d = inputs(n);
      const pods = d[0];
      const own = d[2];
      const xg = d[3];
      const lk = d[4];
      // own / xg / lk keep their identity while their content is unchanged
      // (ownersByNode + the metrics client's structural sharing).
      return memo('node-card:' + name, [n, pods, own, xg, lk, podsPend], function () {
        const blocks = [kv(nodeCardRows(n, pods, now, podsPend))];
        const facts = nodeFacts(n);
        if (facts.capacity > 0) {
          // Without the pods the strip is exact only from exporter owners.
          if (!podsPend || own) blocks.push(slotsBlock(n, podsPend ? NO_PODS : pods, own));
          const phys = facts.physicalGpus;
          if (phys > 1) blocks.push(matrixBlock(phys, xg, lk, false)); // no xGMI peers on a single-GPU node
        }
        return section(name, blocks, n.metadata.uid || name);
      }, now);
    }, now, inputs);
    return head.concat(cards);
  }, now);
  return page(BRAND + ' — Nodes', refreshButton('Refresh node data', !!(opts && opts.fetching)), items);
}

// ownersByNode, nodePowerKeys, nodeTempKeys: per-node summaries of a
// telemetry snapshot, derived when it arrives (api/nodeSummaries.js).
export { nodePowerKeys, nodeTempKeys, ownersByNode };

/** The Hottest GPU cell from its snapshot facts (nodeSummaries.js nodeTempKeys): a status when warm or throttling. */
function nodeTempCell(c) {
  if (!c) return '—';
  return c.level === 'ok' ? c.text : status(c.level, c.text);
}

/** The Power cell from its snapshot facts (nodeSummaries.js nodePowerKeys). */
function nodePowerCell(b) {
  return b ? bar(b.watts, b.cap, b.pct, b.color, b.text) : '—';
}

function nodesHeadItems(ctx, now, power, pg, sort, podsPend, temps) {
  const pw = power.byNode;
  const withPower = power.sig !== '';
  const tp = temps.byNode;
  const withTemp = temps.sig !== '';
  const items = [];
  if (ctx.error) items.push(errorSection(ctx.error));

  if (ctx.gpuNodes.length === 0) {
    items.push(
      section('No GPU Nodes Found', [
        kv([
          row('Status', status('warning', 'No nodes with AMD GPU resources or labels were found')),
          row(
            'Note',
            'Nodes appear here when they advertise amd.com/gpu or carry AMD node-feature-discovery / node-labeller labels. ' +
              'Ensure the AMD GPU Operator (or the AMD k8s device plugin) and Node Feature Discovery are installed.'
          ),
        ]),
      ])
    );
    return items;
  }

  items.push(pager(pg, pg.ranked ? 'GPU nodes reporting' : 'GPU nodes', { sort: sort, sorts: RANKED_NODE_SORTS, label: 'GPU nodes' }));
  const idx = ctx.index;
  if (pg.nodes.length > 0) {
    items.push(
      section('GPU Node Summary', [
        table(
          // "Power" and "Hottest GPU" (beyond the reference): the node's GPUs'
          // live power against their summed cap; its hottest junction temperature.
          ['Node', 'Ready', 'GPU Model', 'GPU Devices', 'Allocation', 'GPU Pods'].concat(withPower ? ['Power'] : [],
            withTemp ? ['Hottest GPU'] : [], ['Age']),
          chunkedRows('node-summary-rows', pg.nodes, [withPower, withTemp, podsPend], function (n) {
            const st = idx.nodeStats.get(n.metadata.name);
            const pk = pw[n.metadata.name];
            const tk = tp[n.metadata.name];
            // Per-node stats keep their identity while unchanged (buildClusterIndex).
            return nodeSummaryRows(n, [st, withPower, pk, withTemp, tk, podsPend], function () {
              const f = nodeFacts(n);
              const count = f.capacity;
              return [
                n.metadata.name,
                nodeReadyCell(n),
                f.modelText,
                count > 0 ? String(count) : '—',
                podsPend ? PODS_LOADING : allocationBar(st ? st.inUse : 0, (st && st.allocatable) || count),
                podsPend ? PODS_LOADING : String(st ? st.pods : 0),
              ].concat(withPower ? [nodePowerCell(power.bars[n.metadata.name])] : [], withTemp ? [nodeTempCell(temps.cells[n.metadata.name])] : [],
                [ageText(n.metadata.creationTimestamp, now)]);
            }, now);
          }, now, function (n) { return [idx.nodeStats.get(n.metadata.name), withPower, pw[n.metadata.name], tp[n.metadata.name]]; }),
          pg.nodes.map(function (n) { return n.metadata.uid || n.metadata.name; })
        ),
      ])
    );
  }

  return items;
}

/**
 * GPU Nodes in power order: the ranked page's names (metrics.rank) as the
 * listed node objects; a ranked hostname that is no listed node is left out.
 */
function rankedNodePage(ctx, m, state) {
  const byName = memo('nodes-by-name', [ctx.gpuNodes], function () {
    const out = new Map();
    for (let i = 0; i < ctx.gpuNodes.length; i++) out.set(ctx.gpuNodes[i].metadata.name, ctx.gpuNodes[i]);
    return out;
  });
  return memo('nodes-ranked-page', [m, byName], function () {
    const base = rankedPage(m, state);
    const nodes = [];
    for (let i = 0; i < base.names.length; i++) if (byName.has(base.names[i])) nodes.push(byName.get(base.names[i]));
    return Object.assign({}, base, { nodes: nodes, names: nodes.map(nodeNameOf), ranked: true });
  });
}
