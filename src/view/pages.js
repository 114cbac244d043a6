/**
 * Page view-models: snapshot → View IR. Pure functions, no React, no I/O.
 *
 * One function per reference page / integration (SURVEY.md C5–C12):
 *   overviewView        ← src/components/OverviewPage.tsx
 *   devicePluginsView   ← src/components/DevicePluginsPage.tsx
 *   nodesView           ← src/components/NodesPage.tsx
 *   podsView            ← src/components/PodsPage.tsx
 *   metricsView         ← src/components/MetricsPage.tsx
 *   nodeDetailView      ← src/components/NodeDetailSection.tsx
 *   podDetailView       ← src/components/PodDetailSection.tsx
 *   nodeColumns         ← src/components/integrations/NodeColumns.tsx
 *
 * Section titles, loader texts, empty states and refresh aria-labels keep
 * the reference's wording with AMD vocabulary, so the reference's component
 * assertions translate one-for-one. Behavioural differences are listed in
 * each function's comment.
 *
 * `opts.now` (ms epoch) makes ages deterministic in tests.
 */

import {
  AMD_GPU_OPERATOR_NAMESPACE,
  AMD_GPU_RESOURCE,
  BAR_COLORS,
  MI355X,
  OPERANDS,
  containerGpuEntries,
  countsToStatus,
  countsToText,
  deviceConfigStatus,
  deviceConfigStatusText,
  formatAge,
  nextAgeChange,
  podFacts,
  formatBytes,
  formatComponent,
  formatGpuModel,
  formatGpuResourceName,
  formatPercent,
  formatPodGpuRequests,
  formatSelector,
  formatWatts,
  get,
  getGpuResources,
  getNodeGpuCount,
  getNodeGpuModel,
  getNodePhysicalGpuCount,
  getPodGpuCount,
  getPodGpuDemand,
  getPodRestarts,
  gpuContainers,
  gpuInitContainers,
  isAmdGpuNode,
  isGpuRequestingPod,
  isNodeReady,
  isPodReady,
  labellerValue,
  operandEnabled,
  operandStatus,
  pct,
  pctToColor,
  pctToStatus,
  phaseToStatus,
  pluginPodComponent,
  podPhase,
  podWaitingMessage,
  podWaitingReason,
  unwrapKubeObject,
} from '../api/amdgpu.js';
import { buildGpuSlots, buildXgmiMatrix, isFullMesh } from '../api/topology.js';
import { PROMETHEUS_SERVICES, SMALL_CLUSTER_NODES, SMALL_CLUSTER_PODS, clusterPowerStats, summarizeMetrics } from '../api/metrics.js';
import { bar, createMemo, createObjectCache, kv, lines, loader, noteExpiry, page, pager, pctbar, row, section, status, table } from './ir.js';

export const BRAND = 'AMD GPU';

/**
 * Section-level memo shared by all views. Deps are the snapshot fields a
 * section reads plus the age clock (ages are shown with 1 s resolution), so a
 * refresh that returns unchanged Kubernetes objects reuses the section IR.
 */
// One slot per section: node cards, node details, metrics nodes and pod details
// of a few hundred nodes / thousands of pods fit without LRU churn.
const memo = createMemo(8192);
// Table rows per Kubernetes object, one cache per table (pods, nodes): an
// event rebuilds the changed object's row only.
const ovPluginRows = createObjectCache();
const dpPluginRows = createObjectCache();
const nodeSummaryRows = createObjectCache();
const podRows = createObjectCache();
const pendingRows = createObjectCache();
const ROW_CACHES = [ovPluginRows, dpPluginRows, nodeSummaryRows, podRows, pendingRows];
const podDetailCache = typeof WeakMap === 'function' ? new WeakMap() : null;

/** Rows per memo slot in the large tables (see chunkedRows). */
const ROW_CHUNK = 64;

/**
 * `objs.map(build)` for a large table, memoised in chunks of ROW_CHUNK
 * objects keyed on their identities: after a watch event that replaced one
 * pod in a 5000-row table, 78 chunks are identity-compared and one is
 * rebuilt (its other rows come from `rowCacheOf`'s per-object cache).
 */
function chunkedRows(name, objs, deps, build, now, depsOf) {
  const out = [];
  for (let c = 0; c < objs.length; c += ROW_CHUNK) {
    const part = objs.slice(c, c + ROW_CHUNK);
    const key = part.concat(deps);
    // Per-object inputs besides the object itself (its stats, its pods).
    if (depsOf) {
      for (let i = 0; i < part.length; i++) {
        const d = depsOf(part[i]);
        for (let k = 0; k < d.length; k++) key.push(d[k]);
      }
    }
    const rows = memo(name + ':' + c / ROW_CHUNK, key, function () { return part.map(build); }, now);
    for (let i = 0; i < rows.length; i++) out.push(rows[i]);
  }
  return out;
}

/** `objs.filter(pred)` memoised in chunks the same way (pred depends on the object only). */
function chunkedFilter(name, objs, pred) {
  const out = [];
  for (let c = 0; c < objs.length; c += ROW_CHUNK) {
    const part = objs.slice(c, c + ROW_CHUNK);
    const kept = memo(name + ':' + c / ROW_CHUNK, part, function () { return part.filter(pred); });
    for (let i = 0; i < kept.length; i++) out.push(kept[i]);
  }
  return out;
}

/** formatAge, noting when the label changes (the enclosing memo holds until then). */
function ageText(timestamp, now) {
  noteExpiry(nextAgeChange(timestamp, now));
  return formatAge(timestamp, now);
}

/** Seconds → "30 min" / "1 h" / "6 h" / "90 s" for section titles. */
export function formatWindow(sec) {
  if (sec >= 3600 && sec % 3600 === 0) return sec / 3600 + ' h';
  if (sec >= 60 && sec % 60 === 0) return sec / 60 + ' min';
  return sec + ' s';
}

/** Drop memoised sections (tests; cluster switch). */
export function clearViewMemo() {
  memo.clear();
  for (let i = 0; i < ROW_CACHES.length; i++) ROW_CACHES[i].clear();
}
export const ACTIVE_PODS_LIMIT = 10;

export const HELM_INSTALL =
  'helm repo add rocm https://rocm.github.io/gpu-operator && ' +
  'helm install amd-gpu-operator rocm/gpu-operator-charts --namespace ' + AMD_GPU_OPERATOR_NAMESPACE + ' --create-namespace';
export const OPERATOR_DOCS = 'https://instinct.docs.amd.com/projects/gpu-operator/';

function nowOf(opts) {
  return opts && typeof opts.now === 'number' ? opts.now : Date.now();
}

function refreshButton(ariaLabel, busy) {
  return { label: busy ? 'Refreshing…' : 'Refresh', ariaLabel: ariaLabel, disabled: !!busy };
}

function errorSection(err) {
  return section('Error', [kv([row('Status', status('error', err))])]);
}

/** Inline allocation bar (reference NodesPage.tsx:35-63; 70/90 thresholds). */
export function allocationBar(used, allocatable) {
  if (!(allocatable > 0)) return '—';
  const p = Math.min(100, pct(used, allocatable));
  return bar(used, allocatable, p, pctToColor(p), used + '/' + allocatable + ' (' + p + '%)');
}

function podName(p) {
  return p.metadata.name;
}
function podNs(p) {
  return p.metadata.namespace || '—';
}
function podNode(p) {
  return get(p, ['spec', 'nodeName'], '—');
}

function readyLabel(p) {
  const r = isPodReady(p);
  return status(r ? 'success' : 'warning', r ? 'Ready' : get(p, ['status', 'phase'], 'Unknown'));
}

function restartsCell(p) {
  const n = getPodRestarts(p);
  return n > 0 ? status('warning', n) : String(n);
}

// ---------------------------------------------------------------------------
// Overview (reference OverviewPage.tsx:54-420)
// ---------------------------------------------------------------------------

/**
 * Differences: the loader only replaces the page on the FIRST load — later
 * refreshes keep the data (stale-while-revalidate). Aggregates come from
 * the store's memoised index. In-use counts GPUs held by bound,
 * non-terminated pods (the scheduler's view), and Free is clamped at 0.
 */
export function overviewView(ctx, opts) {
  const now = nowOf(opts);
  if (ctx.loading) return page(null, null, [loader('Loading ' + BRAND + ' data...')]);
  const items = memo(
    'overview',
    [ctx.deviceConfigs, ctx.pluginPods, ctx.pluginInstalled, ctx.crdAvailable, ctx.gpuNodes, ctx.gpuPods, ctx.index, ctx.error],
    function () { return overviewItems(ctx, now); },
    now
  );
  return page(BRAND + ' — Overview', refreshButton('Refresh AMD GPU data', ctx.refreshing), items);
}

const MODE_COLORS = ['#ed1c24', '#f06b6f', '#7a0c10', '#ff9e80', '#9e9e9e'];

/** PercentageBar data: nodes per compute/memory partition mode ("SPX/NPS1" when unlabelled). */
export function partitionModeDistribution(gpuNodes) {
  const counts = {};
  const order = [];
  for (let i = 0; i < gpuNodes.length; i++) {
    const m = getNodeGpuModel(gpuNodes[i]);
    const k = (m.computePartition || 'SPX') + '/' + (m.memoryPartition || 'NPS1');
    if (!(k in counts)) {
      counts[k] = 0;
      order.push(k);
    }
    counts[k]++;
  }
  return order.map(function (k, i) { return { name: k, value: counts[k], fill: MODE_COLORS[i % MODE_COLORS.length] }; });
}

function overviewItems(ctx, now) {
  const items = [];
  const t = ctx.index.totals;

  if (ctx.error) items.push(errorSection(ctx.error));

  if (!ctx.pluginInstalled) {
    items.push(
      section('Plugin Not Detected', [
        kv([
          row('Status', status('warning', 'AMD GPU device plugin not found on this cluster')),
          row('Install (Helm)', HELM_INSTALL),
          row('Documentation', OPERATOR_DOCS),
        ]),
      ])
    );
  }

  if (!ctx.crdAvailable && ctx.pluginInstalled) {
    items.push(
      section('Notice', [
        kv([
          row('CRD Status', status('warning', ctx.crdForbidden
            ? 'DeviceConfig list forbidden for this user (HTTP 403) — limited visibility available'
            : 'DeviceConfig CRD not found — limited visibility available')),
          row(
            'Note',
            'Device plugin pods detected via DaemonSet labels. Install the AMD GPU Operator for DeviceConfig-based management.'
          ),
        ]),
      ])
    );
  }

  if (ctx.crdAvailable && ctx.deviceConfigs.length > 0) {
    items.push(memo('overview-dc', [ctx.deviceConfigs], function () { return overviewDeviceConfigs(ctx.deviceConfigs, now); }, now));
  }

  if (ctx.pluginPods.length > 0) {
    items.push(memo('overview-plugin-pods', [ctx.pluginPods], function () { return overviewPluginPods(ctx.pluginPods, now); }, now));
  }

  items.push(memo('overview-nodes', [ctx.gpuNodes, t], function () { return overviewNodes(ctx.gpuNodes, t); }));
  if (t.capacity > 0) items.push(memo('overview-alloc', [t], function () { return overviewAllocation(t); }));
  const ph = ctx.index.phases;
  items.push(memo('overview-workloads', [ph, ctx.gpuPods.length], function () { return overviewWorkloads(ph, ctx.gpuPods.length); }));
  const active = memo('overview-active', [ctx.gpuPods], function () { return overviewActivePods(ctx.gpuPods, now); }, now);
  if (active) items.push(active);
  return items;
}

function overviewDeviceConfigs(dcs, now) {
  return section('Device Config Status', [
    table(
      ['Name', 'Namespace', 'Status', 'Metrics Exporter', 'Node Labeller', 'Selector', 'Age'],
      dcs.map(function (dc) {
        return [
          dc.metadata.name,
          dc.metadata.namespace || '—',
          status(deviceConfigStatus(dc), deviceConfigStatusText(dc)),
          operandEnabled(dc, 'metricsExporter') ? status('success', 'Enabled') : status('warning', 'Disabled'),
          operandEnabled(dc, 'nodeLabeller') ? status('success', 'Enabled') : status('warning', 'Disabled'),
          formatSelector(get(dc, ['spec', 'selector'], null)),
          ageText(dc.metadata.creationTimestamp, now),
        ];
      }),
      dcs.map(function (dc) { return dc.metadata.uid || dc.metadata.name; })
    ),
  ]);
}

/** Operator pods listed on the Overview (the Device Plugins page pages through all of them). */
export const OVERVIEW_PLUGIN_PODS = 10;

/**
 * Operator pods on the Overview: the not-ready ones first, at most
 * OVERVIEW_PLUGIN_PODS rows, with a count of the rest. The reference lists
 * every daemon pod here (OverviewPage.tsx:252-272): three per GPU node, so
 * thousands of rows on a large cluster.
 */
function overviewPluginPods(pods, now) {
  const notReady = chunkedFilter('ov-plugin-not-ready', pods, function (p) { return !isPodReady(p); });
  let shown = pods;
  if (pods.length > OVERVIEW_PLUGIN_PODS) {
    shown = notReady.slice(0, OVERVIEW_PLUGIN_PODS);
    for (let i = 0; i < pods.length && shown.length < OVERVIEW_PLUGIN_PODS; i++) {
      if (isPodReady(pods[i])) shown.push(pods[i]);
    }
  }
  const blocks = [
    table(
      ['Name', 'Namespace', 'Component', 'Node', 'Status', 'Age'],
      chunkedRows('ov-plugin-rows', shown, [], function (p) {
        return ovPluginRows(p, [], function () {
          return [podName(p), podNs(p), formatComponent(pluginPodComponent(p)), podNode(p), readyLabel(p), ageText(p.metadata.creationTimestamp, now)];
        }, now);
      }, now)
    ),
  ];
  if (shown.length < pods.length) {
    const nr = notReady.length > 0 ? status('warning', notReady.length + ' not ready') : status('success', 'all ready');
    blocks.push(kv([
      row('Shown', shown.length + ' of ' + pods.length + ' operator pods (not-ready first; all of them on the Device Plugins page)'),
      row('Readiness', nr),
    ]));
  }
  return section('Plugin Daemon Pods', blocks);
}

function overviewNodes(gpuNodes, t) {
  const nodeBlocks = [];
  if (t.nodes > 0) {
    nodeBlocks.push(
      pctbar(
        'Node Readiness',
        [
          { name: 'Ready', value: t.readyNodes, fill: BAR_COLORS.ok },
          { name: 'Not Ready', value: t.nodes - t.readyNodes, fill: BAR_COLORS.mute },
        ].filter(function (d) { return d.value > 0; }),
        t.nodes
      )
    );
    // Analog of the reference's GPU-type distribution (OverviewPage.tsx:37-48):
    // every GPU is an MI355X, so what varies between nodes is the partition mode.
    // Node labels only: holds across pod events.
    const modes = memo('overview-modes', [gpuNodes], function () { return partitionModeDistribution(gpuNodes); });
    if (modes.length > 0) nodeBlocks.push(pctbar('GPU Partition Modes', modes, t.nodes));
  }
  const nodeRows = [
    row('Total GPU Nodes', status(t.nodes > 0 ? 'success' : 'warning', t.nodes)),
    row('Ready Nodes', String(t.readyNodes)),
  ];
  if (t.cordonedNodes > 0) nodeRows.push(row('Cordoned Nodes', status('warning', t.cordonedNodes + ' (SchedulingDisabled)')));
  if (t.nodes > 0) nodeRows.push(row('GPU Model', MI355X.product + ' (' + MI355X.arch + ')'));
  if (t.capacity > 0) {
    nodeRows.push(row('Total GPU Devices', String(t.capacity)));
    if (t.physicalGpus !== t.capacity) nodeRows.push(row('Physical GPUs', String(t.physicalGpus)));
    nodeRows.push(row('Total HBM', formatBytes(t.hbmBytes) + ' (' + MI355X.hbmLabel + ' per GPU)'));
  }
  if (t.partitions > 0) nodeRows.push(row('GPU Partitions', String(t.partitions)));
  nodeBlocks.push(kv(nodeRows));
  return section('GPU Nodes', nodeBlocks);
}

function overviewAllocation(t) {
  return section('GPU Allocation', [
    pctbar(
      'GPU Allocation (' + t.utilizationPct + '%)',
      [
        { name: 'In Use', value: t.inUse, fill: BAR_COLORS.ok },
        { name: 'Available', value: t.free, fill: BAR_COLORS.track },
      ],
      t.allocatable
    ),
    kv([
      row('Total Capacity (GPU devices)', String(t.capacity)),
      row('Allocatable', String(t.allocatable)),
      row('In Use', String(t.inUse)),
      row('Free', status(t.free > 0 ? 'success' : 'warning', t.free)),
    ].concat(t.cordonedNodes > 0 || t.readyNodes < t.nodes ? [
      // Free GPUs on cordoned / not-Ready nodes take no new pods.
      row('Free on Schedulable Nodes', status(t.schedulableFree > 0 ? 'success' : 'warning', t.schedulableFree)),
    ] : [], [
      row('HBM Allocated', formatBytes(t.hbmAllocatedBytes)),
    ])),
  ]);
}

function overviewWorkloads(ph, total) {
  const wl = [row('Total GPU Pods', String(total))];
  if (ph.Running > 0) wl.push(row('Running', status('success', ph.Running)));
  if (ph.Pending > 0) wl.push(row('Pending', status('warning', ph.Pending)));
  if (ph.Failed > 0) wl.push(row('Failed', status('error', ph.Failed)));
  return section('GPU Workloads', [kv(wl)]);
}

/** The first ACTIVE_PODS_LIMIT running GPU pods (reference OverviewPage.tsx:414), or null. */
function overviewActivePods(gpuPods, now) {
  const running = [];
  for (let i = 0; i < gpuPods.length && running.length < ACTIVE_PODS_LIMIT; i++) {
    if (podFacts(gpuPods[i]).phase === 'Running') running.push(gpuPods[i]);
  }
  if (running.length === 0) return null;
  return section('Active GPU Pods', [
    table(
      ['Name', 'Namespace', 'Node', 'GPU Request', 'Age'],
      running.map(function (p) {
        return [podName(p), podNs(p), podNode(p), formatPodGpuRequests(p), ageText(p.metadata.creationTimestamp, now)];
      })
    ),
  ]);
}

// ---------------------------------------------------------------------------
// Device Plugins (reference DevicePluginsPage.tsx:20-219)
// ---------------------------------------------------------------------------

function enabledCell(on, detail) {
  return on ? status('success', detail ? 'Enabled — ' + detail : 'Enabled') : status('warning', 'Disabled');
}

/**
 * One card per DeviceConfig (reference: one per GpuDevicePlugin). Per-operand
 * DaemonSet counts replace the single desired/ready pair.
 */
export function devicePluginsView(ctx, opts) {
  const now = nowOf(opts);
  if (ctx.loading) return page(null, null, [loader('Loading device plugin data...')]);
  // One page of the operator pod table (PODS_PER_PAGE; filter on
  // namespace/name and node): three per GPU node on a real cluster.
  const pg = podPage(ctx.pluginPods, opts && opts.pager, 'plugin-pod');
  const items = memo(
    'device-plugins',
    [ctx.deviceConfigs, pg, ctx.crdAvailable, ctx.error],
    function () { return devicePluginsItems(ctx, now, pg); },
    now
  );
  return page(BRAND + ' — Device Plugins', refreshButton('Refresh device plugin data', ctx.refreshing), items);
}

function devicePluginsItems(ctx, now, pg) {
  const items = [];
  if (ctx.error) items.push(errorSection(ctx.error));

  if (!ctx.crdAvailable) {
    items.push(
      section('CRD Not Available', [
        kv(ctx.crdForbidden
          ? [
            // 403: the operator may well be installed; this user cannot list its CRs.
            row('Status', status('warning', 'DeviceConfig list forbidden for this user (HTTP 403)')),
            row('Note', 'Grant list on deviceconfigs.amd.com (deploy/rbac/headlamp-amd-gpu-viewer.yaml). Device plugin daemon pods are shown below if detected.'),
          ]
          : [
            row('Status', status('warning', 'DeviceConfig CRD (amd.com/v1alpha1) is not installed')),
            row(
              'Note',
              'Install the AMD GPU Operator to manage DeviceConfig resources. Device plugin daemon pods are shown below if detected.'
            ),
          ]),
      ])
    );
  }

  if (ctx.crdAvailable && ctx.deviceConfigs.length === 0) {
    items.push(
      section('No Device Configs', [
        kv([
          row('Status', status('warning', 'No DeviceConfig resources found on this cluster')),
          row('Create', 'kubectl apply -f deviceconfig.yaml (see the AMD GPU Operator documentation)'),
        ]),
      ])
    );
  }

  for (let i = 0; i < ctx.deviceConfigs.length; i++) {
    const dc = ctx.deviceConfigs[i];
    const dp = operandStatus(dc, 'devicePlugin');
    const rows = [
      row('Status', status(deviceConfigStatus(dc), deviceConfigStatusText(dc))),
      row('Namespace', dc.metadata.namespace || '—'),
      row('Device Plugin Image', get(dc, ['spec', 'devicePlugin', 'devicePluginImage'], '—')),
      row(
        'Driver',
        enabledCell(operandEnabled(dc, 'driver'), get(dc, ['spec', 'driver', 'version'], null))
      ),
      row('Node Labeller', enabledCell(operandEnabled(dc, 'nodeLabeller'))),
      row(
        'Metrics Exporter',
        enabledCell(
          operandEnabled(dc, 'metricsExporter'),
          get(dc, ['spec', 'metricsExporter', 'port'], null) !== null ? 'port ' + get(dc, ['spec', 'metricsExporter', 'port'], '') : null
        )
      ),
      row('Desired Nodes', String(dp.desired)),
      row('Ready Nodes', String(dp.available)),
    ];
    if (dp.unavailable > 0) rows.push(row('Unavailable Nodes', status('error', dp.unavailable)));
    for (let k = 0; k < OPERANDS.length; k++) {
      const op = OPERANDS[k];
      if (op.key === 'devicePlugin' || !operandEnabled(dc, op.key)) continue;
      const st = operandStatus(dc, op.key);
      rows.push(row(op.label + ' Pods', status(countsToStatus(st.desired, st.available), countsToText(st.desired, st.available))));
    }
    rows.push(row('Node Selector', formatSelector(get(dc, ['spec', 'selector'], null))));
    rows.push(row('Age', ageText(dc.metadata.creationTimestamp, now)));
    items.push(section('DeviceConfig: ' + dc.metadata.name, [kv(rows)], dc.metadata.uid || dc.metadata.name));
  }

  if (ctx.pluginPods.length > 0) {
    items.push(pager(pg, 'operator pods'));
    items.push(
      section('Plugin Daemon Pods', [
        table(
          ['Name', 'Namespace', 'Component', 'Node', 'Ready', 'Restarts', 'Age'],
          chunkedRows('dp-plugin-rows', pg.nodes, [], function (p) {
            return dpPluginRows(p, [], function () {
              return [
                podName(p), podNs(p), formatComponent(pluginPodComponent(p)), podNode(p), readyLabel(p),
                restartsCell(p), ageText(p.metadata.creationTimestamp, now),
              ];
            }, now);
          }, now)
        ),
      ])
    );
  }

  return items;
}

// ---------------------------------------------------------------------------
// Nodes (reference NodesPage.tsx:145-293)
// ---------------------------------------------------------------------------

/** GPU nodes per page on the GPU Nodes and Metrics pages. */
export const NODES_PER_PAGE = 8;

function nodeNameOf(n) {
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

function podKeyOf(p) {
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

/** The rank of a power-ordered owners answer as a pager page: its pods, in rank order, out of the pods ranked. */
function rankedPodPage(ctx, m, state) {
  const byKey = memo('pods-by-key', [ctx.gpuPods], function () {
    const out = new Map();
    for (let i = 0; i < ctx.gpuPods.length; i++) out.set(podKeyOf(ctx.gpuPods[i]), ctx.gpuPods[i]);
    return out;
  });
  return memo('pods-ranked-page', [m, byKey], function () {
    const r = m.rank;
    const pods = [];
    for (let i = 0; i < r.order.length; i++) if (byKey.has(r.order[i])) pods.push(byKey.get(r.order[i]));
    const count = Math.max(r.count, r.page * r.per + pods.length);
    const from = Math.min(r.page * r.per, count);
    return {
      nodes: pods, names: pods.map(podKeyOf), page: r.page, pages: Math.max(1, Math.ceil(count / r.per)), from: from,
      to: from + pods.length, total: count, matched: count, filter: (state && state.filter) || '', perPage: r.per, ranked: true,
    };
  });
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

/** Names of the GPU nodes a paged view shows ([] while the node list is loading). */
export function visibleNodeNames(ctx, state) {
  if (!ctx || ctx.loading || !ctx.gpuNodes) return [];
  return nodePage(ctx.gpuNodes, state, ctx.index).names;
}

/**
 * What a paged page asks Prometheus for:
 *   * while the node list is loading, and while every GPU node fits on one
 *     page: `small` — the whole cluster if it has at most SMALL_CLUSTER_GPUS
 *     GPUs, else the page's nodes, decided by Prometheus in the same request
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
  if (nodes !== 'ready' && ctx.loading) return { enabled: true, scope: [], small: true };
  if (ctx.error && (!ctx.gpuNodes || ctx.gpuNodes.length === 0)) return { enabled: true, scope: undefined };
  const names = nodePage(ctx.gpuNodes, state, ctx.index).names;
  return ctx.gpuNodes.length <= SMALL_CLUSTER_NODES ? { enabled: true, scope: names, small: true } : { enabled: true, scope: names };
}

/** Per-GPU allocation strip block. */
export function slotsBlock(node, podsOnNode, owners) {
  const s = buildGpuSlots(node, podsOnNode, owners);
  return { t: 'slots', slots: s.slots, exact: s.exact, partitionsPerGpu: s.partitionsPerGpu };
}

/** xGMI neighbour matrix block; `measuredTopology` when link hops came from the exporter. */
export function matrixBlock(gpuCount, measured, probed) {
  const hasProbe = !!probed && Object.keys(probed).length > 0;
  const m = buildXgmiMatrix(gpuCount, measured, hasProbe ? probed : undefined);
  return {
    t: 'matrix',
    matrix: m,
    fullMesh: isFullMesh(m),
    // Link types / hops come from the exporter's gpu_xgmi_link_hops (this
    // repo's amdgpu-exporter); without them the matrix is the MI355X
    // platform model, and only per-link throughput (stock exporter
    // xgmi_neighbor_*_tx_throughput) is measured.
    measuredTopology: hasProbe,
    measuredThroughput: !!measured && Object.keys(measured).length > 0,
  };
}

/**
 * Readiness as `kubectl get nodes` words it: "Ready", "Not Ready", and
 * ", SchedulingDisabled" on a cordoned node (spec.unschedulable) — whose free
 * GPUs new pods cannot use, hence a warning.
 */
export function nodeReadyCell(node) {
  const ready = isNodeReady(node);
  const cordoned = get(node, ['spec', 'unschedulable'], false) === true;
  const text = (ready ? 'Ready' : 'Not Ready') + (cordoned ? ', SchedulingDisabled' : '');
  return status(!ready ? 'error' : cordoned ? 'warning' : 'success', text);
}

/** "key=value:Effect" per taint (the reference models NodeSpec.taints, k8s.ts:92-122, but never shows them). */
export function formatTaints(node) {
  const ts = get(node, ['spec', 'taints'], []);
  if (!Array.isArray(ts) || ts.length === 0) return null;
  return ts.map(function (t) { return (t.key || '') + (t.value ? '=' + t.value : '') + ':' + (t.effect || ''); }).join(', ');
}

function nodeCardRows(node, podsOnNode, stats, now) {
  const model = getNodeGpuModel(node);
  const count = getNodeGpuCount(node);
  const cap = getGpuResources(get(node, ['status', 'capacity'], null));
  const alloc = getGpuResources(get(node, ['status', 'allocatable'], null));
  const rows = [
    row('Status', nodeReadyCell(node)),
    row('GPU Model', model.product),
  ];
  const taints = formatTaints(node);
  if (taints) rows.push(row('Taints', taints));
  if (count > 0) {
    const phys = getNodePhysicalGpuCount(node);
    rows.push(row('GPU Devices (amd.com/gpu)', phys !== count ? count + ' (' + phys + ' × ' + model.shortName + ' in ' + model.computePartition + ')' : String(count)));
    rows.push(row('HBM', formatBytes(phys * MI355X.hbmBytes) + ' (' + phys + ' × ' + model.vram + ')'));
  }
  for (const k in cap) rows.push(row(formatGpuResourceName(k) + ' (capacity)', cap[k]));
  for (const k in alloc) rows.push(row(formatGpuResourceName(k) + ' (allocatable)', alloc[k]));
  if (stats) rows.push(row('GPU Allocation', allocationBar(stats.inUse, stats.allocatable || count)));
  if (model.computePartition || model.memoryPartition) rows.push(row('Partition Mode', formatGpuModel(model)));
  const drv = labellerValue(node, 'driver-version');
  if (drv) rows.push(row('amdgpu Driver', drv));
  rows.push(row('GPU Workload Pods', podsOnNode.length > 0 ? podsOnNode.map(podName).join(', ') : '—'));
  rows.push(row('OS Image', get(node, ['status', 'nodeInfo', 'osImage'], '—')));
  rows.push(row('Kernel', get(node, ['status', 'nodeInfo', 'kernelVersion'], '—')));
  rows.push(row('Kubelet', get(node, ['status', 'nodeInfo', 'kubeletVersion'], '—')));
  rows.push(row('Age', ageText(node.metadata.creationTimestamp, now)));
  return rows;
}

/**
 * Differences: Allocation = GPUs held / allocatable GPUs (reference used the
 * pod count, quirk Q2); each node card adds HBM, the per-GPU allocation
 * strip and the xGMI neighbour matrix. `metrics` (optional) supplies exact
 * per-GPU owners and measured xGMI throughput.
 */
export function nodesView(ctx, opts) {
  const now = nowOf(opts);
  const metrics = opts && opts.metrics ? opts.metrics : null;
  if (ctx.loading) return page(null, null, [loader('Loading GPU node data...')]);
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
  const head = memo('nodes-head', [pg, ctx.index, ctx.error, power.sig], function () {
    return nodesHeadItems(ctx, now, power.byNode, pg, sort);
  }, now);
  const owners = ownersByNode(metrics);
  const xgmi = metrics ? metrics.xgmi : undefined;
  const links = metrics ? metrics.links : undefined;
  // The card list as a whole holds while no input changed (most watch events
  // touch no GPU node or pod); otherwise only changed cards are rebuilt.
  const items = memo('nodes-cards', [head, pg, ctx.index, owners, xgmi, links], function () {
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
      const stats = d[1];
      const own = d[2];
      const xg = d[3];
      const lk = d[4];
      // own / xg / lk keep their identity while their content is unchanged
      // (ownersByNode + the metrics client's structural sharing).
      return memo('node-card:' + name, [n, pods, stats, own, xg, lk], function () {
        const blocks = [kv(nodeCardRows(n, pods, stats, now))];
        const count = getNodeGpuCount(n);
        if (count > 0) {
          blocks.push(slotsBlock(n, pods, own));
          blocks.push(matrixBlock(getNodePhysicalGpuCount(n), xg, lk));
        }
        return section(name, blocks, n.metadata.uid || name);
      }, now);
    }, now, inputs);
    return head.concat(cards);
  }, now);
  return page(BRAND + ' — Nodes', refreshButton('Refresh node data', !!(opts && opts.fetching)), items);
}

const ownersCache = typeof WeakMap === 'function' ? new WeakMap() : null;
let lastOwners = {};

function sameOwners(a, b) {
  if (!a || !b || a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) {
    if (a[i].gpu !== b[i].gpu || a[i].pod !== b[i].pod || a[i].namespace !== b[i].namespace) return false;
  }
  return true;
}

/**
 * node → [{gpu, pod, namespace}] from exporter pod labels, computed once per
 * GPU list; a node's array keeps its identity while its owners are unchanged
 * (telemetry values change every scrape, GPU ownership rarely).
 */
const NO_OWNERS = Object.freeze({});
const NO_PODS = Object.freeze([]);

function ownersByNode(metrics) {
  if (!metrics || !metrics.gpus) return NO_OWNERS;
  if (ownersCache && ownersCache.has(metrics.gpus)) return ownersCache.get(metrics.gpus);
  const out = {};
  for (let i = 0; i < metrics.gpus.length; i++) {
    const g = metrics.gpus[i];
    if (!g.pod) continue;
    if (!out[g.nodeName]) out[g.nodeName] = [];
    out[g.nodeName].push({ gpu: g.gpu, pod: g.pod, namespace: g.namespace });
  }
  for (const k in out) {
    if (sameOwners(lastOwners[k], out[k])) out[k] = lastOwners[k];
  }
  lastOwners = out;
  if (ownersCache) ownersCache.set(metrics.gpus, out);
  return out;
}

let lastAssign = {};

function sameAssign(a, b) {
  if (!a || !b || a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) if (a[i] !== b[i]) return false;
  return true;
}

/**
 * "namespace/pod" → the GPUs the exporter attributes to that pod (its
 * pod/namespace labels), as GPU objects of the metrics snapshot. Kubernetes
 * itself does not say which device a pod got; this is the exporter's view.
 * A pod's array keeps its identity while its GPUs are the same objects
 * (see the metrics client's structural sharing), and the whole map keeps
 * its identity while no pod's list changed.
 */
export function podGpuAssignments(metrics) {
  if (!metrics || !metrics.gpus) return {};
  if (assignCache && assignCache.has(metrics.gpus)) return assignCache.get(metrics.gpus);
  const out = {};
  for (let i = 0; i < metrics.gpus.length; i++) {
    const g = metrics.gpus[i];
    if (!g.pod) continue;
    const k = (g.namespace || '') + '/' + g.pod;
    if (!out[k]) out[k] = [];
    out[k].push(g);
  }
  let same = Object.keys(out).length === Object.keys(lastAssign).length;
  for (const k in out) {
    if (sameAssign(lastAssign[k], out[k])) out[k] = lastAssign[k];
    else same = false;
  }
  const res = same ? lastAssign : out;
  lastAssign = res;
  if (assignCache) assignCache.set(metrics.gpus, res);
  return res;
}
const assignCache = typeof WeakMap === 'function' ? new WeakMap() : null;

function assignedLines(gs) {
  return lines(
    gs.map(function (g) {
      const parts = [];
      if (g.powerWatts !== null && g.powerWatts !== undefined) parts.push(formatWatts(g.powerWatts));
      if (g.gfxActivityPct !== null && g.gfxActivityPct !== undefined) parts.push(Math.round(g.gfxActivityPct) + '% GFX');
      if (g.vramUsedBytes !== null && g.vramUsedBytes !== undefined) parts.push(formatBytes(g.vramUsedBytes) + ' HBM');
      return { label: g.nodeName + ' GPU ' + g.gpu, text: parts.length ? parts.join(', ') : 'no telemetry' };
    })
  );
}

function assignedText(gs) {
  if (!gs || gs.length === 0) return '—';
  const byNode = {};
  const order = [];
  for (let i = 0; i < gs.length; i++) {
    if (!byNode[gs[i].nodeName]) {
      byNode[gs[i].nodeName] = [];
      order.push(gs[i].nodeName);
    }
    byNode[gs[i].nodeName].push(gs[i].gpu);
  }
  return order.map(function (n) { return n + ': GPU ' + byNode[n].join(', '); }).join('; ');
}

/** Per-node GPU power from a telemetry snapshot: {byNode: {node: "watts|cap"}, sig} (whole watts). */
export function nodePowerKeys(metrics) {
  const sum = {};
  const gs = metrics && Array.isArray(metrics.gpus) ? metrics.gpus : [];
  for (let i = 0; i < gs.length; i++) {
    const g = gs[i];
    if (typeof g.powerWatts !== 'number' || !isFinite(g.powerWatts)) continue;
    const e = sum[g.nodeName] || (sum[g.nodeName] = [0, 0]);
    e[0] += g.powerWatts;
    e[1] += typeof g.powerCapWatts === 'number' && isFinite(g.powerCapWatts) ? g.powerCapWatts : 0;
  }
  const byNode = {};
  const names = Object.keys(sum).sort();
  for (let i = 0; i < names.length; i++) byNode[names[i]] = Math.round(sum[names[i]][0]) + '|' + Math.round(sum[names[i]][1]);
  return { byNode: byNode, sig: names.map(function (n) { return n + '=' + byNode[n]; }).join(',') };
}

function nodePowerCell(key) {
  if (!key) return '—';
  const parts = key.split('|');
  const cap = Number(parts[1]);
  return powerBar(Number(parts[0]), cap > 0 ? cap : null);
}

function nodesHeadItems(ctx, now, powerByNode, pg, sort) {
  const pw = powerByNode || {};
  const withPower = Object.keys(pw).length > 0;
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
          // "Power" (beyond the reference): the node's GPUs' live power against their summed cap.
          ['Node', 'Ready', 'GPU Model', 'GPU Devices', 'Allocation', 'GPU Pods'].concat(withPower ? ['Power'] : [], ['Age']),
          chunkedRows('node-summary-rows', pg.nodes, [withPower], function (n) {
            const st = idx.nodeStats.get(n.metadata.name);
            const pk = pw[n.metadata.name];
            // Per-node stats keep their identity while unchanged (buildClusterIndex).
            return nodeSummaryRows(n, [st, withPower, pk], function () {
              const count = getNodeGpuCount(n);
              return [
                n.metadata.name,
                nodeReadyCell(n),
                formatGpuModel(getNodeGpuModel(n)),
                count > 0 ? String(count) : '—',
                allocationBar(st ? st.inUse : 0, (st && st.allocatable) || count),
                String(st ? st.pods : 0),
              ].concat(withPower ? [nodePowerCell(pk)] : [], [ageText(n.metadata.creationTimestamp, now)]);
            }, now);
          }, now, function (n) { return [idx.nodeStats.get(n.metadata.name), withPower, pw[n.metadata.name]]; }),
          pg.nodes.map(function (n) { return n.metadata.uid || n.metadata.name; })
        ),
      ])
    );
  }

  return items;
}

/**
 * The Pods page's owner query: `small` (every owner when at most
 * SMALL_CLUSTER_PODS pods hold a GPU, else the page's pods) while the pod
 * list loads or is that short; the pods of its page (namespace/name keys)
 * once a longer list is in; cluster-wide when the pod list failed.
 * @returns {{enabled: boolean, pods: (string[]|undefined), small?: boolean}}
 */
export function ownersScope(ctx, state) {
  if (!ctx) return { enabled: false, pods: [] };
  // Power order: Prometheus picks the page — no pod list needed.
  if (podSortOf(state, RANKED_POD_SORTS) === 'power') {
    const st = state || {};
    return {
      enabled: true,
      rank: { by: 'power', page: Math.max(0, Math.floor(st.page) || 0), per: PODS_PER_PAGE, filter: (st.filter || '').trim().toLowerCase() },
    };
  }
  if (ctx.podsState === 'error') return { enabled: true, pods: undefined };
  // As telemetryScope: every owner of a small cluster in the first wave.
  if (ctx.podsState !== 'ready' && ctx.loading) return { enabled: true, pods: [], small: true };
  if (ctx.error && (!ctx.gpuPods || ctx.gpuPods.length === 0)) return { enabled: true, pods: undefined };
  const pods = podPage(ctx.gpuPods, state).names;
  return ctx.gpuPods.length <= SMALL_CLUSTER_PODS ? { enabled: true, pods: pods, small: true } : { enabled: true, pods: pods };
}

// ---------------------------------------------------------------------------
// Pods (reference PodsPage.tsx:94-270)
// ---------------------------------------------------------------------------

/** Per-container GPU lines (reference GpuContainerList, PodsPage.tsx:49-88), init containers included. */
export function gpuContainerLines(pod) {
  const out = [];
  function add(c, init) {
    const es = containerGpuEntries(c);
    const parts = [];
    for (let i = 0; i < es.length; i++) {
      const e = es[i];
      const label = formatGpuResourceName(e.key);
      if (e.request !== null && e.limit !== null && e.request === e.limit) parts.push(label + ': ' + e.request);
      else parts.push(label + ': req=' + (e.request === null ? '—' : e.request) + ' lim=' + (e.limit === null ? '—' : e.limit));
    }
    out.push({ label: c.name + (init ? ' (init)' : ''), text: parts.join(', ') });
  }
  const ics = gpuInitContainers(pod);
  for (let i = 0; i < ics.length; i++) add(ics[i], true);
  const cs = gpuContainers(pod);
  for (let i = 0; i < cs.length; i++) add(cs[i], false);
  return out.length ? lines(out) : '—';
}

export function podsView(ctx, opts) {
  const now = nowOf(opts);
  if (ctx.loading) return page(null, null, [loader('Loading GPU pod data...')]);
  const assign = opts && opts.metrics ? podGpuAssignments(opts.metrics) : null;
  // One page of the GPU pod table (PODS_PER_PAGE, filter on namespace/name
  // and node): the reference lists every GPU pod (PodsPage.tsx:201-236).
  const sort = podSortOf(opts && opts.pager, RANKED_POD_SORTS);
  const m = opts && opts.metrics;
  const ranked = sort === 'power' && m && m.rank && Array.isArray(m.rank.order);
  const pg = ranked ? rankedPodPage(ctx, m, opts.pager) : podPage(ctx.gpuPods, opts && opts.pager);
  const items = memo('pods', [pg, ctx.index, ctx.error, assign, sort], function () {
    return podsItems(ctx, now, assign, pg, sort);
  }, now);
  return page(BRAND + ' — Pods', refreshButton('Refresh pod data', !!(opts && opts.fetching)), items);
}

function podsItems(ctx, now, assign, pg, sort) {
  const items = [];
  if (ctx.error) items.push(errorSection(ctx.error));
  const pods = ctx.gpuPods;

  if (pods.length === 0) {
    items.push(
      section('No GPU Pods Found', [
        kv([
          row('Status', status('warning', 'No pods requesting AMD GPU resources were found')),
          row('Note', 'Pods appear here when they request resources like amd.com/gpu.'),
        ]),
      ])
    );
  }

  const ph = ctx.index.phases;
  const pending = ph.Pending > 0 ? chunkedFilter('pending-pods', pods, function (p) { return podFacts(p).phase === 'Pending'; }) : [];
  if (pods.length > 0) {
    const rows = [row('Total GPU Pods', String(pods.length))];
    if (ph.Running > 0) rows.push(row('Running', status('success', ph.Running)));
    if (ph.Pending > 0) rows.push(row('Pending', status('warning', ph.Pending)));
    if (ph.Failed > 0) rows.push(row('Failed', status('error', ph.Failed)));
    rows.push(row('GPUs Held', String(ctx.index.totals.heldGpus)));
    items.push(section('Summary', [kv(rows)]));

    // With exporter pod labels, show which physical GPUs each pod holds.
    const exact = assign && Object.keys(assign).length > 0;
    const cols = ['Name', 'Namespace', 'Node', 'Phase', 'GPU Resources', 'Restarts', 'Age'];
    if (exact) cols.splice(5, 0, 'Assigned GPUs', 'GPU Power');
    items.push(pager(pg, pg.ranked ? 'GPU pods drawing power' : 'GPU pods', { sort: sort, sorts: RANKED_POD_SORTS, label: 'GPU pods' }));
    items.push(
      section('All GPU Pods', [
        table(
          cols,
          chunkedRows('pod-rows', pg.nodes, [exact, assign], function (p) {
            // A pod's assignment keeps its identity while its GPUs are unchanged (podGpuAssignments).
            const gs = exact ? assign[(p.metadata.namespace || '') + '/' + p.metadata.name] : undefined;
            return podRows(p, [exact, gs], function () {
              const phase = podPhase(p);
              const r = [
                podName(p), podNs(p), podNode(p), status(phaseToStatus(phase), phase), gpuContainerLines(p),
                restartsCell(p), ageText(p.metadata.creationTimestamp, now),
              ];
              if (exact) r.splice(5, 0, assignedText(gs), podPowerText(gs));
              return r;
            }, now);
          }, now),
          pg.nodes.map(function (p) { return p.metadata.uid || (p.metadata.namespace + '/' + p.metadata.name); })
        ),
      ])
    );
  }

  if (pending.length > 0) {
    // The oldest PODS_PER_PAGE pending pods (a scheduler backlog can be
    // thousands deep); the rest are counted, and found with the filter.
    const shown = pending.length > PODS_PER_PAGE ? pending.slice(0, PODS_PER_PAGE) : pending;
    const blocks = [
      table(
        // "Message" (beyond the reference): why the scheduler cannot place the pod.
        ['Name', 'Namespace', 'GPU Resources', 'Waiting Reason', 'Message', 'Age'],
        shown.map(function (p) {
          return pendingRows(p, [], function () {
            return [podName(p), podNs(p), formatPodGpuRequests(p), podWaitingReason(p) || '—', podWaitingMessage(p) || '—',
              ageText(p.metadata.creationTimestamp, now)];
          }, now);
        })
      ),
    ];
    if (shown.length < pending.length) {
      blocks.push(kv([row('Not shown', (pending.length - shown.length) + ' more pending GPU pods (filter the table above by name)')]));
    }
    items.push(section('Attention: Pending GPU Pods', blocks));
  }

  return items;
}

// ---------------------------------------------------------------------------
// Metrics (reference MetricsPage.tsx:191-355)
// ---------------------------------------------------------------------------

/** Live power of the GPUs a pod holds (exporter pod labels), summed; "—" without a reading. */
export function podPowerText(gs) {
  if (!gs || !gs.length) return '—';
  let w = 0;
  let any = false;
  for (let i = 0; i < gs.length; i++) {
    if (typeof gs[i].powerWatts === 'number' && isFinite(gs[i].powerWatts)) {
      w += gs[i].powerWatts;
      any = true;
    }
  }
  return any ? formatWatts(w) : '—';
}

/** Mean value per node of a series map (node → [[t, v]]); nodes without samples are left out. */
export function seriesMeans(byNode) {
  const out = {};
  for (const n in byNode || {}) {
    const pts = byNode[n] || [];
    let sum = 0;
    let k = 0;
    for (let i = 0; i < pts.length; i++) {
      if (typeof pts[i][1] === 'number' && isFinite(pts[i][1])) {
        sum += pts[i][1];
        k++;
      }
    }
    if (k) out[n] = sum / k;
  }
  return out;
}

/** "k / n GPU nodes": nodes with telemetry out of the cluster's GPU nodes (reference mock-up "Nodes Reporting"). */
export function nodesReporting(m, ctx) {
  const seen = {};
  let k = 0;
  for (let i = 0; i < m.gpus.length; i++) {
    if (!seen[m.gpus[i].nodeName]) {
      seen[m.gpus[i].nodeName] = true;
      k++;
    }
  }
  const n = ctx && ctx.gpuNodes ? ctx.gpuNodes.length : 0;
  if (!n) return String(k);
  let missing = 0;
  for (let i = 0; i < ctx.gpuNodes.length; i++) if (!seen[ctx.gpuNodes[i].metadata.name]) missing++;
  const text = k + ' / ' + n + ' GPU nodes';
  return missing > 0 ? status('warning', text + ' (' + missing + ' without telemetry)') : text;
}

/** "k / n GPU nodes" from an aggregate count of nodes reporting (paged snapshot totals). */
export function nodesReportingCount(k, ctx) {
  const n = ctx && ctx.gpuNodes ? ctx.gpuNodes.length : 0;
  if (!n) return String(k);
  const text = k + ' / ' + n + ' GPU nodes';
  return k < n ? status('warning', text + ' (' + (n - k) + ' without telemetry)') : text;
}

/** The "GPU Nodes" row of the empty state: names, capped (a 1,000-node list is no help in one cell). */
function gpuNodeNamesText(ctx) {
  const ns = ctx.gpuNodes || [];
  if (!ns.length) return 'None detected';
  const shown = ns.slice(0, 20).map(function (n) { return n.metadata.name; }).join(', ');
  return ns.length > 20 ? shown + ' … (' + ns.length + ' GPU nodes)' : shown;
}

/** Label of the cluster-wide line in the series table. */
export const ALL_NODES_SERIES = 'All GPU nodes';

function withTotal(pts) {
  const o = {};
  if (pts && pts.length) o[ALL_NODES_SERIES] = pts;
  return o;
}

/** The entries of `byNode` for `names`, in that order. */
function pick(byNode, names) {
  const out = {};
  for (let i = 0; i < names.length; i++) if (byNode[names[i]]) out[names[i]] = byNode[names[i]];
  return out;
}

/** Per-step sum over every node of a cluster-wide series window (memoised per window). */
function seriesTotal(sr) {
  return memo('series-total', [sr], function () {
    function sum(byNode) {
      const total = {};
      for (const n in byNode || {}) {
        const pts = byNode[n] || [];
        for (let i = 0; i < pts.length; i++) {
          if (typeof pts[i][1] === 'number' && isFinite(pts[i][1])) total[pts[i][0]] = (total[pts[i][0]] || 0) + pts[i][1];
        }
      }
      return Object.keys(total).map(Number).sort(function (a, b) { return a - b; }).map(function (t) { return [t, total[t]]; });
    }
    return { power: sum(sr.power), vram: sum(sr.vram) };
  });
}

function noTelemetrySection(name) {
  return section(name + ' — no telemetry', [
    kv([row('Status', status('warning', 'No exporter series for this node (exporter not scheduled here, or not scraped yet)'))]),
  ], name);
}

/** Power bar: "X W / Y W (Z%)" with 70/90 colouring (reference PowerBar, MetricsPage.tsx:50-89). */
export function powerBar(watts, capWatts) {
  const hasCap = capWatts !== null && capWatts > 0;
  const p = hasCap ? Math.min(100, pct(watts, capWatts)) : null;
  const txt = formatWatts(watts) + (hasCap ? ' / ' + formatWatts(capWatts) + ' (' + formatPercent(watts, capWatts) + ')' : '');
  return bar(watts, hasCap ? capWatts : null, p, p === null ? BAR_COLORS.ok : pctToColor(p), txt);
}

export function hbmBar(used, total) {
  if (used === null) return '—';
  if (total === null || !(total > 0)) return formatBytes(used);
  const p = Math.min(100, pct(used, total));
  return bar(used, total, p, pctToColor(p), formatBytes(used) + ' / ' + formatBytes(total) + ' (' + p + '%)');
}

function pctText(v) {
  return v === null ? '—' : Math.round(v) + '%';
}

/** Static availability box (reference MetricRequirements, MetricsPage.tsx:125-185) — on AMD everything is available. */
export function metricAvailabilitySection() {
  return section('Metric Availability', [
    kv([
      row('Power (W)', lines([
        { label: '', text: 'Available — gpu_power_usage (AMD Device Metrics Exporter) or amdgpu hwmon power via node-exporter (power1_input on MI355X, which has no power1_average)' },
      ])),
      row('HBM used / total', lines([
        { label: '', text: 'Available — gpu_used_vram / gpu_total_vram, or node-exporter --collector.drm node_drm_memory_vram_* (288 GB HBM3E per MI355X)' },
      ])),
      row('GFX activity (%)', lines([{ label: '', text: 'Available — gpu_gfx_activity, or node_drm_gpu_busy_percent' }])),
      row('HBM controller activity (%)', lines([{ label: '', text: 'Available — gpu_umc_activity (exporter only)' }])),
      row('xGMI link throughput', lines([{ label: '', text: 'Available — xgmi_neighbor_N_tx_throughput (exporter only; 7 links per GPU)' }])),
      row('Per-GPU pod owner', lines([{ label: '', text: 'Available when the exporter runs with pod association (pod / namespace labels)' }])),
    ]),
  ]);
}

/**
 * @param {{gpuNodes: any[], loading: boolean}} ctx
 * @param {{ metrics: any|null, fetchError: string|null, fetching: boolean, series?: any }} mstate
 *
 * Differences: one card per NODE with a per-GPU table (the reference renders
 * one card per chip — 64 cards at 8 nodes); HBM, activity and temperature
 * columns; per-node power/HBM series when range data is present.
 */
export function metricsView(ctx, mstate, opts) {
  const now = nowOf(opts);
  const items = [];
  if (ctx.loading) items.push(loader('Loading ' + BRAND + ' data...'));
  items.push(metricAvailabilitySection());
  const m = mstate.metrics;
  if (mstate.fetching && !m) items.push(loader('Querying Prometheus for GPU metrics...'));

  if (mstate.fetchError) {
    // RBAC (HTTP 403 from the service proxy) is not an outage: say which permission is missing.
    const denied = /denied \(HTTP 403\)/.test(String(mstate.fetchError));
    items.push(
      section(denied ? 'Prometheus Access Denied' : 'Prometheus Unreachable', [
        kv([
          row('Error', status('error', mstate.fetchError)),
          row(
            'Checked services',
            PROMETHEUS_SERVICES.map(function (s) { return s.service + ':' + s.port; }).join(', ') + ' (monitoring namespace)'
          ),
        ]),
      ])
    );
  }

  const tot = m && m.totals ? m.totals : null;
  if (m && m.gpus.length === 0 && !(tot && tot.gpus > 0) && !(m.scope && !tot)) {
    items.push(
      section('No AMD GPU Metrics in Prometheus', [
        kv([
          row('Status', status('warning', 'Prometheus reachable — no gpu_power_usage or amdgpu hwmon series found')),
          row('GPU Nodes', gpuNodeNamesText(ctx)),
          row(
            'Likely cause',
            'The AMD Device Metrics Exporter is not deployed (DeviceConfig spec.metricsExporter.enable) or not scraped, and node-exporter is not running on the GPU nodes.'
          ),
        ]),
      ])
    );
  }

  if (m && (m.gpus.length > 0 || (tot && tot.gpus > 0))) {
    // Cluster totals: server-side aggregates on a paged (scoped) snapshot,
    // else summed here from every GPU of the snapshot.
    const sum = tot || summarizeMetrics(m);
    items.push(
      section('GPU Power Summary', [
        kv([
          row('GPUs Monitored', String(sum.gpus)),
          row('Nodes Reporting', tot ? nodesReportingCount(tot.nodes, ctx) : nodesReporting(m, ctx)),
          row('Total Power', powerBar(sum.powerWatts, sum.powerCapWatts > 0 ? sum.powerCapWatts : null)),
          row('HBM In Use', hbmBar(sum.vramUsedBytes, sum.vramTotalBytes > 0 ? sum.vramTotalBytes : null)),
          row('Avg GFX Activity', pctText(sum.avgGfxActivityPct)),
        ].concat(sum.eccUncorrectable === null ? [] : [row('RAS Errors', eccCell(sum))], [
          row('Source', m.source === 'node-exporter' ? 'node-exporter (amdgpu hwmon + DRM)' : 'AMD Device Metrics Exporter'),
        ], limitsRows(sum), [
          // Browser-local time, as the reference shows it (MetricsPage.tsx:336-338).
          row(
            'Last Fetched',
            m.stale
              ? status('warning', new Date(m.fetchedAt).toLocaleTimeString() + ' (stale: the latest refresh failed)')
              : new Date(m.fetchedAt).toLocaleTimeString()
          ),
        ], m.query ? [row('Query', m.query)] : [])),
      ])
    );

    const byNode = {};
    const order = [];
    for (let i = 0; i < m.gpus.length; i++) {
      const g = m.gpus[i];
      if (!byNode[g.nodeName]) {
        byNode[g.nodeName] = [];
        order.push(g.nodeName);
      }
      byNode[g.nodeName].push(g);
    }
    // One page of per-node cards. A paged snapshot covers the GPU nodes of
    // the page (m.scope); a cluster-wide one is paged over the nodes reporting.
    const scoped = Array.isArray(m.scope);
    const k8s = scoped && !ctx.loading && ctx.gpuNodes && ctx.gpuNodes.length > 0;
    // Power order: Prometheus picked and ranked the page (metrics.js rankedSnapshot).
    const pagerState = opts && opts.pager;
    const rankedView = !!m.rank && nodeSortOf(pagerState, RANKED_NODE_SORTS) === 'power';
    const pg = rankedView ? rankedPage(m, pagerState)
      : k8s ? nodePage(ctx.gpuNodes, pagerState, ctx.index) : nodePage(scoped ? m.scope : order, pagerState);

    const sr = mstate.series;
    if (sr && sr.power) {
      const win = formatWindow(sr.rangeSec || 1800);
      // A paged snapshot's series carry the cluster line apart (series.total);
      // a cluster-wide one is summed here. Peak / average are the cluster's;
      // the table shows the cluster line and the nodes of the page.
      const total = sr.total || seriesTotal(sr);
      const ps = clusterPowerStats({ cluster: total.power || [] });
      const cap = sum.powerCapWatts > 0 ? sum.powerCapWatts : null;
      const statRows = ps
        ? [kv([
          row('Peak Power (' + win + ')', powerBar(ps.peakWatts, cap)),
          row('Average Power (' + win + ')', powerBar(ps.avgWatts, cap)),
        ])]
        : [];
      const power = Object.assign(withTotal(total.power), pick(sr.power, pg.names));
      const vram = Object.assign(withTotal(total.vram), pick(sr.vram || {}, pg.names));
      items.push(
        section('Power & HBM (last ' + win + ')', statRows.concat([
          { t: 'series', power: power, vram: vram, avgPower: seriesMeans(power) },
        ]))
      );
    }

    items.push(rankedView ? pager(pg, 'GPU nodes reporting', { sort: 'power', sorts: RANKED_NODE_SORTS, label: 'GPU nodes' })
      : k8s ? pager(pg, 'GPU nodes', { sort: nodeSortOf(pagerState, RANKED_NODE_SORTS), sorts: RANKED_NODE_SORTS })
        : pager(pg, scoped ? 'GPU nodes' : 'GPU nodes reporting', { label: 'GPU nodes' }));
    const covered = {};
    if (scoped) for (let i = 0; i < m.scope.length; i++) covered[m.scope[i]] = true;
    let matched = 0;
    for (let i = 0; i < pg.names.length; i++) {
      const name = pg.names[i];
      const gs = byNode[name];
      if (gs) {
        matched++;
        // Deps are the node's GPU objects, which the metrics client reuses while unchanged.
        items.push(memo('metrics-node:' + name, gs, function () { return metricsNodeSection(name, gs); }));
      } else if (!scoped || covered[name]) {
        items.push(memo('metrics-none:' + name, [], function () { return noTelemetrySection(name); }));
      } else {
        items.push(section(name + ' — fetching telemetry…', [], name));
      }
    }
    if (scoped && tot && tot.gpus > 0 && matched === 0 && pg.names.length > 0 && pg.names.every(function (n) { return covered[n]; })) {
      items.push(section('Telemetry Not Matched To Nodes', [
        kv([
          row('Status', status('warning', 'Prometheus reports ' + tot.gpus + ' GPUs on ' + tot.nodes + ' nodes, none under the names of the nodes on this page')),
          row('Likely cause', 'The exporter\'s hostname label is not the Kubernetes node name (Device Metrics Exporter: set the node name as hostname).'),
        ]),
      ]));
    }
  }

  void now;
  return page(BRAND + ' — Metrics', refreshButton('Refresh metrics', mstate.fetching || ctx.loading), items);
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

/** The pager page of a power-ranked answer: its nodes, in rank order, out of the nodes ranked. */
function rankedPage(m, state) {
  return memo('metrics-ranked-page', [m], function () {
    const r = m.rank;
    const count = Math.max(r.count, r.page * r.per + m.scope.length);
    const from = Math.min(r.page * r.per, count);
    return {
      nodes: m.scope, names: m.scope, page: r.page, pages: Math.max(1, Math.ceil(count / r.per)), from: from,
      to: from + m.scope.length, total: count, matched: count, filter: (state && state.filter) || '', perPage: r.per,
    };
  });
}

/**
 * Junction temperature, coloured against the GPU's throttle threshold
 * (exporter-reported, else the MI355X's 100 °C): warning within 10 °C of
 * it, error at or above it.
 */
/** Says which limits are MI355X platform values because the source reports none. */
function limitsRows(sum) {
  const parts = [];
  if (sum.powerCapAssumed > 0) {
    parts.push('power cap ' + formatWatts(MI355X.tdpWatts) + ' (MI355X board limit; no gpu_power_cap series for ' +
      sum.powerCapAssumed + ' of ' + sum.gpus + ' GPUs)');
  }
  if (sum.tempLimitAssumed > 0) {
    parts.push('throttle threshold ' + MI355X.junctionSlowdownC + ' °C (MI355X; no gpu_junction_temperature_slowdown series for ' +
      sum.tempLimitAssumed + ' of ' + sum.gpus + ' GPUs)');
  }
  return parts.length ? [row('Assumed Limits', status('warning', parts.join('; ')))] : [];
}

export function tempCell(g) {
  if (g.tempC === null || g.tempC === undefined) return '—';
  const limit = g.tempSlowdownC > 0 ? g.tempSlowdownC : MI355X.junctionSlowdownC;
  const text = Math.round(g.tempC) + ' °C';
  if (g.tempC >= limit) return status('error', text + ' (throttling at ' + Math.round(limit) + ' °C)');
  if (g.tempC >= limit - 10) return status('warning', text);
  return text;
}

/**
 * RAS error counts of one GPU (or cluster totals): uncorrected errors are an
 * error (the driver may already have retired HBM pages or poisoned data),
 * corrected ones a warning, none "OK". '—' when the source reports no RAS
 * counters (node-exporter).
 */
export function eccCell(g) {
  if (g.eccUncorrectable === null || g.eccUncorrectable === undefined) return '—';
  const ce = g.eccCorrectable || 0;
  if (g.eccUncorrectable > 0) {
    return status('error', g.eccUncorrectable + ' uncorrected' + (ce > 0 ? ', ' + ce + ' corrected' : ''));
  }
  if (ce > 0) return status('warning', ce + ' corrected');
  return 'OK';
}

function metricsNodeSection(name, gs) {
  return section(
    name + ' — ' + gs.length + ' × ' + MI355X.shortName,
    [
      table(
        ['GPU', 'Power', 'HBM Used', 'GFX', 'HBM Activity', 'Temp', 'ECC', 'Pod'],
        gs.map(function (g) {
          return [
            'GPU ' + g.gpu,
            g.powerWatts !== null ? powerBar(g.powerWatts, g.powerCapWatts) : status('warning', 'No data'),
            hbmBar(g.vramUsedBytes, g.vramTotalBytes),
            pctText(g.gfxActivityPct),
            pctText(g.memActivityPct),
            tempCell(g),
            eccCell(g),
            g.pod ? (g.namespace ? g.namespace + '/' : '') + g.pod : '—',
          ];
        }),
        gs.map(function (g) { return g.nodeName + '-' + g.gpu; })
      ),
    ],
    name
  );
}

// ---------------------------------------------------------------------------
// Node detail section (reference NodeDetailSection.tsx:36-138)
// ---------------------------------------------------------------------------

/**
 * @param {any} resource  Headlamp KubeObject or raw Node
 * @param {{gpuPods: any[], loading: boolean, index?: any}} ctx
 * @returns {any|null}  a section, or null for non-GPU nodes
 *
 * Differences: in-use counts GPUs of every bound non-terminated pod
 * including init containers (reference: running pods' regular containers
 * only, quirk Q3); adds HBM, slots and the xGMI matrix.
 */
export function nodeDetailView(resource, ctx, opts) {
  const raw = unwrapKubeObject(resource);
  if (!isAmdGpuNode(raw)) return null;
  const cap = getGpuResources(get(raw, ['status', 'capacity'], null));
  const alloc = getGpuResources(get(raw, ['status', 'allocatable'], null));
  if (Object.keys(cap).length === 0 && Object.keys(alloc).length === 0) return null;
  const name = raw.metadata.name;
  let podsOnNode;
  if (ctx.loading) podsOnNode = [];
  else if (ctx.index && ctx.index.podsByNode && ctx.index.podsByNode.get(name)) podsOnNode = ctx.index.podsByNode.get(name);
  else podsOnNode = ctx.gpuPods.filter(function (p) { return get(p, ['spec', 'nodeName'], null) === name; });
  const metrics = opts && opts.metrics ? opts.metrics : null;
  const own = ownersByNode(metrics)[name];
  const xg = metrics && metrics.xgmi ? metrics.xgmi[name] : undefined;
  const lk = metrics && metrics.links ? metrics.links[name] : undefined;
  const podsUnreadable = ctx.podsState === 'error';
  const series = opts && opts.series && opts.series.power && opts.series.power.length ? opts.series : null;
  return memo('node-detail:' + name, [raw, podsOnNode, !!ctx.loading, podsUnreadable, own, xg, lk, series], function () {
    return nodeDetailSection(raw, name, cap, alloc, podsOnNode, ctx.loading, own, xg, lk, podsUnreadable, series);
  });
}

function nodeDetailSection(raw, name, cap, alloc, podsOnNode, loading, own, xg, lk, podsUnreadable, series) {
  const allocatable = parseInt(alloc[AMD_GPU_RESOURCE] || '0', 10) || 0;
  let inUse = 0;
  for (let i = 0; i < podsOnNode.length; i++) {
    const ph = podPhase(podsOnNode[i]);
    if (ph !== 'Succeeded' && ph !== 'Failed') inUse += getPodGpuCount(podsOnNode[i]);
  }
  const p = pct(inUse, allocatable);
  const model = getNodeGpuModel(raw);
  const rows = [row('GPU Model', model.product)];
  for (const k in cap) rows.push(row(formatGpuResourceName(k) + ' (capacity)', cap[k]));
  for (const k in alloc) rows.push(row(formatGpuResourceName(k) + ' (allocatable)', alloc[k]));
  const count = getNodeGpuCount(raw);
  const phys = getNodePhysicalGpuCount(raw);
  if (count > 0) rows.push(row('HBM', formatBytes(phys * MI355X.hbmBytes)));
  if (allocatable > 0 && !podsUnreadable) {
    rows.push(row('GPU Allocation', status(pctToStatus(p), inUse + '/' + allocatable + ' (' + p + '%)')));
  }
  // With the pod list unreadable (RBAC) the node's pods are unknown, not
  // absent: say so rather than "None" or an endless "Loading…".
  rows.push(
    row(
      'GPU Workload Pods',
      podsOnNode.length > 0
        ? podsOnNode.map(podName).join(', ')
        : podsUnreadable
          ? status('warning', 'Unavailable — the pod list could not be read')
          : loading ? 'Loading…' : 'None'
    )
  );
  let blocks = [kv(rows)];
  if (count > 0) {
    blocks.push(slotsBlock(raw, podsOnNode, own));
    blocks.push(matrixBlock(phys, xg, lk));
  }
  if (series) blocks = blocks.concat(powerHistoryBlocks(name, 'Node', series));
  return section('AMD GPU', blocks);
}

// ---------------------------------------------------------------------------
// Pod detail section (reference PodDetailSection.tsx:25-114)
// ---------------------------------------------------------------------------

/**
 * Self-contained (no store). Differences: init containers are listed too, so
 * an init-only GPU pod renders (reference quirk Q3), and the effective GPU
 * demand the scheduler uses is shown.
 */
export function podDetailView(resource, opts) {
  const raw = unwrapKubeObject(resource);
  const metrics = opts && opts.metrics ? opts.metrics : null;
  const series = opts && opts.series && opts.series.power && opts.series.power.length ? opts.series : null;
  if ((metrics || series) && raw && typeof raw === 'object' && raw.metadata) {
    // Live telemetry of the GPUs this pod holds (exporter pod labels), and
    // their power over the series window.
    const gs = metrics ? podGpuAssignments(metrics)[(raw.metadata.namespace || '') + '/' + raw.metadata.name] : undefined;
    if (gs || series) {
      return memo('pod-detail:' + (raw.metadata.uid || raw.metadata.namespace + '/' + raw.metadata.name), [raw, gs, series], function () {
        return podDetailSection(raw, gs, series);
      });
    }
  }
  if (podDetailCache && raw && typeof raw === 'object') {
    if (podDetailCache.has(raw)) return podDetailCache.get(raw);
    const s = podDetailSection(raw);
    podDetailCache.set(raw, s);
    return s;
  }
  return podDetailSection(raw);
}

/**
 * Blocks of a node's or pod's GPU power history: peak / average / energy over
 * the window and the sparkline row (`label` heads its first column).
 */
function powerHistoryBlocks(name, label, series) {
  const win = formatWindow(series.rangeSec || 1800);
  const byPod = {};
  byPod[name] = series.power;
  const st = clusterPowerStats(byPod);
  if (!st) return []; // no numeric sample in the window
  return [
    kv([
      row('Peak GPU Power (' + win + ')', formatWatts(st.peakWatts)),
      row('Average GPU Power (' + win + ')', formatWatts(st.avgWatts)),
      // Σ samples × query step: the energy the GPUs drew while observed.
      row('GPU Energy (' + win + ')', formatEnergy(seriesEnergyJoules(series.power, series.stepSec))),
    ]),
    { t: 'series', label: label, power: byPod, vram: {}, avgPower: seriesMeans(byPod) },
  ];
}

/**
 * Energy (J) of a power series [[t s, W]]; null with fewer than 2 samples.
 * With the range query's `stepSec` each sample holds for one step, so a gap
 * Prometheus left (an exporter restart) adds nothing instead of stretching
 * the step guessed from the first and last timestamps. Without it the
 * trapezoid rule runs over the real timestamps.
 */
export function seriesEnergyJoules(pts, stepSec) {
  if (!pts || pts.length < 2) return null;
  let sum = 0;
  if (stepSec > 0) {
    for (let i = 0; i < pts.length; i++) sum += pts[i][1];
    return sum * stepSec;
  }
  for (let i = 1; i < pts.length; i++) sum += ((pts[i][1] + pts[i - 1][1]) / 2) * (pts[i][0] - pts[i - 1][0]);
  return sum;
}

/** Joules → "x Wh" / "x kWh"; "—" when unknown. */
export function formatEnergy(joules) {
  if (joules === null || joules === undefined || !isFinite(joules)) return '—';
  const wh = joules / 3600;
  return wh >= 1000 ? (wh / 1000).toFixed(2) + ' kWh' : wh.toFixed(1) + ' Wh';
}

function podDetailSection(raw, assigned, series) {
  if (!isGpuRequestingPod(raw)) return null;
  const ics = gpuInitContainers(raw);
  const cs = gpuContainers(raw);
  const all = ics.map(function (c) { return [c, true]; }).concat(cs.map(function (c) { return [c, false]; }));
  if (all.length === 0) return null;
  const rows = [];
  for (let i = 0; i < all.length; i++) {
    const c = all[i][0];
    const cname = c.name + (all[i][1] ? ' (init)' : '');
    const es = containerGpuEntries(c);
    for (let j = 0; j < es.length; j++) {
      const res = formatGpuResourceName(es[j].key);
      rows.push(row(cname + ' → ' + res + ' request', es[j].request === null ? '—' : es[j].request));
      if (es[j].limit !== null && es[j].limit !== es[j].request) rows.push(row(cname + ' → ' + res + ' limit', es[j].limit));
    }
  }
  const phase = get(raw, ['status', 'phase'], null);
  const phaseStatus = phase === 'Running' || phase === 'Succeeded' ? 'success' : phase === 'Pending' ? 'warning' : 'error';
  const gpus = getPodGpuCount(raw);
  const whole = getPodGpuDemand(raw)[AMD_GPU_RESOURCE] === gpus;
  return section('AMD GPU Resources', [
    kv(
      [
        row('Phase', status(phaseStatus, phase || 'Unknown')),
        row('Scheduled Node', get(raw, ['spec', 'nodeName'], '—')),
        row('GPU Containers', String(all.length)),
        row(
          'GPUs (effective)',
          gpus === 0 ? '—'
            : whole ? gpus + ' × ' + MI355X.shortName + ' (' + formatBytes(gpus * MI355X.hbmBytes) + ' HBM)'
              : gpus + ' GPU device' + (gpus === 1 ? '' : 's') + ' (partitions)'
        ),
      ].concat(assigned ? [row('Assigned GPUs', assignedLines(assigned))] : []).concat(rows)
    ),
  ].concat(series ? powerHistoryBlocks(raw.metadata.name, 'Pod', series) : []));
}

// ---------------------------------------------------------------------------
// Nodes-table columns (reference integrations/NodeColumns.tsx:17-48)
// ---------------------------------------------------------------------------

/**
 * Column descriptors for the native `headlamp-nodes` table. Getters return
 * IR cells; the TSX wrapper turns status cells into StatusLabels.
 * Each getter unwraps and classifies the row once via a WeakMap cache, so
 * N columns cost one `isAmdGpuNode` per row (reference re-ran it per column).
 */
export function nodeColumns() {
  const cache = typeof WeakMap === 'function' ? new WeakMap() : null;
  function info(resource) {
    const key = resource && typeof resource === 'object' ? resource : null;
    if (cache && key && cache.has(key)) return cache.get(key);
    const raw = unwrapKubeObject(resource);
    const v = isAmdGpuNode(raw)
      ? { raw: raw, count: getNodeGpuCount(raw), physical: getNodePhysicalGpuCount(raw), model: getNodeGpuModel(raw) }
      : null;
    if (cache && key) cache.set(key, v);
    return v;
  }
  return [
    {
      label: 'GPU Model',
      getter: function (resource) {
        const i = info(resource);
        return i ? status('success', formatGpuModel(i.model)) : '—';
      },
    },
    {
      label: 'GPU Devices',
      getter: function (resource) {
        const i = info(resource);
        return i && i.count > 0 ? String(i.count) : '—';
      },
    },
    {
      label: 'GPU HBM',
      getter: function (resource) {
        const i = info(resource);
        return i && i.count > 0 ? formatBytes(i.physical * MI355X.hbmBytes) : '—';
      },
    },
  ];
}
