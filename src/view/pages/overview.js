/**
 * Overview page view-model (reference src/components/OverviewPage.tsx:54-420,
 * SURVEY C5).
 */

import { formatPodGpuRequests, isPodReady } from '../../api/amdPods.js';
import { nodeFacts, podFacts } from '../../api/clusterIndex.js';
import { AMD_GPU_OPERATOR_NAMESPACE, BAR_COLORS, formatBytes, MI355X } from '../../api/k8sCore.js';
import { assignmentTexts, podGpuAssignments } from '../../api/nodeSummaries.js';
import { deviceConfigFacts, operatorPodFacts } from '../../api/operatorFacts.js';
import { SMALL_CLUSTER_NODES } from '../../api/series.js';
import { kv, loader, page, pctbar, row, section, status, table } from '../ir.js';
import {
  ageText,
  BRAND,
  chunkedFilter,
  chunkedRows,
  errorSection,
  memo,
  nowOf,
  ovPluginRows,
  podName,
  podNode,
  podNs,
  refreshButton,
  crdPending,
  nodesPending,
  PODS_LOADING,
  pluginPodsPending,
  podsPending,
} from './common.js';

export const ACTIVE_PODS_LIMIT = 10;

export const HELM_INSTALL =
  'helm repo add rocm https://rocm.github.io/gpu-operator && ' +
  'helm install amd-gpu-operator rocm/gpu-operator-charts --namespace ' + AMD_GPU_OPERATOR_NAMESPACE + ' --create-namespace';

export const OPERATOR_DOCS = 'https://instinct.docs.amd.com/projects/gpu-operator/';

/**
 * Differences: the loader only replaces the page on the FIRST load — later
 * refreshes keep the data (stale-while-revalidate). It waits for the node
 * list only: the node and capacity sections render while the DeviceConfig
 * request (up to its timeout when the CRD is slow or absent) and the
 * all-namespaces pod list (tens of MB on a large cluster) are still out; the
 * DeviceConfig section and the pod-derived ones (in use, workloads, active
 * pods, operator pods) show a loader until theirs is in — the reference
 * shows a full-page Loader until every list is in (OverviewPage.tsx:67-69,
 * IntelGpuDataContext.tsx:214). Aggregates come from the store's memoised
 * index. In-use counts GPUs held by bound, non-terminated pods (the
 * scheduler's view), and Free is clamped at 0. On a cluster of more than one
 * page of GPU nodes, `opts.metrics` (the exporter's owner answer,
 * overviewOwnersScope) shows the pods drawing the most power while the pod
 * list is still on its way (ADR 013).
 */
export function overviewView(ctx, opts) {
  const now = nowOf(opts);
  if (nodesPending(ctx)) return page(null, null, [loader('Loading ' + BRAND + ' data...')]);
  const podsPend = podsPending(ctx);
  const opPend = pluginPodsPending(ctx);
  const crdPend = crdPending(ctx);
  const owners = podsPend && opts && opts.metrics && Array.isArray(opts.metrics.gpus) ? opts.metrics : null;
  const items = memo(
    'overview',
    [ctx.deviceConfigs, ctx.pluginPods, ctx.pluginInstalled, ctx.crdAvailable, ctx.gpuNodes, ctx.gpuPods, ctx.index, ctx.error, podsPend, opPend,
      crdPend, owners && owners.gpus],
    function () { return overviewItems(ctx, now, podsPend, opPend, owners, crdPend); },
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
    const k = nodeFacts(gpuNodes[i]).partitionMode;
    if (!(k in counts)) {
      counts[k] = 0;
      order.push(k);
    }
    counts[k]++;
  }
  return order.map(function (k, i) { return { name: k, value: counts[k], fill: MODE_COLORS[i % MODE_COLORS.length] }; });
}

/**
 * Overview's exporter query (plugin.js OverviewPage): only while a cluster
 * of more than one page of GPU nodes has its node list and not yet its pod
 * list. The owner answer shows the pods drawing the most power until the list
 * is in (overviewPodsPreview). A smaller cluster's pod list comes in the first
 * wave with its nodes: the page sends no Prometheus request there.
 * @returns {{enabled: boolean, pods?: string[], small?: boolean, preview?: number}}
 */
export function overviewOwnersScope(ctx) {
  if (!ctx || ctx.nodesState !== 'ready' || !podsPending(ctx) || !ctx.gpuNodes || ctx.gpuNodes.length <= SMALL_CLUSTER_NODES) {
    return { enabled: false };
  }
  return { enabled: true, pods: [], small: true, preview: ACTIVE_PODS_LIMIT };
}

/**
 * The pods holding GPUs as the exporter's owner answer names them, while
 * the pod list loads: the ACTIVE_PODS_LIMIT drawing the most power on a
 * cluster with more owners than that (the answer's preview ranking), else
 * every owner in namespace / name order. Null without owners.
 */
export function overviewPodsPreview(metrics) {
  if (!metrics || !Array.isArray(metrics.gpus)) return null;
  const assign = podGpuAssignments(metrics);
  const pv = metrics.preview;
  return memo('overview-preview', [assign, pv], function () {
    const keys = (pv && Array.isArray(pv.order) ? pv.order.filter(function (k) { return assign[k]; })
      : Object.keys(assign).sort()).slice(0, ACTIVE_PODS_LIMIT);
    if (!keys.length) return null;
    const count = pv ? pv.count : Object.keys(assign).length;
    return section(pv ? 'GPU Pods Drawing the Most Power (partial)' : 'GPU Pods (partial)', [
      kv([
        row('Status', status('warning', 'Partial — the pod list is loading; these rows come from the GPU exporter')),
        row('Pods Holding GPUs', String(count)),
      ]),
      table(['Name', 'Namespace', 'Assigned GPUs', 'GPU Power'], keys.map(function (k) {
        const slash = k.indexOf('/');
        const t = assignmentTexts(assign[k]);
        return [k.slice(slash + 1), k.slice(0, slash) || '—', t.assigned, t.power];
      }), keys),
    ]);
  });
}

function overviewItems(ctx, now, podsPend, opPend, owners, crdPend) {
  const items = [];
  const t = ctx.index.totals;

  if (ctx.error) items.push(errorSection(ctx.error));

  // Operator pods come from the pod list (or the plugin-pod requests), the
  // DeviceConfigs from their request: while either loads, "not detected" is
  // not known yet.
  if (!ctx.pluginInstalled && !opPend && !crdPend) {
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

  if (crdPend) {
    items.push(loader('Loading DeviceConfigs...'));
  } else if (!ctx.crdAvailable && ctx.pluginInstalled) {
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
  if (podsPend) {
    // Capacity is known from the nodes; what is in use needs the pods.
    if (t.capacity > 0) items.push(memo('overview-alloc-nodes', [t], function () { return overviewCapacity(t); }));
    const preview = owners ? overviewPodsPreview(owners) : null;
    if (preview) items.push(preview);
    items.push(loader('Loading GPU pods...'));
    return items;
  }
  if (t.capacity > 0) items.push(memo('overview-alloc', [t], function () { return overviewAllocation(t); }));
  const ph = ctx.index.phases;
  items.push(memo('overview-workloads', [ph, ctx.gpuPods.length], function () { return overviewWorkloads(ph, ctx.gpuPods.length); }));
  const active = memo('overview-active', [ctx.gpuPods], function () { return overviewActivePods(ctx.gpuPods, now); }, now);
  if (active) items.push(active);
  return items;
}

const ENABLED = status('success', 'Enabled');
const DISABLED = status('warning', 'Disabled');
const READY = status('success', 'Ready');

function overviewDeviceConfigs(dcs, now) {
  return section('Device Config Status', [
    table(
      ['Name', 'Namespace', 'Status', 'Metrics Exporter', 'Node Labeller', 'Selector', 'Age'],
      dcs.map(function (dc) {
        // Derived when the store took the list (api/operatorFacts.js).
        const f = deviceConfigFacts(dc);
        return [
          dc.metadata.name,
          f.namespace,
          status(f.level, f.text),
          f.metricsExporter.enabled ? ENABLED : DISABLED,
          f.nodeLabeller.enabled ? ENABLED : DISABLED,
          f.selector,
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
  // Readiness of every pod (the not-ready count), the other facts of the rows shown only.
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
          const f = operatorPodFacts(p);
          return [podName(p), podNs(p), f.component, f.node, f.ready ? READY : status('warning', f.phase), ageText(p.metadata.creationTimestamp, now)];
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

/** GPU Allocation before the pod list is in: the node-side figures, In Use pending. */
function overviewCapacity(t) {
  return section('GPU Allocation', [
    kv([
      row('Total Capacity (GPU devices)', String(t.capacity)),
      row('Allocatable', String(t.allocatable)),
      row('In Use', PODS_LOADING),
    ]),
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
