/**
 * Device Plugins page view-model (reference
 * src/components/DevicePluginsPage.tsx:20-219, SURVEY C6): one card per AMD
 * GPU Operator DeviceConfig and one page of operator pods.
 */

import {
  countsToStatus,
  countsToText,
  deviceConfigStatus,
  deviceConfigStatusText,
  formatSelector,
  operandEnabled,
  operandStatus,
} from '../../api/amdNodes.js';
import { formatComponent, pluginPodComponent } from '../../api/amdPods.js';
import { get } from '../../api/k8sCore.js';
import { kv, loader, page, pager, row, section, status, table } from '../ir.js';
import {
  ageText,
  BRAND,
  chunkedRows,
  dpPluginRows,
  errorSection,
  memo,
  nowOf,
  podName,
  podNode,
  podNs,
  readyLabel,
  refreshButton,
  restartsCell,
  crdPending,
  pluginPodsPending,
} from './common.js';
import { podPage } from './paging.js';

/** DeviceConfig operands of later AMD GPU Operator releases (`spec.<key>.enable`). */
const EXTRA_OPERANDS = [
  { key: 'testRunner', label: 'Test Runner' },
  { key: 'configManager', label: 'Config Manager' },
];

/**
 * An operand's row: "Disabled", or "Enabled" (— its version / port) and, when
 * the DeviceConfig's status counts its DaemonSet, "· ready/desired" in the
 * same cell, coloured by the pods (one row per operand; the reference has no
 * operand rows, DevicePluginsPage.tsx:115-180).
 */
function operandCell(dc, key, detail, counted) {
  if (!operandEnabled(dc, key)) return status('warning', 'Disabled');
  const head = detail ? 'Enabled — ' + detail : 'Enabled';
  if (!counted) return status('success', head);
  const st = operandStatus(dc, key);
  return status(countsToStatus(st.desired, st.available), head + ' · ' + countsToText(st.desired, st.available));
}

/**
 * One card per DeviceConfig (reference: one per GpuDevicePlugin). Per-operand
 * DaemonSet counts replace the single desired/ready pair. The page needs no
 * node list and no all-namespaces pod list: its route (plugin.js PAGE_NEEDS)
 * mounts OperatorPodFeed, a list + watch of the operator namespace and one of
 * the device plugin / labeller labels elsewhere (providerCore.js), in the
 * same wave as the DeviceConfig request, so it renders whole after one round
 * trip on any cluster size. The plugin-pod requests (requests.js
 * PLUGIN_POD_QUERIES) stand in when both lists fail, or re-read on a timer
 * when the host ignores list selectors (ADR 012). Reference: a full-page
 * Loader until both cluster-wide lists and its four serial requests are in,
 * DevicePluginsPage.tsx:23-25, IntelGpuDataContext.tsx:98-165,214.
 */
export function devicePluginsView(ctx, opts) {
  const now = nowOf(opts);
  if (crdPending(ctx)) return page(null, null, [loader('Loading device plugin data...')]);
  const podsPend = pluginPodsPending(ctx);
  // One page of the operator pod table (PODS_PER_PAGE; filter on
  // namespace/name and node): three per GPU node on a real cluster.
  const pg = podPage(ctx.pluginPods, opts && opts.pager, 'plugin-pod');
  const items = memo(
    'device-plugins',
    [ctx.deviceConfigs, pg, ctx.crdAvailable, ctx.error, podsPend],
    function () { return devicePluginsItems(ctx, now, pg, podsPend); },
    now
  );
  return page(BRAND + ' — Device Plugins', refreshButton('Refresh device plugin data', ctx.refreshing), items);
}

function devicePluginsItems(ctx, now, pg, podsPend) {
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
      row('Driver', operandCell(dc, 'driver', get(dc, ['spec', 'driver', 'version'], null), true)),
      row('Node Labeller', operandCell(dc, 'nodeLabeller', null, true)),
      row(
        'Metrics Exporter',
        operandCell(dc, 'metricsExporter',
          get(dc, ['spec', 'metricsExporter', 'port'], null) !== null ? 'port ' + get(dc, ['spec', 'metricsExporter', 'port'], '') : null, true)
      ),
      row('Desired Nodes', String(dp.desired)),
      row('Ready Nodes', String(dp.available)),
    ];
    if (dp.unavailable > 0) rows.push(row('Unavailable Nodes', status('error', dp.unavailable)));
    // Later operator releases' operands (GPU test runner, partition config
    // manager): shown when the DeviceConfig names them, their DaemonSet
    // counts when its status reports them.
    for (let k = 0; k < EXTRA_OPERANDS.length; k++) {
      const op = EXTRA_OPERANDS[k];
      if (get(dc, ['spec', op.key], null) === null) continue;
      rows.push(row(op.label, operandCell(dc, op.key, null, get(dc, ['status', op.key], null) !== null)));
    }
    rows.push(row('Node Selector', formatSelector(get(dc, ['spec', 'selector'], null))));
    rows.push(row('Age', ageText(dc.metadata.creationTimestamp, now)));
    items.push(section('DeviceConfig: ' + dc.metadata.name, [kv(rows)], dc.metadata.uid || dc.metadata.name));
  }

  if (podsPend) {
    items.push(loader('Loading operator pods...'));
  } else if (ctx.pluginPods.length > 0) {
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
