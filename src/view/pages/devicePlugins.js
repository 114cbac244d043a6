/**
 * Device Plugins page view-model (reference
 * src/components/DevicePluginsPage.tsx:20-219, SURVEY C6): one card per AMD
 * GPU Operator DeviceConfig and one page of operator pods.
 */

import { deviceConfigFacts, operatorPodFacts } from '../../api/operatorFacts.js';
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
  podNs,
  refreshButton,
  crdPending,
  pluginPodsPending,
} from './common.js';
import { podPage } from './paging.js';

const READY = status('success', 'Ready');

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
    // Derived when the store took the list (api/operatorFacts.js).
    const f = deviceConfigFacts(dc);
    const rows = [
      row('Status', status(f.level, f.text)),
      row('Namespace', f.namespace),
      row('Device Plugin Image', f.image),
      row('Driver', status(f.driver.level, f.driver.text)),
      row('Node Labeller', status(f.nodeLabeller.level, f.nodeLabeller.text)),
      row('Metrics Exporter', status(f.metricsExporter.level, f.metricsExporter.text)),
      row('Desired Nodes', String(f.plugin.desired)),
      row('Ready Nodes', String(f.plugin.available)),
    ];
    if (f.plugin.unavailable > 0) rows.push(row('Unavailable Nodes', status('error', f.plugin.unavailable)));
    // Later operator releases' operands (GPU test runner, partition config
    // manager): shown when the DeviceConfig names them, their DaemonSet
    // counts when its status reports them.
    for (let k = 0; k < f.extra.length; k++) rows.push(row(f.extra[k].label, status(f.extra[k].level, f.extra[k].text)));
    rows.push(row('Node Selector', f.selector));
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
              const f = operatorPodFacts(p);
              return [
                podName(p), podNs(p), f.component, f.node, f.ready ? READY : status('warning', f.phase),
                f.restarts > 0 ? status('warning', f.restarts) : String(f.restarts), ageText(p.metadata.creationTimestamp, now),
              ];
            }, now);
          }, now)
        ),
      ])
    );
  }

  return items;
}
