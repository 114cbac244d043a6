/**
 * Facts of the AMD GPU Operator's objects, derived once per object and read
 * by Overview and Device Plugins:
 *
 *   * deviceConfigFacts: a DeviceConfig's status (worst operand) and its
 *     device-plugin counts, image, each operand's row (enabled, version /
 *     port, its DaemonSet's ready / desired) and node selector — when the
 *     store takes the list (clusterStore.js build; a handful of objects);
 *   * operatorPodFacts: an operator pod's component, node, readiness and
 *     restarts — on first read: the pages show one page of the operator pods
 *     (three per GPU node: 3,000 on a 1,000-node cluster), so only the rows
 *     shown pay for them (ADR 015).
 *
 * Reference: the same derivations run on every render of its pages
 * (DevicePluginsPage.tsx:110-182, OverviewPage.tsx:222-272).
 */

import {
  countsToStatus,
  countsToText,
  deviceConfigStatus,
  deviceConfigStatusText,
  formatSelector,
  operandEnabled,
  operandStatus,
} from './amdNodes.js';
import { formatComponent, getPodRestarts, isPodReady, pluginPodComponent } from './amdPods.js';
import { get } from './k8sCore.js';

/** DeviceConfig operands of later AMD GPU Operator releases (`spec.<key>.enable`). */
export const EXTRA_OPERANDS = Object.freeze([
  { key: 'testRunner', label: 'Test Runner' },
  { key: 'configManager', label: 'Config Manager' },
]);

const dcCache = new WeakMap();
const podCache = new WeakMap();

/**
 * An operand's row: "Disabled", or "Enabled" (— its version / port) and, when
 * the DeviceConfig's status counts its DaemonSet, "· ready/desired", the
 * level set by the pods. {enabled, level, text}.
 */
function operandRow(dc, key, detail, counted) {
  if (!operandEnabled(dc, key)) return { enabled: false, level: 'warning', text: 'Disabled' };
  const head = detail ? 'Enabled — ' + detail : 'Enabled';
  if (!counted) return { enabled: true, level: 'success', text: head };
  const st = operandStatus(dc, key);
  return { enabled: true, level: countsToStatus(st.desired, st.available), text: head + ' · ' + countsToText(st.desired, st.available) };
}

/**
 * @returns {{level: string, text: string, namespace: string, image: string, plugin: {desired: number, available: number, unavailable: number},
 *   driver: object, nodeLabeller: object, metricsExporter: object, extra: Array<{label: string, enabled: boolean, level: string, text: string}>,
 *   selector: string}}
 */
export function deviceConfigFacts(dc) {
  let f = dcCache.get(dc);
  if (f) return f;
  const port = get(dc, ['spec', 'metricsExporter', 'port'], null);
  const extra = [];
  for (let k = 0; k < EXTRA_OPERANDS.length; k++) {
    const op = EXTRA_OPERANDS[k];
    if (get(dc, ['spec', op.key], null) === null) continue;
    extra.push(Object.assign({ label: op.label }, operandRow(dc, op.key, null, get(dc, ['status', op.key], null) !== null)));
  }
  f = {
    level: deviceConfigStatus(dc),
    text: deviceConfigStatusText(dc),
    namespace: (dc.metadata && dc.metadata.namespace) || '—',
    image: get(dc, ['spec', 'devicePlugin', 'devicePluginImage'], '—'),
    plugin: operandStatus(dc, 'devicePlugin'),
    driver: operandRow(dc, 'driver', get(dc, ['spec', 'driver', 'version'], null), true),
    nodeLabeller: operandRow(dc, 'nodeLabeller', null, true),
    metricsExporter: operandRow(dc, 'metricsExporter', port !== null ? 'port ' + port : null, true),
    extra: extra,
    selector: formatSelector(get(dc, ['spec', 'selector'], null)),
  };
  dcCache.set(dc, f);
  return f;
}

/** @returns {{component: string, node: string, ready: boolean, phase: string, restarts: number}} */
export function operatorPodFacts(p) {
  let f = podCache.get(p);
  if (f) return f;
  f = {
    component: formatComponent(pluginPodComponent(p)),
    node: get(p, ['spec', 'nodeName'], '—'),
    ready: isPodReady(p),
    phase: get(p, ['status', 'phase'], 'Unknown'),
    restarts: getPodRestarts(p),
  };
  podCache.set(p, f);
  return f;
}

/** Derive the facts of every DeviceConfig of a snapshot (once per object); operator pods' on first read. */
export function primeOperatorFacts(deviceConfigs) {
  for (let i = 0; i < deviceConfigs.length; i++) deviceConfigFacts(deviceConfigs[i]);
}
