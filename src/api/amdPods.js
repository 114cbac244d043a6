/**
 * GPU pods and operator pods: which pods request amd.com/* (init containers
 * included), their effective GPU demand (the scheduler's rule:
 * max(Σ app containers, max init container), limits for limits-only
 * extended resources), readiness, restarts, waiting reason, and the AMD GPU
 * Operator's own pods by component. Pure, I/O-free.
 *
 * Reference: src/api/k8s.ts:209-309 (C2.8-C2.11; quirks Q3, Q4).
 */

import { isDeviceResource } from './amdNodes.js';
import {
  AMD_DEVICE_PLUGIN_POD_LABEL,
  AMD_GPU_OPERATOR_NAMESPACE,
  AMD_NODE_LABELLER_POD_LABEL,
  AMD_RESOURCE_PREFIX,
  formatGpuResourceName,
  get,
  isNamedObject,
  labelsOf,
  parseCount,
} from './k8sCore.js';

const NO_RESOURCES = Object.freeze({});

/** A container's `resources.requests` / `resources.limits` map, or an empty one. */
function resourcesOf(c, which) {
  const r = c !== null && typeof c === 'object' ? c.resources : undefined;
  const m = r !== null && typeof r === 'object' ? r[which] : undefined;
  return m !== null && typeof m === 'object' ? m : NO_RESOURCES;
}

/** The container's `amd.com/*` resource names: requested ones first, then limits-only ones. */
function containerAmdKeys(c) {
  const req = resourcesOf(c, 'requests');
  const lim = resourcesOf(c, 'limits');
  const keys = [];
  for (const k in req) if (k.indexOf(AMD_RESOURCE_PREFIX) === 0 && hasOwn.call(req, k)) keys.push(k);
  for (const k in lim) if (k.indexOf(AMD_RESOURCE_PREFIX) === 0 && hasOwn.call(lim, k) && !hasOwn.call(req, k)) keys.push(k);
  return keys;
}

const hasOwn = Object.prototype.hasOwnProperty;

/** `res` (requests or limits) names an `amd.com/*` resource — no allocation (runs on every pod of the cluster). */
function hasAmdKey(res) {
  if (res === null || typeof res !== 'object') return false;
  for (const k in res) {
    if (k.indexOf(AMD_RESOURCE_PREFIX) === 0 && hasOwn.call(res, k)) return true;
  }
  return false;
}

/** containerAmdKeys(c).length > 0, without building the list. */
function containerHasAmd(c) {
  const r = c !== null && typeof c === 'object' ? c.resources : undefined;
  if (r === null || typeof r !== 'object') return false;
  return hasAmdKey(r.requests) || hasAmdKey(r.limits);
}

/**
 * True if any container, init or regular, requests or limits an `amd.com/*`
 * resource. This is the classification every pod of the cluster goes
 * through when the pod list arrives (37k pods at 1,000 nodes), so it reads
 * the containers directly and allocates nothing.
 */
export function isGpuRequestingPod(pod) {
  if (!isNamedObject(pod)) return false;
  const spec = pod.spec;
  if (spec === null || typeof spec !== 'object') return false;
  const cs = spec.containers;
  if (cs !== null && cs !== undefined) for (let i = 0; i < cs.length; i++) if (containerHasAmd(cs[i])) return true;
  const ics = spec.initContainers;
  if (ics !== null && ics !== undefined) for (let i = 0; i < ics.length; i++) if (containerHasAmd(ics[i])) return true;
  return false;
}

export function filterGpuRequestingPods(items) {
  const out = [];
  if (!Array.isArray(items)) return out;
  for (let i = 0; i < items.length; i++) if (isGpuRequestingPod(items[i])) out.push(items[i]);
  return out;
}

/** Containers (regular only) that carry an AMD resource — for per-container displays. */
export function gpuContainers(pod) {
  const cs = get(pod, ['spec', 'containers'], []);
  const out = [];
  for (let i = 0; i < cs.length; i++) if (containerHasAmd(cs[i])) out.push(cs[i]);
  return out;
}

/** Init containers that carry an AMD resource. */
export function gpuInitContainers(pod) {
  const cs = get(pod, ['spec', 'initContainers'], []);
  const out = [];
  for (let i = 0; i < cs.length; i++) if (containerHasAmd(cs[i])) out.push(cs[i]);
  return out;
}

/**
 * Per-container AMD demand. For extended resources Kubernetes defaults the
 * request to the limit, so a limits-only container still consumes devices.
 * @returns {Array<{ key: string, request: string|null, limit: string|null, effective: number }>}
 */
export function containerGpuEntries(c) {
  const req = resourcesOf(c, 'requests');
  const lim = resourcesOf(c, 'limits');
  const keys = containerAmdKeys(c);
  const out = [];
  for (let i = 0; i < keys.length; i++) {
    const k = keys[i];
    const r = req[k] !== undefined ? String(req[k]) : null;
    const l = lim[k] !== undefined ? String(lim[k]) : null;
    out.push({ key: k, request: r, limit: l, effective: parseCount(r !== null ? r : l) });
  }
  return out;
}

function addInto(acc, c) {
  const es = containerGpuEntries(c);
  for (let i = 0; i < es.length; i++) acc[es[i].key] = (acc[es[i].key] || 0) + es[i].effective;
}

/**
 * Effective pod demand per AMD resource using the scheduler's rule:
 *   max( Σ regular + Σ sidecars, max_i(init_i + Σ sidecars started before i) ).
 * Sidecars are init containers with `restartPolicy: Always`.
 * @returns {Record<string, number>}
 */
export function getPodGpuDemand(pod) {
  const regular = {};
  const cs = get(pod, ['spec', 'containers'], []);
  for (let i = 0; i < cs.length; i++) addInto(regular, cs[i]);
  const ics = get(pod, ['spec', 'initContainers'], []);
  const sidecars = {};
  const initPeak = {};
  for (let i = 0; i < ics.length; i++) {
    const c = ics[i];
    const own = {};
    addInto(own, c);
    if (c && c.restartPolicy === 'Always') {
      for (const k in own) sidecars[k] = (sidecars[k] || 0) + own[k];
    } else {
      for (const k in own) {
        const v = own[k] + (sidecars[k] || 0);
        if (v > (initPeak[k] || 0)) initPeak[k] = v;
      }
    }
  }
  const out = {};
  const keys = Object.keys(Object.assign({}, regular, sidecars, initPeak));
  for (let i = 0; i < keys.length; i++) {
    const k = keys[i];
    const steady = (regular[k] || 0) + (sidecars[k] || 0);
    const v = Math.max(steady, initPeak[k] || 0);
    if (v > 0) out[k] = v;
  }
  return out;
}

/** GPU devices the pod holds: `amd.com/gpu` plus partition resources. */
export function getPodGpuCount(pod) {
  const d = getPodGpuDemand(pod);
  let n = 0;
  for (const k in d) if (isDeviceResource(k)) n += d[k];
  return n;
}

/** String map of the pod's effective AMD demand (API-compatible with the reference's requests map). */
export function getPodGpuRequests(pod) {
  const d = getPodGpuDemand(pod);
  const out = {};
  for (const k in d) out[k] = String(d[k]);
  return out;
}

/** `amd.com/gpu: 2, amd.com/cpx_nps4: 1` → "GPU: 2, GPU partition (CPX/NPS4): 1". */
export function formatPodGpuRequests(pod) {
  const d = getPodGpuDemand(pod);
  const parts = [];
  for (const k in d) parts.push(formatGpuResourceName(k) + ': ' + d[k]);
  return parts.length ? parts.join(', ') : '—';
}

export function isPodReady(pod) {
  const conds = get(pod, ['status', 'conditions'], []);
  if (!Array.isArray(conds)) return false;
  for (let i = 0; i < conds.length; i++) {
    if (conds[i] && conds[i].type === 'Ready' && conds[i].status === 'True') return true;
  }
  return false;
}

export function getPodRestarts(pod) {
  const st = get(pod, ['status', 'containerStatuses'], []);
  let n = 0;
  for (let i = 0; i < st.length; i++) n += (st[i] && typeof st[i].restartCount === 'number') ? st[i].restartCount : 0;
  return n;
}

export function podPhase(pod) {
  return get(pod, ['status', 'phase'], 'Unknown');
}

/** First waiting reason across init and regular container statuses. */
export function podWaitingReason(pod) {
  const lists = [get(pod, ['status', 'initContainerStatuses'], []), get(pod, ['status', 'containerStatuses'], [])];
  for (let j = 0; j < lists.length; j++) {
    for (let i = 0; i < lists[j].length; i++) {
      const r = get(lists[j][i], ['state', 'waiting', 'reason'], null);
      if (r) return r;
    }
  }
  // Unschedulable pods have no container statuses; the scheduler sets a condition instead.
  const conds = get(pod, ['status', 'conditions'], []);
  for (let i = 0; i < conds.length; i++) {
    if (conds[i] && conds[i].type === 'PodScheduled' && conds[i].status === 'False' && conds[i].reason) {
      return conds[i].reason;
    }
  }
  return null;
}

/**
 * The message behind podWaitingReason: the scheduler's explanation of an
 * unschedulable pod ("0/8 nodes are available: 8 Insufficient amd.com/gpu.")
 * or the kubelet's for a waiting container (image pull errors, …). Null when
 * there is none.
 */
export function podWaitingMessage(pod) {
  const lists = [get(pod, ['status', 'initContainerStatuses'], []), get(pod, ['status', 'containerStatuses'], [])];
  for (let j = 0; j < lists.length; j++) {
    for (let i = 0; i < lists[j].length; i++) {
      if (get(lists[j][i], ['state', 'waiting', 'reason'], null)) return get(lists[j][i], ['state', 'waiting', 'message'], null);
    }
  }
  const conds = get(pod, ['status', 'conditions'], []);
  for (let i = 0; i < conds.length; i++) {
    if (conds[i] && conds[i].type === 'PodScheduled' && conds[i].status === 'False' && conds[i].reason) {
      return conds[i].message || null;
    }
  }
  return null;
}

/** Running/Succeeded → success, Pending/unknown → warning, Failed → error (reference PodsPage.tsx:30-43). */
export function phaseToStatus(phase) {
  switch (phase) {
    case 'Running':
    case 'Succeeded':
      return 'success';
    case 'Failed':
      return 'error';
    default:
      return 'warning';
  }
}

/**
 * Which operator operand a pod belongs to, or null if it is not an AMD GPU
 * infrastructure pod. Standalone DaemonSets are matched on their `name=`
 * label; operator-managed operands on their namespace + name pattern.
 * @returns {'device-plugin'|'node-labeller'|'metrics-exporter'|'driver'|'operator'|null}
 */
export function pluginPodComponent(pod) {
  if (!isNamedObject(pod)) return null;
  const labels = labelsOf(pod);
  if (labels.name === AMD_DEVICE_PLUGIN_POD_LABEL) return 'device-plugin';
  if (labels.name === AMD_NODE_LABELLER_POD_LABEL) return 'node-labeller';
  const appName = labels['app.kubernetes.io/name'] || labels.app || '';
  if (/amd-gpu-operator|gpu-operator-charts/.test(appName)) return 'operator';
  if (pod.metadata.namespace !== AMD_GPU_OPERATOR_NAMESPACE) return null;
  const name = String(pod.metadata.name || '');
  if (/device-plugin/.test(name)) return 'device-plugin';
  if (/node-labeller/.test(name)) return 'node-labeller';
  if (/metrics-exporter/.test(name)) return 'metrics-exporter';
  if (/kmm|driver/.test(name)) return 'driver';
  if (/operator/.test(name)) return 'operator';
  return null;
}

export function isAmdGpuPluginPod(pod) {
  return pluginPodComponent(pod) !== null;
}

export function filterAmdGpuPluginPods(items) {
  const out = [];
  if (!Array.isArray(items)) return out;
  for (let i = 0; i < items.length; i++) if (isAmdGpuPluginPod(items[i])) out.push(items[i]);
  return out;
}

/**
 * Dedupe plugin pods found by several queries. Keyed by uid, falling back
 * to namespace/name so uid-less fixtures are kept (fixes reference Q5).
 */
export function dedupePods(pods) {
  const uids = new Set();
  const names = new Set();
  const out = [];
  for (let i = 0; i < pods.length; i++) {
    const m = pods[i].metadata || {};
    if (m.uid) {
      if (uids.has(m.uid)) continue;
      uids.add(m.uid);
    } else {
      const key = (m.namespace || '') + '/' + (m.name || '');
      if (names.has(key)) continue;
      names.add(key);
    }
    out.push(pods[i]);
  }
  return out;
}

const COMPONENT_LABEL = {
  'device-plugin': 'Device Plugin',
  'node-labeller': 'Node Labeller',
  'metrics-exporter': 'Metrics Exporter',
  driver: 'Driver',
  operator: 'Operator',
};

export function formatComponent(c) {
  return COMPONENT_LABEL[c] || '—';
}
