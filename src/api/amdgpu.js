/**
 * AMD Instinct MI355X domain model — pure, I/O-free.
 *
 * Everything the plugin knows about AMD GPUs in Kubernetes lives here:
 * resource names, the AMD GPU Operator `DeviceConfig` CRD, node-labeller /
 * NFD labels, pod accounting, xGMI platform facts, formatters and status
 * mappers. All inputs arriving from the API server are `unknown` and are
 * narrowed with `is*` guards at this boundary.
 *
 * Parity map (reference = privilegedescalation/headlamp-intel-gpu-plugin):
 *   constants            src/api/k8s.ts:13-31      (C2.1)
 *   CRD model + guard    src/api/k8s.ts:56-86      (C2.3)
 *   node detection       src/api/k8s.ts:125-156    (C2.5)
 *   resource extraction  src/api/k8s.ts:159-180    (C2.6)
 *   GPU "type"           src/api/k8s.ts:183-203    (C2.7) → product model
 *   pod detection        src/api/k8s.ts:250-268    (C2.9)
 *   plugin-pod detection src/api/k8s.ts:271-286    (C2.10)
 *   pod aggregation      src/api/k8s.ts:289-309    (C2.11)
 *   list envelope        src/api/k8s.ts:315-323    (C2.12)
 *   readiness            src/api/k8s.ts:329-331    (C2.13)
 *   formatters           src/api/k8s.ts:337-364    (C2.14)
 *   status mapping       src/api/k8s.ts:370-386    (C2.15)
 *
 * Deliberate departures from the reference (SURVEY.md §7.3, Appendix A):
 *   - Pod GPU demand follows the Kubernetes effective-request rule
 *     (max(Σ app + Σ sidecar, max init)) and falls back to limits for
 *     extended resources (Q3, Q4).
 *   - Node allocation counts GPUs, not pods (Q2); "free" is clamped (Q10).
 *
 * Written as ES2019 (no `?.` / `??`) so it runs unchanged under the Node 12
 * test runner in this repo and under Headlamp's vite build.
 *
 * Label / CRD names marked (verify) come from the AMD GPU Operator and
 * k8s-device-plugin manifests and must be re-checked against the deployed
 * operator version; they are centralised here so that is a one-line change.
 */

// ---------------------------------------------------------------------------
// Constants
// ---------------------------------------------------------------------------

/** AMD GPU Operator CRD (verify: amd.com/v1alpha1 DeviceConfig, namespaced). */
export const AMD_GPU_OPERATOR_API_GROUP = 'amd.com';
export const AMD_GPU_OPERATOR_API_VERSION = 'v1alpha1';
export const DEVICE_CONFIG_KIND = 'DeviceConfig';
export const DEVICE_CONFIG_PLURAL = 'deviceconfigs';
export const DEVICE_CONFIG_LIST_PATH =
  '/apis/' + AMD_GPU_OPERATOR_API_GROUP + '/' + AMD_GPU_OPERATOR_API_VERSION + '/' + DEVICE_CONFIG_PLURAL;

/** Whole-GPU extended resource advertised by the AMD k8s device plugin. */
export const AMD_GPU_RESOURCE = 'amd.com/gpu';
/** Every AMD extended resource shares this prefix (partition resources too). */
export const AMD_RESOURCE_PREFIX = 'amd.com/';
/**
 * Partition resources exposed with the device plugin's "mixed" naming
 * strategy, e.g. `amd.com/cpx_nps4` (verify per operator release).
 */
export const AMD_PARTITION_RESOURCE_RE = /^amd\.com\/(spx|dpx|qpx|cpx)_(nps[1-8])$/;

/** Label set by the GPU Operator's Node Feature Discovery rule. */
export const AMD_NFD_GPU_LABEL = 'feature.node.kubernetes.io/amd-gpu';
/** Node-labeller labels (verify: `amd.com/gpu.<prop>`, legacy `beta.amd.com/gpu.<prop>`). */
export const AMD_LABELLER_PREFIX = 'amd.com/gpu.';
export const AMD_LABELLER_LEGACY_PREFIX = 'beta.amd.com/gpu.';
export const LABEL_PRODUCT_NAME = 'amd.com/gpu.product-name';
export const LABEL_FAMILY = 'amd.com/gpu.family';
export const LABEL_DEVICE_ID = 'amd.com/gpu.device-id';
export const LABEL_VRAM = 'amd.com/gpu.vram';
export const LABEL_CU_COUNT = 'amd.com/gpu.cu-count';
export const LABEL_DRIVER_VERSION = 'amd.com/gpu.driver-version';
export const LABEL_COMPUTE_PARTITION = 'amd.com/compute-partitioning-mode';
export const LABEL_MEMORY_PARTITION = 'amd.com/memory-partitioning-mode';

/** Namespace the AMD GPU Operator deploys its operands into (verify). */
export const AMD_GPU_OPERATOR_NAMESPACE = 'kube-amd-gpu';
/** `name=` pod labels of the standalone k8s-device-plugin DaemonSets (verify). */
export const AMD_DEVICE_PLUGIN_POD_LABEL = 'amdgpu-dp-ds';
export const AMD_NODE_LABELLER_POD_LABEL = 'amdgpu-labeller-ds';

/**
 * Plugin-pod discovery requests. Issued in PARALLEL by the data layer
 * (the reference issues its three selectors serially,
 * src/api/IntelGpuDataContext.tsx:155-165). One set-based selector replaces
 * two equality selectors.
 */
export const PLUGIN_POD_QUERIES = [
  '/api/v1/pods?labelSelector=' +
    encodeURIComponent('name in (' + AMD_DEVICE_PLUGIN_POD_LABEL + ',' + AMD_NODE_LABELLER_POD_LABEL + ')'),
  '/api/v1/namespaces/' + AMD_GPU_OPERATOR_NAMESPACE + '/pods',
];

/** MI355X platform facts (MI355X_MICROARCH.md chip-level table). */
export const MI355X = Object.freeze({
  product: 'AMD Instinct MI355X',
  shortName: 'MI355X',
  arch: 'gfx950 (CDNA4)',
  hbmBytes: 294896 * 1024 * 1024, // 288 GiB HBM3E less 16 MiB: what the device reports (amd-smi total_vram 294896 MB)
  hbmLabel: '288 GB HBM3E',
  hbmPeakTBs: 8.0,
  computeUnits: 256,
  xcds: 8,
  gpusPerNode: 8,
  xgmiLinksPerGpu: 7,
  xgmiLinkGBs: 153,
  tdpWatts: 1400,
  // Junction (hotspot) throttle threshold: amd-smi slowdown_hotspot_temperature
  // on an MI355X (tests/fixtures/mi355x/amd_smi_static.json).
  junctionSlowdownC: 100,
});

/** Allocation / power colour thresholds (reference NodesPage.tsx:38, MetricsPage.tsx:52-53). */
export const WARN_PCT = 70;
export const ERROR_PCT = 90;

// ---------------------------------------------------------------------------
// Small generic helpers
// ---------------------------------------------------------------------------

/** @param {unknown} v @returns {v is Record<string, unknown>} */
export function isObject(v) {
  return v !== null && typeof v === 'object' && !Array.isArray(v);
}

const optString = function (v) { return v === undefined || v === null || typeof v === 'string'; };

/**
 * A Kubernetes object the views can name: metadata with a non-empty string
 * name, and a namespace / uid that are strings when present. What fails this
 * (a half-written object, a wrong-shaped watch event) is never classified as
 * a GPU node, GPU pod, operator pod or DeviceConfig, so no page renders its
 * name — a view never hands React an object where it expects text.
 */
export function isNamedObject(v) {
  if (!isObject(v) || !isObject(v.metadata)) return false;
  const m = v.metadata;
  return typeof m.name === 'string' && m.name !== '' && optString(m.namespace) && optString(m.uid);
}

/** Safe nested getter: get(obj, ['a','b']) without optional chaining. */
export function get(obj, path, dflt) {
  let cur = obj;
  for (let i = 0; i < path.length; i++) {
    if (cur === null || cur === undefined || typeof cur !== 'object') return dflt;
    cur = cur[path[i]];
  }
  return cur === undefined || cur === null ? dflt : cur;
}

/** Parse a Kubernetes integer quantity ("8", "8k" is not valid for devices). */
export function parseCount(v) {
  if (v === undefined || v === null) return 0;
  const n = parseInt(String(v), 10);
  return isFinite(n) && n > 0 ? n : 0;
}

/** Headlamp `useList()` returns KubeObject wrappers that keep raw JSON in `.jsonData`. */
export function unwrapKubeObject(item) {
  if (item && typeof item === 'object' && 'jsonData' in item && item.jsonData && typeof item.jsonData === 'object') {
    return item.jsonData;
  }
  return item;
}

export function unwrapAll(items) {
  if (!Array.isArray(items)) return [];
  const out = new Array(items.length);
  for (let i = 0; i < items.length; i++) out[i] = unwrapKubeObject(items[i]);
  return out;
}

function labelsOf(obj) {
  const l = get(obj, ['metadata', 'labels'], null);
  return isObject(l) ? l : {};
}

// ---------------------------------------------------------------------------
// List envelope
// ---------------------------------------------------------------------------

/** @returns {boolean} true for `{ items: [...] }` list responses. */
export function isKubeList(value) {
  return isObject(value) && Array.isArray(value.items);
}

// ---------------------------------------------------------------------------
// DeviceConfig CRD (AMD GPU Operator)
// ---------------------------------------------------------------------------

/**
 * @typedef {{ nodesMatchingSelectorNumber?: number, desiredNumber?: number, availableNumber?: number }} OperandStatus
 * @typedef {{ metadata: { name: string, namespace?: string, uid?: string, creationTimestamp?: string },
 *             spec?: Record<string, any>, status?: Record<string, any>, kind?: string }} DeviceConfig
 */

export function isDeviceConfig(value) {
  return isNamedObject(value) && value.kind === DEVICE_CONFIG_KIND;
}

/** Operand components the operator manages, in display order. */
export const OPERANDS = [
  { key: 'devicePlugin', label: 'Device Plugin' },
  { key: 'nodeLabeller', label: 'Node Labeller' },
  { key: 'metricsExporter', label: 'Metrics Exporter' },
  { key: 'driver', label: 'Driver' },
];

/**
 * Whether an operand is enabled in the DeviceConfig spec. The device plugin is
 * always deployed; the labeller hangs off `spec.devicePlugin.enableNodeLabeller`
 * and other operands off `spec.<operand>.enable` (verify per operator release).
 */
export function operandEnabled(dc, key) {
  if (key === 'devicePlugin') return true;
  if (key === 'nodeLabeller') return get(dc, ['spec', 'devicePlugin', 'enableNodeLabeller'], false) === true;
  return get(dc, ['spec', key, 'enable'], false) === true;
}

/**
 * Normalised operand status {desired, available, unavailable, matching}.
 * `status.<operand>` has {nodesMatchingSelectorNumber, desiredNumber, availableNumber}.
 */
export function operandStatus(dc, key) {
  const s = get(dc, ['status', key], {});
  const desired = typeof s.desiredNumber === 'number' ? s.desiredNumber : 0;
  const available = typeof s.availableNumber === 'number' ? s.availableNumber : 0;
  const matching = typeof s.nodesMatchingSelectorNumber === 'number' ? s.nodesMatchingSelectorNumber : desired;
  return { desired: desired, available: available, unavailable: Math.max(0, desired - available), matching: matching };
}

/**
 * Same semantics as the reference (k8s.ts:370-379) with DaemonSet counts:
 * nothing scheduled → warning, all available → success, some → warning, none → error.
 * @returns {'success'|'warning'|'error'}
 */
export function countsToStatus(desired, available) {
  if (desired === 0) return 'warning';
  if (available >= desired) return 'success';
  if (available > 0) return 'warning';
  return 'error';
}

export function countsToText(desired, available) {
  if (desired === 0) return 'No nodes scheduled';
  return available + '/' + desired + ' ready';
}

const STATUS_RANK = { success: 0, warning: 1, error: 2 };

/** Worst status over the enabled operands (the device plugin always counts). */
export function deviceConfigStatus(dc) {
  let worst = 'success';
  for (let i = 0; i < OPERANDS.length; i++) {
    const key = OPERANDS[i].key;
    if (!operandEnabled(dc, key)) continue;
    const st = operandStatus(dc, key);
    const s = countsToStatus(st.desired, st.available);
    if (STATUS_RANK[s] > STATUS_RANK[worst]) worst = s;
  }
  return worst;
}

export function deviceConfigStatusText(dc) {
  const st = operandStatus(dc, 'devicePlugin');
  return countsToText(st.desired, st.available);
}

/** `spec.selector` (node selector map) rendered as `k=v, …`. */
export function formatSelector(sel) {
  if (!isObject(sel)) return '—';
  const keys = Object.keys(sel);
  if (keys.length === 0) return '—';
  return keys.map(function (k) { return k + '=' + sel[k]; }).join(', ');
}

// ---------------------------------------------------------------------------
// Nodes
// ---------------------------------------------------------------------------

function hasAmdLabel(labels) {
  if (labels[AMD_NFD_GPU_LABEL] === 'true') return true;
  const keys = Object.keys(labels);
  for (let i = 0; i < keys.length; i++) {
    const k = keys[i];
    if (k.indexOf(AMD_LABELLER_PREFIX) === 0 || k.indexOf(AMD_LABELLER_LEGACY_PREFIX) === 0) return true;
  }
  return false;
}

function hasAmdResource(res) {
  if (!isObject(res)) return false;
  const keys = Object.keys(res);
  for (let i = 0; i < keys.length; i++) {
    if (keys[i].indexOf(AMD_RESOURCE_PREFIX) === 0) return true;
  }
  return false;
}

/** A node is an AMD GPU node if NFD/labeller labels say so or it advertises `amd.com/*`. */
export function isAmdGpuNode(node) {
  if (!isNamedObject(node)) return false;
  if (hasAmdLabel(labelsOf(node))) return true;
  return hasAmdResource(get(node, ['status', 'capacity'], null));
}

export function filterAmdGpuNodes(items) {
  const out = [];
  if (!Array.isArray(items)) return out;
  for (let i = 0; i < items.length; i++) if (isAmdGpuNode(items[i])) out.push(items[i]);
  return out;
}

/** Every `amd.com/*` entry of a capacity/allocatable map. */
export function getGpuResources(resources) {
  const out = {};
  if (!isObject(resources)) return out;
  const keys = Object.keys(resources);
  for (let i = 0; i < keys.length; i++) {
    const k = keys[i];
    if (k.indexOf(AMD_RESOURCE_PREFIX) === 0 && resources[k] !== undefined && resources[k] !== null) {
      out[k] = String(resources[k]);
    }
  }
  return out;
}

/** True for resources that schedule GPU compute: `amd.com/gpu` and partition resources. */
export function isDeviceResource(key) {
  return key === AMD_GPU_RESOURCE || AMD_PARTITION_RESOURCE_RE.test(key);
}

function deviceSum(resources) {
  if (!isObject(resources)) return 0;
  let n = 0;
  const keys = Object.keys(resources);
  for (let i = 0; i < keys.length; i++) if (isDeviceResource(keys[i])) n += parseCount(resources[keys[i]]);
  return n;
}

/**
 * Schedulable GPU devices on the node: `amd.com/gpu` plus partition
 * resources (`amd.com/cpx_nps4` … in the device plugin's mixed naming). On
 * an SPX node this is the number of MI355X boards; on a partitioned node it
 * is the number of partitions (see getNodePhysicalGpuCount).
 */
export function getNodeGpuCount(node) {
  return deviceSum(get(node, ['status', 'capacity'], null));
}

export function getNodeGpuAllocatable(node) {
  return deviceSum(get(node, ['status', 'allocatable'], null));
}

/**
 * Compute partitions per MI355X in each mode: the chip has 8 XCDs, so CPX
 * exposes 8 devices per board, QPX 4, DPX 2, SPX 1.
 */
export const COMPUTE_PARTITIONS = Object.freeze({ SPX: 1, DPX: 2, QPX: 4, CPX: 8 });

/** Devices per physical GPU on this node (1 unless the labeller reports a partition mode). */
export function partitionsPerGpu(node) {
  const labels = labelsOf(node);
  const cp = labels[LABEL_COMPUTE_PARTITION] || labellerValue(node, 'compute-partitioning-mode');
  return (cp && COMPUTE_PARTITIONS[String(cp).toUpperCase()]) || 1;
}

/** MI355X boards on the node: devices ÷ partitions per board. */
export function getNodePhysicalGpuCount(node) {
  const d = getNodeGpuCount(node);
  return d > 0 ? Math.ceil(d / partitionsPerGpu(node)) : 0;
}

/** Partition resources (`amd.com/cpx_nps4` …) summed, for nodes in mixed naming mode. */
export function getNodePartitionCount(node) {
  const cap = get(node, ['status', 'capacity'], {});
  let n = 0;
  const keys = Object.keys(cap);
  for (let i = 0; i < keys.length; i++) if (AMD_PARTITION_RESOURCE_RE.test(keys[i])) n += parseCount(cap[keys[i]]);
  return n;
}

export function isNodeReady(node) {
  const conds = get(node, ['status', 'conditions'], []);
  if (!Array.isArray(conds)) return false;
  for (let i = 0; i < conds.length; i++) {
    if (conds[i] && conds[i].type === 'Ready' && conds[i].status === 'True') return true;
  }
  return false;
}

/** Look up a labeller property under the current or the legacy prefix. */
export function labellerValue(node, prop) {
  const labels = labelsOf(node);
  const v = labels[AMD_LABELLER_PREFIX + prop];
  if (v !== undefined) return v;
  const legacy = labels[AMD_LABELLER_LEGACY_PREFIX + prop];
  return legacy !== undefined ? legacy : null;
}

/**
 * PCI device ids → short product name. Only ids confirmed on hardware are
 * listed: 0x75a3 is what amd-smi reports for an MI355X (market name
 * "AMD Instinct MI355 OAM", IFWI "AMD MI355X"; tests/fixtures/mi355x).
 */
export const GPU_DEVICE_IDS = Object.freeze({ '75a3': 'MI355X' });

/** Short product name from a device id ("0x75a3") or a product string ("AMD_Instinct_MI355X"). */
export function shortProductName(deviceId, product) {
  if (deviceId) {
    const id = String(deviceId).toLowerCase().replace(/^0x/, '');
    if (GPU_DEVICE_IDS[id]) return GPU_DEVICE_IDS[id];
  }
  const m = product ? /MI\d{3}[A-Z]*/i.exec(String(product)) : null;
  return m ? m[0].toUpperCase() : MI355X.shortName;
}

/**
 * Product model of the node's GPUs. Replaces the reference's
 * discrete/integrated "GPU type" (k8s.ts:183-203): every GPU this plugin
 * targets is an MI355X, so the interesting fact is the product and its
 * partition mode, read from the node labeller when present.
 * @returns {{ product: string, shortName: string, fromLabels: boolean, computePartition: string|null, memoryPartition: string|null, vram: string, cuCount: number }}
 */
export function getNodeGpuModel(node) {
  const productLabel = labellerValue(node, 'product-name');
  const labels = labelsOf(node);
  const cp = labels[LABEL_COMPUTE_PARTITION] || labellerValue(node, 'compute-partitioning-mode');
  const mp = labels[LABEL_MEMORY_PARTITION] || labellerValue(node, 'memory-partitioning-mode');
  const vram = labellerValue(node, 'vram');
  const cu = labellerValue(node, 'cu-count');
  const deviceId = labellerValue(node, 'device-id');
  return {
    product: productLabel ? String(productLabel).replace(/_/g, ' ') : MI355X.product,
    shortName: shortProductName(deviceId, productLabel),
    fromLabels: !!productLabel,
    computePartition: cp ? String(cp).toUpperCase() : null,
    memoryPartition: mp ? String(mp).toUpperCase() : null,
    vram: vram ? String(vram) : MI355X.hbmLabel,
    cuCount: cu ? parseCount(cu) : MI355X.computeUnits,
  };
}

/** Column / row text for the node's GPU model, e.g. "MI355X" or "MI355X (CPX/NPS4)". */
export function formatGpuModel(model) {
  if (!model) return '—';
  let s = model.shortName;
  if (model.computePartition || model.memoryPartition) {
    s += ' (' + (model.computePartition || 'SPX') + '/' + (model.memoryPartition || 'NPS1') + ')';
  }
  return s;
}

// ---------------------------------------------------------------------------
// Pods
// ---------------------------------------------------------------------------

function containerAmdKeys(c) {
  const req = get(c, ['resources', 'requests'], {});
  const lim = get(c, ['resources', 'limits'], {});
  const keys = [];
  const seen = {};
  const all = Object.keys(req).concat(Object.keys(lim));
  for (let i = 0; i < all.length; i++) {
    const k = all[i];
    if (k.indexOf(AMD_RESOURCE_PREFIX) === 0 && !seen[k]) {
      seen[k] = true;
      keys.push(k);
    }
  }
  return keys;
}

/** True if any container, init or regular, requests or limits an `amd.com/*` resource. */
export function isGpuRequestingPod(pod) {
  if (!isNamedObject(pod)) return false;
  const cs = get(pod, ['spec', 'containers'], []);
  const ics = get(pod, ['spec', 'initContainers'], []);
  for (let i = 0; i < cs.length; i++) if (containerAmdKeys(cs[i]).length > 0) return true;
  for (let i = 0; i < ics.length; i++) if (containerAmdKeys(ics[i]).length > 0) return true;
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
  for (let i = 0; i < cs.length; i++) if (containerAmdKeys(cs[i]).length > 0) out.push(cs[i]);
  return out;
}

/** Init containers that carry an AMD resource. */
export function gpuInitContainers(pod) {
  const cs = get(pod, ['spec', 'initContainers'], []);
  const out = [];
  for (let i = 0; i < cs.length; i++) if (containerAmdKeys(cs[i]).length > 0) out.push(cs[i]);
  return out;
}

/**
 * Per-container AMD demand. For extended resources Kubernetes defaults the
 * request to the limit, so a limits-only container still consumes devices.
 * @returns {Array<{ key: string, request: string|null, limit: string|null, effective: number }>}
 */
export function containerGpuEntries(c) {
  const req = get(c, ['resources', 'requests'], {});
  const lim = get(c, ['resources', 'limits'], {});
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

// ---------------------------------------------------------------------------
// Operator / plugin pods
// ---------------------------------------------------------------------------

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
  const seen = {};
  const out = [];
  for (let i = 0; i < pods.length; i++) {
    const m = pods[i].metadata || {};
    const key = m.uid ? 'u:' + m.uid : 'n:' + (m.namespace || '') + '/' + (m.name || '');
    if (seen[key]) continue;
    seen[key] = true;
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

// ---------------------------------------------------------------------------
// Cluster-level aggregation (computed once per data change, not per render)
// ---------------------------------------------------------------------------

// Per-object facts the index needs, cached on the (immutable) object: a
// watch event that changes one pod re-derives that pod only.
const nodeFactCache = new WeakMap();
const podFactCache = new WeakMap();

function nodeFacts(n) {
  let f = nodeFactCache.get(n);
  if (!f) {
    const cap = getNodeGpuCount(n);
    const pp = partitionsPerGpu(n);
    f = {
      capacity: cap,
      allocatable: getNodeGpuAllocatable(n),
      ready: isNodeReady(n),
      cordoned: get(n, ['spec', 'unschedulable'], false) === true,
      partitionsPerGpu: pp,
      physicalGpus: cap > 0 ? Math.ceil(cap / pp) : 0,
      partitions: getNodePartitionCount(n),
    };
    nodeFactCache.set(n, f);
  }
  return f;
}

/**
 * {phase, nodeName, gpus} of a GPU pod, derived once per object; `gpus` is
 * what the pod holds (0 once it terminated).
 */
export function podFacts(p) {
  let f = podFactCache.get(p);
  if (!f) {
    const phase = podPhase(p);
    f = {
      phase: phase,
      nodeName: get(p, ['spec', 'nodeName'], null),
      // The kubelet allocates devices at admission and releases them when the
      // pod terminates, so a bound non-terminal pod holds its GPUs.
      gpus: phase !== 'Succeeded' && phase !== 'Failed' ? getPodGpuCount(p) : 0,
    };
    podFactCache.set(p, f);
  }
  return f;
}

function sameArray(a, b) {
  if (a === b) return true;
  if (!a || !b || a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) if (a[i] !== b[i]) return false;
  return true;
}

function sameFields(a, b) {
  if (a === b) return true;
  if (!a || !b) return false;
  for (const k in a) if (a[k] !== b[k]) return false;
  return true;
}

/**
 * Per-node GPU accounting and the pod index every page needs:
 * `podsByNode` and `nodeStats` are Maps keyed by node name.
 * Fixes reference quirks Q2 (pods vs GPUs), Q3 (init containers), Q10 (negative free).
 *
 * With `prev` (the index of the previous data), every per-node pod array and
 * stats object whose content did not change is taken from `prev`, and `prev`
 * itself is returned when nothing changed — so a memoised per-node view
 * (node card, Node detail section) is rebuilt only for the nodes an event
 * touched.
 * @param {any[]} gpuNodes
 * @param {any[]} gpuPods
 * @param {ReturnType<typeof buildClusterIndex>} [prev]
 */
export function buildClusterIndex(gpuNodes, gpuPods, prev) {
  const podsByNode = new Map();
  const nodeStats = new Map();
  let capacity = 0;
  let allocatable = 0;
  let inUse = 0;
  let readyNodes = 0;
  let cordonedNodes = 0;
  let partitions = 0;
  let physicalGpus = 0;
  let hbmBytes = 0;
  let hbmAllocatedBytes = 0;
  let heldGpus = 0;
  const phases = { Running: 0, Pending: 0, Succeeded: 0, Failed: 0, Other: 0 };
  for (let i = 0; i < gpuNodes.length; i++) {
    const n = gpuNodes[i];
    const name = n.metadata.name;
    const f = nodeFacts(n);
    capacity += f.capacity;
    allocatable += f.allocatable;
    partitions += f.partitions;
    physicalGpus += f.physicalGpus;
    hbmBytes += f.physicalGpus * MI355X.hbmBytes;
    if (f.ready) readyNodes++;
    if (f.cordoned) cordonedNodes++;
    nodeStats.set(name, {
      capacity: f.capacity, allocatable: f.allocatable, inUse: 0, pods: 0, ready: f.ready,
      // New pods can land here: Ready and not cordoned.
      schedulable: f.ready && !f.cordoned,
      physicalGpus: f.physicalGpus, partitionsPerGpu: f.partitionsPerGpu,
    });
    podsByNode.set(name, []);
  }
  for (let i = 0; i < gpuPods.length; i++) {
    const p = gpuPods[i];
    const f = podFacts(p);
    if (f.phase in phases) phases[f.phase]++;
    else phases.Other++;
    const nodeName = f.nodeName;
    if (!nodeName) continue;
    heldGpus += f.gpus;
    let bucket = podsByNode.get(nodeName);
    if (!bucket) podsByNode.set(nodeName, (bucket = []));
    bucket.push(p);
    const st = nodeStats.get(nodeName);
    if (!st) continue;
    st.pods++;
    st.inUse += f.gpus;
    inUse += f.gpus;
    // A partition holds its share of the board's HBM.
    hbmAllocatedBytes += (f.gpus * MI355X.hbmBytes) / st.partitionsPerGpu;
  }
  let schedulableFree = 0;
  nodeStats.forEach(function (st) { schedulableFree += schedulableFreeOf(st); });
  const totals = {
    nodes: gpuNodes.length,
    readyNodes: readyNodes,
    cordonedNodes: cordonedNodes,
    // Free GPUs a new pod can get: on Ready, uncordoned nodes only.
    schedulableFree: schedulableFree,
    capacity: capacity,
    allocatable: allocatable,
    inUse: inUse,
    free: Math.max(0, allocatable - inUse),
    partitions: partitions,
    physicalGpus: physicalGpus,
    hbmBytes: hbmBytes,
    hbmAllocatedBytes: hbmAllocatedBytes,
    utilizationPct: pct(inUse, allocatable),
    // GPUs held by bound, non-terminated pods, on any node (GPU Pods summary).
    heldGpus: heldGpus,
  };
  if (!prev) return { podsByNode: podsByNode, nodeStats: nodeStats, totals: totals, phases: phases };

  // Structural sharing with the previous index.
  let same = podsByNode.size === prev.podsByNode.size && nodeStats.size === prev.nodeStats.size;
  podsByNode.forEach(function (pods, name) {
    const old = prev.podsByNode.get(name);
    if (sameArray(old, pods)) podsByNode.set(name, old);
    else same = false;
  });
  nodeStats.forEach(function (st, name) {
    const old = prev.nodeStats.get(name);
    if (sameFields(old, st)) nodeStats.set(name, old);
    else same = false;
  });
  const sameTotals = sameFields(prev.totals, totals);
  const samePhases = sameFields(prev.phases, phases);
  if (same && sameTotals && samePhases) return prev;
  return {
    podsByNode: podsByNode,
    nodeStats: nodeStats,
    totals: sameTotals ? prev.totals : totals,
    phases: samePhases ? prev.phases : phases,
  };
}

function phaseBucket(phase) {
  return phase === 'Running' || phase === 'Pending' || phase === 'Succeeded' || phase === 'Failed' ? phase : 'Other';
}

/** Free GPUs of one node that a new pod could be scheduled onto (0 on a cordoned or not-Ready node). */
function schedulableFreeOf(st) {
  return st && st.schedulable ? Math.max(0, st.allocatable - st.inUse) : 0;
}

/**
 * The index after a delta of the GPU pod list — pods replaced by new
 * versions (status updates), removed and added — derived from `prev` in
 * O(changed pods + nodes) instead of rebuilt from every GPU node and pod.
 * Equal to `buildClusterIndex` of the new lists (tests/js/listCache.test.js
 * pins it); null when it cannot tell (the caller rebuilds).
 * @param {ReturnType<typeof buildClusterIndex>} prev
 * @param {{replaced: Array<[any, any]>, removed: any[], added: any[]}} delta
 * @param {(pod: any) => number} positionOf  list position (orders a node's pods)
 */
export function patchClusterIndex(prev, delta, positionOf) {
  const phases = Object.assign({}, prev.phases);
  const buckets = new Map();
  const stats = new Map();
  let inUse = prev.totals.inUse;
  let hbmAllocatedBytes = prev.totals.hbmAllocatedBytes;
  let heldGpus = prev.totals.heldGpus;

  function bucketOf(node, create) {
    let b = buckets.get(node);
    if (b === undefined) {
      const old = prev.podsByNode.get(node);
      if (!old && !create) return null;
      b = old ? old.slice() : [];
      buckets.set(node, b);
    }
    return b;
  }
  function account(f, sign) {
    phases[phaseBucket(f.phase)] += sign;
    if (!f.nodeName) return;
    heldGpus += sign * f.gpus;
    const base = stats.get(f.nodeName) || prev.nodeStats.get(f.nodeName);
    if (!base) return;
    const st = stats.get(f.nodeName) || Object.assign({}, base);
    stats.set(f.nodeName, st);
    st.pods += sign;
    st.inUse += sign * f.gpus;
    inUse += sign * f.gpus;
    hbmAllocatedBytes += (sign * f.gpus * MI355X.hbmBytes) / st.partitionsPerGpu;
  }
  function remove(p) {
    const f = podFacts(p);
    account(f, -1);
    if (!f.nodeName) return true;
    const b = bucketOf(f.nodeName, false);
    const idx = b ? b.indexOf(p) : -1;
    if (idx < 0) return false;
    b.splice(idx, 1);
    return true;
  }
  function add(p) {
    const f = podFacts(p);
    account(f, +1);
    if (!f.nodeName) return;
    const b = bucketOf(f.nodeName, true);
    const pos = positionOf(p);
    let at = b.length;
    while (at > 0 && positionOf(b[at - 1]) > pos) at--;
    b.splice(at, 0, p);
  }

  for (let k = 0; k < delta.replaced.length; k++) {
    const o = delta.replaced[k][0];
    const n = delta.replaced[k][1];
    const fo = podFacts(o);
    const fn = podFacts(n);
    if (fo.nodeName === fn.nodeName && fn.nodeName) {
      // Same place in its node's list.
      const b = bucketOf(fn.nodeName, false);
      const idx = b ? b.indexOf(o) : -1;
      if (idx < 0) return null;
      b[idx] = n;
      account(fo, -1);
      account(fn, +1);
    } else {
      if (!remove(o)) return null;
      add(n);
    }
  }
  for (let k = 0; k < delta.removed.length; k++) if (!remove(delta.removed[k])) return null;
  for (let k = 0; k < delta.added.length; k++) add(delta.added[k]);

  let podsByNode = prev.podsByNode;
  if (buckets.size > 0) {
    podsByNode = new Map(prev.podsByNode);
    buckets.forEach(function (b, node) {
      // Only GPU nodes keep an empty list (as buildClusterIndex does).
      if (b.length === 0 && !prev.nodeStats.has(node)) podsByNode.delete(node);
      else podsByNode.set(node, b);
    });
  }
  let nodeStats = prev.nodeStats;
  const changedStats = [];
  let schedulableFree = prev.totals.schedulableFree;
  stats.forEach(function (st, node) {
    const old = prev.nodeStats.get(node);
    schedulableFree += schedulableFreeOf(st) - schedulableFreeOf(old);
    if (!sameFields(old, st)) changedStats.push([node, st]);
  });
  if (changedStats.length > 0) {
    nodeStats = new Map(prev.nodeStats);
    for (let k = 0; k < changedStats.length; k++) nodeStats.set(changedStats[k][0], changedStats[k][1]);
  }
  const totals = Object.assign({}, prev.totals, {
    inUse: inUse,
    free: Math.max(0, prev.totals.allocatable - inUse),
    hbmAllocatedBytes: hbmAllocatedBytes,
    utilizationPct: pct(inUse, prev.totals.allocatable),
    heldGpus: heldGpus,
    schedulableFree: schedulableFree,
  });
  return {
    podsByNode: podsByNode,
    nodeStats: nodeStats,
    totals: sameFields(prev.totals, totals) ? prev.totals : totals,
    phases: sameFields(prev.phases, phases) ? prev.phases : phases,
  };
}

/** Rounded percentage, 0 when the denominator is 0. */
export function pct(used, total) {
  if (!(total > 0)) return 0;
  return Math.round((used / total) * 100);
}

/** success <70 %, warning ≥70 %, error ≥90 %. */
export function pctToStatus(p) {
  if (p >= ERROR_PCT) return 'error';
  if (p >= WARN_PCT) return 'warning';
  return 'success';
}

/** Bar colours matching the thresholds (AMD red for healthy "in use"). */
export const BAR_COLORS = { ok: '#ed1c24', warn: '#f57c00', err: '#d32f2f', track: '#e0e0e0', mute: '#9e9e9e' };

export function pctToColor(p) {
  if (p >= ERROR_PCT) return BAR_COLORS.err;
  if (p >= WARN_PCT) return BAR_COLORS.warn;
  return BAR_COLORS.ok;
}

// ---------------------------------------------------------------------------
// Formatters
// ---------------------------------------------------------------------------

/** Age as Ns / Nm / Nh / Nd (reference k8s.ts:337-348 semantics). `now` is injectable for tests. */
const timeCache = new Map();

/** Epoch ms of an RFC 3339 timestamp (NaN when unparseable); parsed once per string. */
export function parseTime(timestamp) {
  let t = timeCache.get(timestamp);
  if (t === undefined) {
    t = new Date(timestamp).getTime();
    if (timeCache.size > 65536) timeCache.clear();
    timeCache.set(timestamp, t);
  }
  return t;
}

/**
 * The instant (epoch ms) at which `formatAge(timestamp, now)` next shows a
 * different label: the next whole second, minute, hour or day of age
 * (Infinity when the label never changes).
 */
export function nextAgeChange(timestamp, now) {
  if (!timestamp) return Infinity;
  const t = parseTime(timestamp);
  if (!isFinite(t)) return Infinity;
  const n = now === undefined ? Date.now() : now;
  const secs = Math.max(0, Math.floor((n - t) / 1000));
  if (secs < 60) return t + (secs + 1) * 1000;
  const mins = Math.floor(secs / 60);
  if (mins < 60) return t + (mins + 1) * 60000;
  const hours = Math.floor(mins / 60);
  if (hours < 24) return t + (hours + 1) * 3600000;
  return t + (Math.floor(hours / 24) + 1) * 86400000;
}

export function formatAge(timestamp, now) {
  if (!timestamp) return 'unknown';
  const t = parseTime(timestamp);
  if (!isFinite(t)) return 'unknown';
  const diffMs = (now === undefined ? Date.now() : now) - t;
  const secs = Math.max(0, Math.floor(diffMs / 1000));
  if (secs < 60) return secs + 's';
  const mins = Math.floor(secs / 60);
  if (mins < 60) return mins + 'm';
  const hours = Math.floor(mins / 60);
  if (hours < 24) return hours + 'h';
  return Math.floor(hours / 24) + 'd';
}

/** Display name for an AMD extended resource key. */
export function formatGpuResourceName(key) {
  if (key === AMD_GPU_RESOURCE) return 'GPU';
  const m = AMD_PARTITION_RESOURCE_RE.exec(key);
  if (m) return 'GPU partition (' + m[1].toUpperCase() + '/' + m[2].toUpperCase() + ')';
  return key.indexOf(AMD_RESOURCE_PREFIX) === 0 ? key.slice(AMD_RESOURCE_PREFIX.length) : key;
}

/**
 * Bytes → "288 GiB" / "2.3 TiB". Binary units: the MI355X's "288 GB" of HBM3E
 * is 288 GiB (measured on the device), and the exporter reports MiB.
 */
export function formatBytes(b) {
  if (!(b >= 0) || b === null) return '—';
  const units = ['B', 'KiB', 'MiB', 'GiB', 'TiB', 'PiB'];
  let v = b;
  let u = 0;
  while (v >= 1024 && u < units.length - 1) {
    v /= 1024;
    u++;
  }
  // Three significant digits, trailing zeros dropped: "288 GiB", "2.25 TiB", "4.5 TiB".
  const digits = v >= 100 || u === 0 ? 0 : v >= 10 ? 1 : 2;
  let t = v.toFixed(digits);
  if (digits > 0) t = t.replace(/\.?0+$/, '');
  return t + ' ' + units[u];
}

export function formatWatts(w) {
  return w.toFixed(1) + ' W';
}

export function formatPercent(used, max) {
  if (!(max > 0)) return '—';
  return Math.round((used / max) * 100) + '%';
}
