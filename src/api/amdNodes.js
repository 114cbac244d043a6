/**
 * The AMD GPU Operator DeviceConfig CRD and GPU nodes: guards, per-operand
 * DaemonSet status, GPU node detection (NFD / labeller labels or amd.com/*
 * capacity), GPU counts incl. compute partitions, readiness and the GPU
 * model from labeller labels. Pure, I/O-free.
 *
 * Reference: src/api/k8s.ts:56-86 (CRD, C2.3), :125-203 (node detection,
 * resources, GPU type, C2.5-C2.7), :329-331 (readiness, C2.13), :370-386
 * (status mapping, C2.15).
 */

import {
  AMD_GPU_RESOURCE,
  AMD_LABELLER_LEGACY_PREFIX,
  AMD_LABELLER_PREFIX,
  AMD_NFD_GPU_LABEL,
  AMD_PARTITION_RESOURCE_RE,
  AMD_RESOURCE_PREFIX,
  DEVICE_CONFIG_KIND,
  get,
  isNamedObject,
  isObject,
  LABEL_COMPUTE_PARTITION,
  LABEL_MEMORY_PARTITION,
  labelsOf,
  MI355X,
  parseCount,
} from './k8sCore.js';

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
  return partitionsOfMode(computePartitionLabel(node));
}

/** Devices per board for a compute partition label value (null: SPX). */
export function partitionsOfMode(cp) {
  return (cp && COMPUTE_PARTITIONS[String(cp).toUpperCase()]) || 1;
}

/** The node's compute partition mode label (the GPU operator's, else the labeller's), or null. */
export function computePartitionLabel(node) {
  return labelsOf(node)[LABEL_COMPUTE_PARTITION] || labellerValue(node, 'compute-partitioning-mode');
}

/**
 * The node's partition mode as the Overview counts it, "SPX/NPS1" when
 * unlabelled (the same labels getNodeGpuModel reads, without the rest of the
 * model).
 */
export function partitionModeKey(node, cp) {
  const c = cp === undefined ? computePartitionLabel(node) : cp;
  const mp = labelsOf(node)[LABEL_MEMORY_PARTITION] || labellerValue(node, 'memory-partitioning-mode');
  return (c ? String(c).toUpperCase() : 'SPX') + '/' + (mp ? String(mp).toUpperCase() : 'NPS1');
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

/** [current, legacy] label key of each labeller property, made once. */
const LABELLER_KEYS = Object.create(null);

/** Look up a labeller property under the current or the legacy prefix. */
export function labellerValue(node, prop) {
  const labels = labelsOf(node);
  const keys = LABELLER_KEYS[prop] || (LABELLER_KEYS[prop] = [AMD_LABELLER_PREFIX + prop, AMD_LABELLER_LEGACY_PREFIX + prop]);
  const v = labels[keys[0]];
  if (v !== undefined) return v;
  const legacy = labels[keys[1]];
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
  // A node object is an immutable snapshot of the watch: its model is read once.
  const key = node && typeof node === 'object' ? node : null;
  if (modelCache && key && modelCache.has(key)) return modelCache.get(key);
  const m = readGpuModel(node);
  if (modelCache && key) modelCache.set(key, m);
  return m;
}

const modelCache = typeof WeakMap === 'function' ? new WeakMap() : null;

function readGpuModel(node) {
  const productLabel = labellerValue(node, 'product-name');
  const labels = labelsOf(node);
  const cp = labels[LABEL_COMPUTE_PARTITION] || labellerValue(node, 'compute-partitioning-mode');
  const mp = labels[LABEL_MEMORY_PARTITION] || labellerValue(node, 'memory-partitioning-mode');
  const vram = labellerValue(node, 'vram');
  const cu = labellerValue(node, 'cu-count');
  const deviceId = labellerValue(node, 'device-id');
  return Object.freeze({
    product: productLabel ? String(productLabel).replace(/_/g, ' ') : MI355X.product,
    shortName: shortProductName(deviceId, productLabel),
    fromLabels: !!productLabel,
    computePartition: cp ? String(cp).toUpperCase() : null,
    memoryPartition: mp ? String(mp).toUpperCase() : null,
    vram: vram ? String(vram) : MI355X.hbmLabel,
    cuCount: cu ? parseCount(cu) : MI355X.computeUnits,
  });
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
