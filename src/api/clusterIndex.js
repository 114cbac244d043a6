/**
 * The cluster index: per-node GPU allocation, pods per node, cluster totals
 * and phase counts, built once per data change and PATCHED per watch event
 * (only the changed pods' nodes are recomputed; unchanged per-node objects
 * keep their identity for the memoised views). Pure, I/O-free.
 *
 * Reference: the aggregation every page recomputed per render
 * (src/components/OverviewPage.tsx:72-130, NodesPage.tsx:153-189).
 */

import {
  formatGpuModel,
  getGpuResources,
  getNodeGpuAllocatable,
  getNodeGpuCount,
  getNodeGpuModel,
  getNodePartitionCount,
  isNodeReady,
  labellerValue,
  computePartitionLabel,
  partitionModeKey,
  partitionsOfMode,
} from './amdNodes.js';
import { containerGpuEntries, getPodGpuCount, gpuContainers, gpuInitContainers, podPhase } from './amdPods.js';
import { derivedCache } from './derivedCache.js';
import { AMD_GPU_RESOURCE, formatBytes, formatGpuResourceName, get, MI355X, pct } from './k8sCore.js';
import { SMALL_CLUSTER_NODES } from './series.js';

// Per-object facts the index needs, cached on the (immutable) object: a
// watch event that changes one pod re-derives that pod only.
const nodeFactCache = new WeakMap();

const podFactCache = new WeakMap();

/**
 * What a GPU node object says, derived once per object. Its GPU accounting
 * and readiness — what the index and every page's totals need — when the
 * index is built, i.e. when the node list arrives. The rest — GPU model,
 * resources, taints, driver, node info, the GPU Nodes card rows — for the
 * first page of nodes with the list (primeFirstPage), for any other node on
 * first read (a page shows eight of up to 1,000 nodes): those fields are
 * prototype getters over one display object made once per node object.
 */
export function nodeFacts(n) {
  let f = nodeFactCache.get(n);
  if (!f) {
    f = new NodeFacts(n);
    nodeFactCache.set(n, f);
  }
  return f;
}

function NodeFacts(n) {
  const cap = getNodeGpuCount(n);
  const cp = computePartitionLabel(n);
  const pp = partitionsOfMode(cp);
  this.node = n;
  this.capacity = cap;
  this.allocatable = getNodeGpuAllocatable(n);
  this.ready = isNodeReady(n);
  this.cordoned = get(n, ['spec', 'unschedulable'], false) === true;
  this.partitionsPerGpu = pp;
  this.physicalGpus = cap > 0 ? Math.ceil(cap / pp) : 0;
  this.partitions = getNodePartitionCount(n);
  // Overview counts nodes per partition mode (its distribution bar).
  this.partitionMode = partitionModeKey(n, cp);
  // Readiness as `kubectl get nodes` words it; a cordoned node's free GPUs
  // are not schedulable, hence a warning.
  this.readyText = (this.ready ? 'Ready' : 'Not Ready') + (this.cordoned ? ', SchedulingDisabled' : '');
  this.readyLevel = !this.ready ? 'error' : this.cordoned ? 'warning' : 'success';
  this.shown = null;
}

/** The display facts of the node, made on first read. */
NodeFacts.prototype.display = function () {
  let d = this.shown;
  if (!d) {
    const n = this.node;
    const model = getNodeGpuModel(n);
    const info = get(n, ['status', 'nodeInfo'], null) || {};
    d = this.shown = {
      model: model,
      modelText: formatGpuModel(model),
      capacityResources: getGpuResources(get(n, ['status', 'capacity'], null)),
      allocatableResources: getGpuResources(get(n, ['status', 'allocatable'], null)),
      taints: taintsText(n),
      driverVersion: labellerValue(n, 'driver-version'),
      osText: [info.osImage || '—', info.kernelVersion || '—', info.kubeletVersion || '—'].join(' · '),
      card: null,
    };
    d.card = cardRows(this, d);
  }
  return d;
};

['model', 'modelText', 'capacityResources', 'allocatableResources', 'taints', 'driverVersion', 'osText', 'card'].forEach(function (k) {
  Object.defineProperty(NodeFacts.prototype, k, { enumerable: true, get: function () { return this.display()[k]; } });
});

/**
 * The display facts of the nodes the GPU Nodes page opens on — the first
 * page in its default (name) order, SMALL_CLUSTER_NODES of them — derived
 * with the list, as their accounting is; every other node's on first read.
 */
function primeFirstPage(gpuNodes) {
  if (gpuNodes.length <= SMALL_CLUSTER_NODES) {
    for (let i = 0; i < gpuNodes.length; i++) nodeFacts(gpuNodes[i]).display();
    return;
  }
  const first = [];
  for (let i = 0; i < gpuNodes.length; i++) {
    const name = gpuNodes[i].metadata.name;
    if (first.length === SMALL_CLUSTER_NODES && !(name < first[first.length - 1].metadata.name)) continue;
    let k = first.length === SMALL_CLUSTER_NODES ? first.length - 1 : first.length;
    while (k > 0 && first[k - 1].metadata.name > name) {
      first[k] = first[k - 1];
      k--;
    }
    first[k] = gpuNodes[i];
  }
  for (let i = 0; i < first.length; i++) nodeFacts(first[i]).display();
}

const hbmTexts = {};

/** HBM of `phys` MI355X boards, formatted once per board count. */
function hbmText(phys) {
  return hbmTexts[phys] || (hbmTexts[phys] = formatBytes(phys * MI355X.hbmBytes));
}

/**
 * A GPU Nodes card's rows that the node alone decides, as {name, value}:
 * `before` the workload pods (taints, devices, HBM, per-resource capacity /
 * allocatable, partition mode, driver), `after` them (node info). The
 * summary row on the same page carries readiness, model and age (the
 * reference repeats them on its card, NodesPage.tsx:69-139).
 */
function cardRows(f, d) {
  const model = d.model;
  const count = f.capacity;
  const cap = d.capacityResources;
  const alloc = d.allocatableResources;
  const before = [];
  if (d.taints) before.push({ name: 'Taints', value: d.taints });
  // One resource (the usual amd.com/gpu): its capacity and allocatable are
  // said on the device row (the reference gives them a row each,
  // NodesPage.tsx:98-113); several (partitioned resources) keep their rows.
  const capKeys = Object.keys(cap);
  const single = capKeys.length === 1 && capKeys[0] === AMD_GPU_RESOURCE && Object.keys(alloc).length <= 1;
  if (count > 0) {
    const phys = f.physicalGpus;
    const devices = phys !== count ? count + ' (' + phys + ' × ' + model.shortName + ' in ' + model.computePartition + ')' : String(count);
    // The devices and the HBM they carry on one row (a card is a row less to mount).
    before.push({
      name: 'GPU Devices (amd.com/gpu) · HBM',
      value: (single
        ? devices + ' · capacity ' + cap[AMD_GPU_RESOURCE] + ', allocatable ' + (alloc[AMD_GPU_RESOURCE] !== undefined ? alloc[AMD_GPU_RESOURCE] : '—')
        : devices) + ' · HBM ' + hbmText(phys) + ' (' + phys + ' × ' + model.vram + ')',
    });
  }
  if (!single || count === 0) {
    for (const k in cap) before.push({ name: formatGpuResourceName(k) + ' (capacity)', value: cap[k] });
    for (const k in alloc) before.push({ name: formatGpuResourceName(k) + ' (allocatable)', value: alloc[k] });
  }
  if (model.computePartition || model.memoryPartition) before.push({ name: 'Partition Mode', value: d.modelText });
  // The node's software on one row: OS image, kernel, kubelet (the reference: a row each, NodesPage.tsx:124-126)
  // and the amdgpu driver the labeller reports.
  return {
    before: before,
    after: [d.driverVersion ? { name: 'OS / Kernel / Kubelet / amdgpu', value: d.osText + ' · amdgpu ' + d.driverVersion }
      : { name: 'OS / Kernel / Kubelet', value: d.osText }],
  };
}

/** "key=value:Effect" per taint, or null (the reference models NodeSpec.taints, k8s.ts:92-122, but never shows them). */
export function taintsText(node) {
  const ts = get(node, ['spec', 'taints'], []);
  if (!Array.isArray(ts) || ts.length === 0) return null;
  return ts.map(function (t) { return (t.key || '') + (t.value ? '=' + t.value : '') + ':' + (t.effect || ''); }).join(', ');
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

/**
 * A GPU pod's containers as the GPU Pods table lists them (pages/pods.js
 * gpuContainerLines): derived on first read and kept with the pod's facts —
 * not when the list arrives (a page shows 25 of 5,000 GPU pods).
 */
export function podContainerLines(p) {
  return containerCache.has(p) ? containerCache.get(p) : containerCache.set(p, containerLines(p));
}

const containerCache = derivedCache();

/**
 * One {label, text} per GPU container, init containers first ("trainer",
 * "GPU: 2"; "req=1 lim=2" when they differ) — the reference's
 * GpuContainerList (PodsPage.tsx:49-88), init containers included.
 */
function containerLines(pod) {
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
  return out;
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
  primeFirstPage(gpuNodes);
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
