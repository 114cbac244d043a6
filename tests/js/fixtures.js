/**
 * Object factories for the JS specs (the reference's k8s.test.ts:33-80 uses
 * makeNode / makeGpuNode / makeGpuPod the same way).
 */

export const NOW = Date.parse('2026-10-15T12:00:00Z');

export function ago(seconds) {
  return new Date(NOW - seconds * 1000).toISOString();
}

export function makeNode(name, extra) {
  const n = {
    kind: 'Node',
    metadata: { name: name || 'cpu-node', uid: 'uid-' + (name || 'cpu-node'), labels: {}, creationTimestamp: ago(3600) },
    status: {
      capacity: { cpu: '64', memory: '512Gi' },
      allocatable: { cpu: '63', memory: '500Gi' },
      conditions: [{ type: 'Ready', status: 'True' }],
      nodeInfo: { osImage: 'Ubuntu 24.04 LTS', kernelVersion: '6.8.0-45-generic', kubeletVersion: 'v1.31.2', architecture: 'amd64' },
    },
  };
  return Object.assign(n, extra || {});
}

/**
 * @param {string} name
 * @param {{gpus?: number, allocatable?: number, labels?: boolean, nfd?: boolean, capacity?: boolean, ready?: boolean,
 *          partition?: string}} [o]
 */
export function makeGpuNode(name, o) {
  const opt = Object.assign({ gpus: 8, labels: true, nfd: true, capacity: true, ready: true }, o || {});
  const n = makeNode(name || 'mi355x-0');
  if (opt.nfd) n.metadata.labels['feature.node.kubernetes.io/amd-gpu'] = 'true';
  if (opt.labels) {
    n.metadata.labels['amd.com/gpu.product-name'] = 'AMD_Instinct_MI355X';
    n.metadata.labels['amd.com/gpu.family'] = 'AI';
    n.metadata.labels['amd.com/gpu.vram'] = '288G';
    n.metadata.labels['amd.com/gpu.cu-count'] = '256';
    n.metadata.labels['amd.com/gpu.driver-version'] = '6.12.12';
  }
  if (opt.partition) {
    n.metadata.labels['amd.com/compute-partitioning-mode'] = opt.partition.split('/')[0];
    n.metadata.labels['amd.com/memory-partitioning-mode'] = opt.partition.split('/')[1];
  }
  if (opt.capacity) {
    n.status.capacity['amd.com/gpu'] = String(opt.gpus);
    n.status.allocatable['amd.com/gpu'] = String(opt.allocatable === undefined ? opt.gpus : opt.allocatable);
  }
  if (!opt.ready) n.status.conditions = [{ type: 'Ready', status: 'False' }];
  return n;
}

/**
 * @param {string} name
 * @param {{gpus?: number, node?: string|null, phase?: string, ns?: string, limitsOnly?: boolean,
 *          init?: number, resource?: string, restarts?: number, waiting?: string}} [o]
 */
export function makeGpuPod(name, o) {
  const opt = Object.assign({ gpus: 1, node: 'mi355x-0', phase: 'Running', ns: 'ml', resource: 'amd.com/gpu', restarts: 0 }, o || {});
  const res = {};
  res[opt.resource] = String(opt.gpus);
  const resources = opt.limitsOnly ? { limits: res } : { requests: Object.assign({}, res), limits: Object.assign({}, res) };
  const p = {
    kind: 'Pod',
    metadata: { name: name, namespace: opt.ns, uid: 'uid-' + name, creationTimestamp: ago(600) },
    spec: {
      nodeName: opt.node === null ? undefined : opt.node,
      containers: opt.gpus > 0 ? [{ name: 'trainer', image: 'rocm/pytorch:latest', resources: resources }] : [{ name: 'app' }],
    },
    status: {
      phase: opt.phase,
      conditions: [{ type: 'Ready', status: opt.phase === 'Running' ? 'True' : 'False' }],
      containerStatuses: [{ name: 'trainer', ready: opt.phase === 'Running', restartCount: opt.restarts, state: {} }],
    },
  };
  if (opt.waiting) p.status.containerStatuses[0].state = { waiting: { reason: opt.waiting } };
  if (opt.init) {
    const ir = {};
    ir[opt.resource] = String(opt.init);
    p.spec.initContainers = [{ name: 'warmup', resources: { requests: ir, limits: Object.assign({}, ir) } }];
  }
  return p;
}

export function makePlainPod(name, node) {
  return {
    kind: 'Pod',
    metadata: { name: name, namespace: 'default', uid: 'uid-' + name },
    spec: { nodeName: node || 'cpu-node', containers: [{ name: 'c', resources: { requests: { cpu: '1' } } }] },
    status: { phase: 'Running' },
  };
}

export function makeDeviceConfig(name, o) {
  const opt = Object.assign({ desired: 2, available: 2, exporter: true, labeller: true, driver: false }, o || {});
  return {
    apiVersion: 'amd.com/v1alpha1',
    kind: 'DeviceConfig',
    metadata: { name: name || 'gpu-operator', namespace: 'kube-amd-gpu', uid: 'uid-dc-' + (name || 'gpu-operator'), creationTimestamp: ago(86400 * 3) },
    spec: {
      driver: { enable: opt.driver, version: '6.12.12' },
      devicePlugin: { devicePluginImage: 'rocm/k8s-device-plugin:latest', enableNodeLabeller: opt.labeller },
      metricsExporter: { enable: opt.exporter, port: 5000 },
      selector: { 'feature.node.kubernetes.io/amd-gpu': 'true' },
    },
    status: {
      devicePlugin: { nodesMatchingSelectorNumber: opt.desired, desiredNumber: opt.desired, availableNumber: opt.available },
      nodeLabeller: { nodesMatchingSelectorNumber: opt.desired, desiredNumber: opt.desired, availableNumber: opt.desired },
      metricsExporter: { nodesMatchingSelectorNumber: opt.desired, desiredNumber: opt.desired, availableNumber: opt.desired },
    },
  };
}

export function makePluginPod(name, o) {
  const opt = Object.assign({ node: 'mi355x-0', ready: true, restarts: 0, label: 'amdgpu-dp-ds', ns: 'kube-system' }, o || {});
  return {
    kind: 'Pod',
    metadata: { name: name, namespace: opt.ns, uid: opt.uid === undefined ? 'uid-' + name : opt.uid, labels: opt.label ? { name: opt.label } : {}, creationTimestamp: ago(7200) },
    spec: { nodeName: opt.node, containers: [{ name: 'plugin' }] },
    status: {
      phase: 'Running',
      conditions: [{ type: 'Ready', status: opt.ready ? 'True' : 'False' }],
      containerStatuses: [{ name: 'plugin', ready: opt.ready, restartCount: opt.restarts }],
    },
  };
}

/** A snapshot shaped like ClusterStore.getSnapshot(), built from raw objects. */
import { filterAmdGpuNodes } from '../../src/api/amdNodes.js';
import { filterGpuRequestingPods } from '../../src/api/amdPods.js';
import { buildClusterIndex } from '../../src/api/clusterIndex.js';

export function makeContext(over) {
  const o = over || {};
  const nodes = o.nodes || [];
  const pods = o.pods || [];
  const gpuNodes = o.gpuNodes || filterAmdGpuNodes(nodes);
  const gpuPods = o.gpuPods || filterGpuRequestingPods(pods);
  const ctx = {
    deviceConfigs: [],
    pluginInstalled: false,
    gpuNodes: gpuNodes,
    gpuPods: gpuPods,
    pluginPods: [],
    crdAvailable: false,
    loading: false,
    refreshing: false,
    error: null,
    lastUpdated: NOW,
    index: buildClusterIndex(gpuNodes, gpuPods),
    version: 1,
  };
  for (const k in o) if (k !== 'nodes' && k !== 'pods') ctx[k] = o[k];
  if (o.pluginInstalled === undefined) ctx.pluginInstalled = ctx.deviceConfigs.length > 0 || ctx.pluginPods.length > 0;
  return ctx;
}
