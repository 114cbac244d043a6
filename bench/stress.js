#!/usr/bin/env node
/**
 * Watch-churn stress of the cluster-size scaling axis (SURVEY.md §5/§7.5).
 *
 *   node bench/stress.js [--nodes 16,64,256,1000] [--plain 30] [--events 500]
 *                        [--rate 50] [--mode identity|rewrapped|reparsed] [--out file.json]
 *
 * A synthetic cluster of N GPU nodes × 8 MI355X (4 training pods per node,
 * 30 plain pods per node, the operator's DaemonSet pods) is fed to the
 * shipped store the way Headlamp's `useList()` feeds it: after every watch
 * event a NEW list of every pod in the cluster. The event stream is
 * `--rate` events/s (the timing only decides how many events there are; each
 * is processed synchronously and timed in CPU ms): 80 % status updates of
 * plain pods, 10 % updates of GPU pods (restart counts / phase), 5 % pod
 * additions, 5 % deletions (half of each on GPU pods).
 *
 * Per event we time, on one thread:
 *   amd        store.setPods(list) → getSnapshot() → all five page
 *              view-models (Overview, Device Plugins, GPU Nodes, GPU Pods,
 *              Metrics) and the Node-detail section of the node the event
 *              touched — the shipped code (src/api/clusterStore.js,
 *              src/view/pages/*.js);
 *   reference  a replay of what the reference recomputes on the same event:
 *              jsonData extraction + GPU-pod filter over every pod
 *              (IntelGpuDataContext.tsx:200-208) and the Overview page's
 *              unmemoised aggregation over all GPU nodes and pods
 *              (OverviewPage.tsx:72-130) — the mounted page only, so the
 *              replay is a LOWER bound of the reference's per-event work.
 *
 * Delivery modes: `identity` — objects the event did not touch keep their
 * identity in the new list (Headlamp's list cache replaces the changed
 * item); `rewrapped` — a new KubeObject wrapper for every object around the
 * same JSON; `reparsed` — every object is a fresh copy (same uid and
 * resourceVersion), the worst case for identity-based caches.
 *
 * Reports per N: CPU ms per event (p50/p95/mean) for both, heap growth over
 * the churn, and bytes per pod / node list.
 */

import { filterAmdGpuNodes, getNodeGpuCount, getNodeGpuModel, isNodeReady } from '../src/api/amdNodes.js';
import { filterGpuRequestingPods, getPodGpuRequests } from '../src/api/amdPods.js';
import { unwrapAll } from '../src/api/k8sCore.js';
import { createClusterStore } from '../src/api/clusterStore.js';
import { clearViewMemo } from '../src/view/pages/common.js';
import { nodeDetailView } from '../src/view/pages/details.js';
import { devicePluginsView } from '../src/view/pages/devicePlugins.js';
import { metricsView } from '../src/view/pages/metricsPage.js';
import { nodesView } from '../src/view/pages/nodes.js';
import { overviewView } from '../src/view/pages/overview.js';
import { podsView } from '../src/view/pages/pods.js';
import fs from 'fs';

function parseArgs(argv) {
  const a = { nodes: [16, 64, 256, 1000], plain: 30, events: 500, rate: 50, mode: 'identity', out: null, seed: 7 };
  for (let i = 0; i < argv.length; i++) {
    const k = argv[i];
    const v = argv[i + 1];
    if (k === '--nodes') a.nodes = v.split(',').map(function (x) { return parseInt(x, 10); });
    else if (k === '--plain') a.plain = parseInt(v, 10);
    else if (k === '--events') a.events = parseInt(v, 10);
    else if (k === '--rate') a.rate = parseFloat(v);
    else if (k === '--mode') a.mode = v;
    else if (k === '--out') a.out = v;
    else if (k === '--seed') a.seed = parseInt(v, 10);
    else continue;
    i++;
  }
  return a;
}

// ---------------------------------------------------------------------------
// Synthetic cluster
// ---------------------------------------------------------------------------

function rng(seed) {
  let x = seed >>> 0 || 1;
  return function () {
    x ^= x << 13;
    x >>>= 0;
    x ^= x >>> 17;
    x ^= x << 5;
    x >>>= 0;
    return x / 4294967296;
  };
}

let rvCounter = 1000;
function nextRv() {
  rvCounter++;
  return String(rvCounter);
}

const T0 = '2026-10-01T00:00:00Z';

export function stressNode(i) {
  const name = 'mi355x-' + String(i).padStart(4, '0');
  return {
    apiVersion: 'v1',
    kind: 'Node',
    metadata: {
      name: name,
      uid: 'node-' + i,
      resourceVersion: nextRv(),
      creationTimestamp: T0,
      labels: {
        'kubernetes.io/hostname': name,
        'kubernetes.io/arch': 'amd64',
        'kubernetes.io/os': 'linux',
        'feature.node.kubernetes.io/amd-gpu': 'true',
        'amd.com/gpu.product-name': 'AMD_Instinct_MI355X',
        'amd.com/gpu.family': 'AI',
        'amd.com/gpu.device-id': '75a3',
        'amd.com/gpu.vram': '288G',
        'amd.com/gpu.cu-count': '256',
        'amd.com/gpu.driver-version': '6.12.12',
      },
    },
    status: {
      capacity: { cpu: '256', memory: '3Ti', 'amd.com/gpu': '8', pods: '250' },
      allocatable: { cpu: '255', memory: '3Ti', 'amd.com/gpu': '8', pods: '250' },
      conditions: [
        { type: 'MemoryPressure', status: 'False' },
        { type: 'DiskPressure', status: 'False' },
        { type: 'Ready', status: 'True', reason: 'KubeletReady' },
      ],
      nodeInfo: { osImage: 'Ubuntu 24.04 LTS', kernelVersion: '6.8.0-45-generic', kubeletVersion: 'v1.31.2', architecture: 'amd64' },
      addresses: [{ type: 'InternalIP', address: '10.0.' + (i >> 8) + '.' + (i & 255) }, { type: 'Hostname', address: name }],
    },
  };
}

function container(name, image, res) {
  return {
    name: name,
    image: image,
    ports: [{ containerPort: 8080, protocol: 'TCP' }],
    env: [{ name: 'POD_NAME', valueFrom: { fieldRef: { fieldPath: 'metadata.name' } } }],
    resources: res,
    volumeMounts: [{ name: 'kube-api-access', mountPath: '/var/run/secrets/kubernetes.io/serviceaccount', readOnly: true }],
    terminationMessagePath: '/dev/termination-log',
    imagePullPolicy: 'IfNotPresent',
  };
}

export function stressPod(name, ns, node, opts) {
  const o = opts || {};
  const gpus = o.gpus || 0;
  const res = gpus
    ? { requests: { cpu: '16', memory: '256Gi', 'amd.com/gpu': String(gpus) }, limits: { 'amd.com/gpu': String(gpus) } }
    : { requests: { cpu: '250m', memory: '256Mi' } };
  const phase = o.phase || 'Running';
  return {
    apiVersion: 'v1',
    kind: 'Pod',
    metadata: {
      name: name,
      namespace: ns,
      uid: 'pod-' + ns + '-' + name,
      resourceVersion: nextRv(),
      creationTimestamp: T0,
      labels: Object.assign({ app: o.app || name.split('-')[0], 'pod-template-hash': '7c9f8d' }, o.labels || {}),
      ownerReferences: [{ apiVersion: 'apps/v1', kind: 'ReplicaSet', name: name.split('-')[0] + '-7c9f8d', uid: 'rs-' + ns, controller: true }],
    },
    spec: {
      nodeName: node,
      serviceAccountName: 'default',
      restartPolicy: 'Always',
      schedulerName: 'default-scheduler',
      containers: [container(o.container || 'main', o.image || 'nginx:1.27', res)],
      volumes: [{ name: 'kube-api-access', projected: { sources: [{ serviceAccountToken: { path: 'token', expirationSeconds: 3607 } }] } }],
      tolerations: [{ key: 'node.kubernetes.io/not-ready', operator: 'Exists', effect: 'NoExecute', tolerationSeconds: 300 }],
    },
    status: {
      phase: phase,
      hostIP: '10.0.0.1',
      podIP: '10.244.0.1',
      startTime: T0,
      qosClass: gpus ? 'Burstable' : 'BestEffort',
      conditions: [
        { type: 'Initialized', status: 'True' },
        { type: 'Ready', status: phase === 'Running' ? 'True' : 'False' },
        { type: 'ContainersReady', status: phase === 'Running' ? 'True' : 'False' },
        { type: 'PodScheduled', status: 'True' },
      ],
      containerStatuses: [{
        name: o.container || 'main', ready: phase === 'Running', restartCount: o.restarts || 0, image: o.image || 'nginx:1.27',
        imageID: 'sha256:0123456789abcdef', containerID: 'containerd://' + name, started: phase === 'Running',
        state: phase === 'Running' ? { running: { startedAt: T0 } } : { waiting: { reason: 'ContainerCreating' } },
      }],
    },
  };
}

/** Nodes + pods of an N-node cluster (plus the operator's per-node DaemonSet pods). */
export function stressCluster(n, plainPerNode) {
  const nodes = [];
  const pods = [];
  for (let i = 0; i < n; i++) {
    const node = stressNode(i);
    nodes.push(node);
    const nn = node.metadata.name;
    const gp = [4, 2, 1, 1];
    for (let j = 0; j < gp.length; j++) {
      pods.push(stressPod('train-' + i + '-' + j, 'ml', nn, { gpus: gp[j], container: 'trainer', image: 'rocm/pytorch:rocm7.0' }));
    }
    pods.push(stressPod('amdgpu-device-plugin-' + i, 'kube-amd-gpu', nn, { labels: { name: 'amdgpu-dp-ds' }, app: 'device-plugin' }));
    pods.push(stressPod('amdgpu-node-labeller-' + i, 'kube-amd-gpu', nn, { labels: { name: 'amdgpu-labeller-ds' }, app: 'node-labeller' }));
    pods.push(stressPod('amdgpu-metrics-exporter-' + i, 'kube-amd-gpu', nn, { app: 'metrics-exporter' }));
    for (let j = 0; j < plainPerNode; j++) pods.push(stressPod('web-' + i + '-' + j, 'apps', nn, {}));
  }
  return { nodes: nodes, pods: pods };
}

function bump(obj, mutate) {
  const c = JSON.parse(JSON.stringify(obj));
  c.metadata.resourceVersion = nextRv();
  mutate(c);
  return c;
}

/**
 * One watch event applied to the cluster state: `pods` (raw objects) and
 * `wrapped` (Headlamp's list of KubeObject wrappers, in the same order) are
 * replaced by new arrays in which only the touched position differs — what
 * Headlamp's list cache does on an ADDED / MODIFIED / DELETED event.
 */
function applyEvent(state, rnd, n, seq) {
  const r = rnd();
  const pods = state.pods.slice();
  const wrapped = state.wrapped.slice();
  function done(node, kind) {
    state.pods = pods;
    state.wrapped = wrapped;
    return { node: node, kind: kind };
  }
  if (r < 0.9) {
    // MODIFIED: plain pod (80 %) or GPU pod (10 %).
    const wantGpu = r >= 0.8;
    for (let tries = 0; tries < 64; tries++) {
      const i = Math.floor(rnd() * pods.length);
      const p = pods[i];
      const isGpu = /^train-/.test(p.metadata.name);
      if (isGpu !== wantGpu) continue;
      pods[i] = bump(p, function (c) {
        const cs = c.status.containerStatuses[0];
        cs.restartCount++;
        if (isGpu && rnd() < 0.3) c.status.phase = c.status.phase === 'Running' ? 'Pending' : 'Running';
      });
      wrapped[i] = { jsonData: pods[i] };
      return done(p.spec.nodeName, isGpu ? 'gpu-modified' : 'modified');
    }
    return done(null, 'noop');
  }
  if (r < 0.95) {
    // ADDED: half GPU pods.
    const node = 'mi355x-' + String(Math.floor(rnd() * n)).padStart(4, '0');
    const gpu = rnd() < 0.5;
    const p = stressPod((gpu ? 'train-x' : 'web-x') + seq, gpu ? 'ml' : 'apps', node, gpu ? { gpus: 1, container: 'trainer' } : {});
    pods.push(p);
    wrapped.push({ jsonData: p });
    return done(node, gpu ? 'gpu-added' : 'added');
  }
  // DELETED: half GPU pods.
  const wantGpu = rnd() < 0.5;
  for (let tries = 0; tries < 64; tries++) {
    const i = Math.floor(rnd() * pods.length);
    const isGpu = /^train-/.test(pods[i].metadata.name);
    if (isGpu !== wantGpu) continue;
    const node = pods[i].spec.nodeName;
    pods.splice(i, 1);
    wrapped.splice(i, 1);
    return done(node, isGpu ? 'gpu-deleted' : 'deleted');
  }
  return done(null, 'noop');
}

/**
 * The list handed to the provider after an event, per delivery mode:
 *   identity   Headlamp's incremental list (untouched wrappers kept);
 *   rewrapped  a new KubeObject wrapper for every object, same JSON inside;
 *   reparsed   new wrappers around new objects (same uid + resourceVersion).
 */
function delivered(state, mode) {
  if (mode === 'identity') return state.wrapped;
  const out = new Array(state.pods.length);
  for (let i = 0; i < out.length; i++) {
    const p = state.pods[i];
    out[i] = { jsonData: mode === 'reparsed' ? Object.assign({}, p, { metadata: Object.assign({}, p.metadata) }) : p };
  }
  return out;
}

// ---------------------------------------------------------------------------
// Reference replay (original code; what the reference recomputes per event)
// ---------------------------------------------------------------------------

function referenceOnEvent(wrappedNodes, wrappedPods) {
  // Provider useMemo on the new allPods identity: extract + filter all pods.
  const gpuNodes = filterAmdGpuNodes(unwrapAll(wrappedNodes));
  const gpuPods = filterGpuRequestingPods(unwrapAll(wrappedPods));
  // OverviewPage render: node-type breakdown, capacity/allocatable sums over
  // every capacity key, GPUs in use summed over every request entry of every
  // running GPU pod, and the phase breakdown — recomputed on every render.
  let typed = 0;
  let total = 0;
  let ready = 0;
  for (let i = 0; i < gpuNodes.length; i++) {
    if (getNodeGpuModel(gpuNodes[i]).product) typed++;
    total += getNodeGpuCount(gpuNodes[i]);
    if (isNodeReady(gpuNodes[i])) ready++;
  }
  let cap = 0;
  let alloc = 0;
  for (let i = 0; i < gpuNodes.length; i++) {
    const c = (gpuNodes[i].status && gpuNodes[i].status.capacity) || {};
    const a = (gpuNodes[i].status && gpuNodes[i].status.allocatable) || {};
    const ks = Object.keys(c);
    for (let k = 0; k < ks.length; k++) {
      if (ks[k].indexOf('amd.com/') === 0) {
        cap += parseInt(c[ks[k]] || '0', 10);
        alloc += parseInt(a[ks[k]] || '0', 10);
      }
    }
  }
  let used = 0;
  const phases = { Running: 0, Pending: 0, Succeeded: 0, Failed: 0, Other: 0 };
  for (let i = 0; i < gpuPods.length; i++) {
    const p = gpuPods[i];
    const ph = (p.status && p.status.phase) || 'Other';
    if (ph in phases) phases[ph]++;
    else phases.Other++;
    if (ph !== 'Running') continue;
    const req = getPodGpuRequests(p);
    const ks = Object.keys(req);
    for (let k = 0; k < ks.length; k++) used += parseInt(req[ks[k]], 10) || 0;
  }
  return { typed: typed, total: total, ready: ready, cap: cap, alloc: alloc, used: used, phases: phases, pods: gpuPods.length };
}

// ---------------------------------------------------------------------------

function hr(t) {
  return t[0] * 1e3 + t[1] / 1e6;
}

function stats(xs) {
  const s = xs.slice().sort(function (a, b) { return a - b; });
  const q = function (p) {
    const idx = (s.length - 1) * p;
    const lo = Math.floor(idx);
    const hi = Math.ceil(idx);
    return s[lo] + (s[hi] - s[lo]) * (idx - lo);
  };
  const mean = s.reduce(function (a, b) { return a + b; }, 0) / (s.length || 1);
  return { n: s.length, p50: q(0.5), p95: q(0.95), max: s[s.length - 1], mean: mean };
}

function gc() {
  if (typeof global.gc === 'function') {
    global.gc();
    global.gc();
  }
}

function heap() {
  gc();
  return process.memoryUsage().heapUsed;
}

function noRequest() {
  return Promise.resolve({ kind: 'List', items: [] });
}

/**
 * Every page view-model for one snapshot (what a mounted dashboard rebuilds),
 * at the wall-clock instant `now` of the event (ages are drawn against it).
 */
function allViews(ctx, touchedNode, now, nodeByName) {
  const o = { now: now };
  const v = [overviewView(ctx, o), devicePluginsView(ctx, o), nodesView(ctx, o), podsView(ctx, o),
    metricsView(ctx, { metrics: null, fetchError: null, fetching: false, now: now })];
  // Headlamp's Node detail page of the node the event touched (it has the node object).
  const node = touchedNode ? nodeByName.get(touchedNode) : null;
  if (node) v.push(nodeDetailView(node, ctx, o));
  return v;
}

export async function runPoint(n, a) {
  const rnd = rng(a.seed + n);
  const cluster = stressCluster(n, a.plain);
  const podBytes = JSON.stringify({ kind: 'PodList', items: cluster.pods }).length;
  const nodeBytes = JSON.stringify({ kind: 'NodeList', items: cluster.nodes }).length;
  const events = Math.max(a.events, 1);

  const state = { pods: cluster.pods, wrapped: cluster.pods.map(function (p) { return { jsonData: p }; }) };
  const kinds = {};
  const byKind = {};
  const wrappedNodes = cluster.nodes.map(function (x) { return { jsonData: x }; });

  // --- amd: the shipped store + views ------------------------------------
  clearViewMemo();
  const store = createClusterStore({ request: noRequest });
  await store.refresh();
  store.setNodes(wrappedNodes, null);
  store.setPods(delivered(state, a.mode), null);
  // Events arrive at `--rate` per second of (simulated) wall clock.
  const clock0 = Date.parse('2026-10-15T12:00:00Z');
  const nodeByName = new Map(cluster.nodes.map(function (x) { return [x.metadata.name, x]; }));
  allViews(store.getSnapshot(), null, clock0, nodeByName);
  const heap0 = heap();
  const amd = [];
  const ref = [];
  let cpuMs = 0;
  let last = null;
  for (let e = 0; e < events; e++) {
    // The event, and the list Headlamp would hand over after it (untimed).
    const ev = applyEvent(state, rnd, n, e);
    kinds[ev.kind] = (kinds[ev.kind] || 0) + 1;
    const list = delivered(state, a.mode);
    const c0 = process.cpuUsage();
    const t0 = process.hrtime();
    store.setPods(list, null);
    allViews(store.getSnapshot(), ev.node, clock0 + ((e + 1) * 1000) / a.rate, nodeByName);
    const took = hr(process.hrtime(t0));
    amd.push(took);
    (byKind[ev.kind] = byKind[ev.kind] || []).push(took);
    const c1 = process.cpuUsage(c0);
    cpuMs += (c1.user + c1.system) / 1000;
    last = list;
  }
  const heap1 = heap();
  const snap = store.getSnapshot();
  const check = referenceOnEvent(wrappedNodes, last);

  // --- reference replay: the same event stream again (same seed), in its
  // own pass so neither side's garbage is collected on the other's clock.
  const rnd2 = rng(a.seed + n);
  const cluster2 = stressCluster(n, a.plain);
  const state2 = { pods: cluster2.pods, wrapped: cluster2.pods.map(function (p) { return { jsonData: p }; }) };
  const wrappedNodes2 = cluster2.nodes.map(function (x) { return { jsonData: x }; });
  heap();
  for (let e = 0; e < events; e++) {
    applyEvent(state2, rnd2, n, e);
    const list = delivered(state2, a.mode);
    const t1 = process.hrtime();
    referenceOnEvent(wrappedNodes2, list);
    ref.push(hr(process.hrtime(t1)));
  }
  return {
    nodes: n,
    pods: state.pods.length,
    gpuPods: snap.gpuPods.length,
    events: events,
    eventKinds: kinds,
    mode: a.mode,
    // Same answer both ways (the replay is a faithful recompute of the same state).
    consistent: check.pods === snap.gpuPods.length && check.cap === snap.index.totals.capacity,
    amd: stats(amd),
    amdByKind: Object.keys(byKind).reduce(function (o, k) { o[k] = stats(byKind[k]); return o; }, {}),
    reference: stats(ref),
    amdCpuMsPerEvent: cpuMs / events,
    storeCounters: store.counters(),
    heapGrowthBytes: heap1 - heap0,
    heapUsedBytes: heap1,
    podListBytes: podBytes,
    nodeListBytes: nodeBytes,
    churnSeconds: events / a.rate,
  };
}

async function main() {
  const a = parseArgs(process.argv.slice(2));
  const res = { events: a.events, rate: a.rate, plainPerNode: a.plain, mode: a.mode, node: process.version, points: [] };
  for (let i = 0; i < a.nodes.length; i++) {
    const p = await runPoint(a.nodes[i], a);
    res.points.push(p);
    process.stderr.write(
      'nodes=' + p.nodes + ' pods=' + p.pods + ' amd p50 ' + p.amd.p50.toFixed(3) + ' ms (p95 ' + p.amd.p95.toFixed(3) +
        ')  ref p50 ' + p.reference.p50.toFixed(3) + ' ms  heap +' + (p.heapGrowthBytes / 1e6).toFixed(1) + ' MB\n'
    );
  }
  const txt = JSON.stringify(res);
  if (a.out) fs.writeFileSync(a.out, txt);
  process.stdout.write(txt + '\n');
}

if (process.argv[1] && process.argv[1].indexOf('stress.js') >= 0) {
  main().then(
    function () { process.exit(0); },
    function (e) {
      process.stderr.write(String(e && e.stack ? e.stack : e) + '\n');
      process.exit(1);
    }
  );
}
