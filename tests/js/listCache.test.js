/**
 * Incremental list tracking (src/api/listCache.js) and the index patch
 * (patchClusterIndex): after every watch event of a seeded random stream —
 * status updates, additions, deletions, reorders, pods moving between
 * nodes, phase changes, new wrappers around the same JSON, re-parsed copies
 * — the store's GPU nodes / GPU pods / operator pods and cluster index are
 * EQUAL to a from-scratch computation over the whole list (the reference's
 * recompute), and unrelated churn leaves every subset's identity alone.
 */
import { createListTracker } from '../../src/api/listCache.js';
import { createClusterStore } from '../../src/api/clusterStore.js';
import { filterAmdGpuNodes } from '../../src/api/amdNodes.js';
import {
  filterAmdGpuPluginPods,
  filterGpuRequestingPods,
  isAmdGpuPluginPod,
  isGpuRequestingPod,
} from '../../src/api/amdPods.js';
import { buildClusterIndex, patchClusterIndex } from '../../src/api/clusterIndex.js';
import { makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from './fixtures.js';

function rng(seed) {
  let a = seed >>> 0;
  return function () {
    a = (a + 0x6d2b79f5) >>> 0;
    let t = a;
    t = Math.imul(t ^ (t >>> 15), t | 1);
    t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}

let rv = 1;
function versioned(obj) {
  obj.metadata.resourceVersion = String(rv++);
  return obj;
}

/** A new version of `p` (copy, new resourceVersion) with `mutate` applied. */
function bump(p, mutate) {
  const c = JSON.parse(JSON.stringify(p));
  mutate(c);
  return versioned(c);
}

function plainIndex(idx) {
  const obj = function (m) {
    const o = {};
    m.forEach(function (v, k) { o[k] = v; });
    return o;
  };
  return { podsByNode: obj(idx.podsByNode), nodeStats: obj(idx.nodeStats), totals: idx.totals, phases: idx.phases };
}

const NODES = ['g0', 'g1', 'g2', 'g3'];

function initialPods(r) {
  const pods = [];
  for (let i = 0; i < 40; i++) {
    const k = r();
    if (k < 0.35) pods.push(versioned(makeGpuPod('gpu-' + i, { node: NODES[i % 4], gpus: 1 + (i % 3) })));
    else if (k < 0.45) pods.push(versioned(makePluginPod('plugin-' + i, { node: NODES[i % 4] })));
    else pods.push(versioned(makePlainPod('plain-' + i, i % 5 === 0 ? 'cpu-0' : NODES[i % 4])));
  }
  return pods;
}

let seq = 0;
/** One random watch event: returns the next raw pod list. */
function step(r, pods) {
  const next = pods.slice();
  const x = r();
  const i = Math.floor(r() * next.length);
  if (x < 0.35 && next.length) {
    next[i] = bump(next[i], function (c) {
      c.status = c.status || {};
      c.status.containerStatuses = [{ name: 'c', restartCount: Math.floor(r() * 5), ready: true }];
    });
  } else if (x < 0.5 && next.length) {
    const phases = ['Running', 'Pending', 'Succeeded', 'Failed', 'Unknown'];
    next[i] = bump(next[i], function (c) { c.status.phase = phases[Math.floor(r() * phases.length)]; });
  } else if (x < 0.6 && next.length) {
    // Bound to another node (or unbound).
    next[i] = bump(next[i], function (c) { c.spec.nodeName = r() < 0.2 ? undefined : NODES[Math.floor(r() * 4)]; });
  } else if (x < 0.72) {
    const n = 'new-' + seq++;
    const p = r() < 0.6 ? makeGpuPod(n, { node: r() < 0.1 ? null : NODES[Math.floor(r() * 4)], gpus: 1 + Math.floor(r() * 4) }) : makePlainPod(n, 'g1');
    next.splice(Math.floor(r() * (next.length + 1)), 0, versioned(p));
  } else if (x < 0.84 && next.length) {
    next.splice(i, 1);
  } else if (x < 0.88 && next.length > 2) {
    // Reorder two objects.
    const k = Math.floor(r() * next.length);
    const t = next[i];
    next[i] = next[k];
    next[k] = t;
  } else if (x < 0.92 && next.length) {
    // Label change: an operator pod stops / starts being one.
    next[i] = bump(next[i], function (c) {
      c.metadata.labels = c.metadata.labels && c.metadata.labels.name ? {} : { name: 'amdgpu-dp-ds' };
    });
  }
  return next;
}

describe('createListTracker', () => {
  it('classifies only the objects an event changed', () => {
    const pods = [];
    for (let i = 0; i < 200; i++) pods.push(versioned(makePlainPod('p' + i, 'g0')));
    pods.push(versioned(makeGpuPod('train', { node: 'g0' })));
    const t = createListTracker([isGpuRequestingPod, isAmdGpuPluginPod]);
    t.update(pods);
    const before = t.stats().classified;
    const gpu = t.subsets()[0];
    const next = pods.slice();
    next[17] = bump(next[17], function (c) { c.status.phase = 'Failed'; });
    const r = t.update(next);
    expect(t.stats().classified - before).toBe(1);
    expect(r.changed).toEqual([false, false]);
    expect(t.subsets()[0]).toBe(gpu);
  });

  it('keeps subsets and their objects across new wrappers around the same JSON', () => {
    const pods = [versioned(makeGpuPod('a', { node: 'g0' })), versioned(makePlainPod('b', 'g0'))];
    const t = createListTracker([isGpuRequestingPod]);
    t.update(pods.map((p) => ({ jsonData: p })));
    const gpu = t.subsets()[0];
    const r = t.update(pods.map((p) => ({ jsonData: p })));
    expect(r.changed).toEqual([false]);
    expect(t.subsets()[0]).toBe(gpu);
    expect(t.stats().classified).toBe(2);
  });

  it('keeps the held object when a re-parsed copy has the same resourceVersion', () => {
    const a = versioned(makeGpuPod('a', { node: 'g0' }));
    const t = createListTracker([isGpuRequestingPod]);
    t.update([a]);
    const r = t.update([JSON.parse(JSON.stringify(a))]);
    expect(r.changed).toEqual([false]);
    expect(t.subsets()[0][0]).toBe(a);
  });

  it('reports a replaced GPU pod as a delta', () => {
    const a = versioned(makeGpuPod('a', { node: 'g0' }));
    const b = versioned(makeGpuPod('b', { node: 'g1' }));
    const t = createListTracker([isGpuRequestingPod]);
    const x = versioned(makePlainPod('x', 'g0'));
    t.update([a, x, b]);
    const b2 = bump(b, function (c) { c.status.phase = 'Pending'; });
    const r = t.update([a, x, b2]);
    expect(r.changed).toEqual([true]);
    expect(r.deltas[0].replaced).toEqual([[b, b2]]);
    expect(t.subsets()[0]).toEqual([a, b2]);
  });

  it('matches a from-scratch filter after every event of a random stream', () => {
    for (let seed = 1; seed <= 6; seed++) {
      const r = rng(seed);
      let pods = initialPods(r);
      const t = createListTracker([isGpuRequestingPod, isAmdGpuPluginPod]);
      t.update(pods);
      for (let e = 0; e < 150; e++) {
        pods = step(r, pods);
        const mode = r();
        const delivered = mode < 0.7 ? pods : mode < 0.85 ? pods.map((p) => ({ jsonData: p })) : pods.map((p) => JSON.parse(JSON.stringify(p)));
        const before = t.subsets().slice();
        const res = t.update(delivered);
        const gpu = t.subsets()[0];
        const plug = t.subsets()[1];
        expect(gpu.map((p) => p.metadata.uid)).toEqual(filterGpuRequestingPods(pods).map((p) => p.metadata.uid));
        expect(plug.map((p) => p.metadata.uid)).toEqual(filterAmdGpuPluginPods(pods).map((p) => p.metadata.uid));
        // Unchanged subsets keep their identity.
        if (!res.changed[0]) expect(gpu).toBe(before[0]);
        if (!res.changed[1]) expect(plug).toBe(before[1]);
      }
    }
  });
});

describe('store: incremental index', () => {
  it('equals buildClusterIndex of the whole lists after every event', () => {
    for (let seed = 11; seed <= 16; seed++) {
      const r = rng(seed);
      const nodes = NODES.map((n, i) => versioned(makeGpuNode(n, { gpus: 8, partition: i === 3 ? 'CPX/NPS4' : undefined })));
      // g1 cordoned: its free GPUs must stay out of the schedulable total through every patch
      nodes[1].spec = Object.assign({}, nodes[1].spec, { unschedulable: true });
      nodes.push(versioned(makeNode('cpu-0')));
      let pods = initialPods(r);
      const store = createClusterStore({ request: () => Promise.resolve({ kind: 'List', items: [] }) });
      store.setNodes(nodes, null);
      store.setPods(pods, null);
      let patched = 0;
      for (let e = 0; e < 150; e++) {
        const prevIdx = store.getSnapshot().index;
        pods = step(r, pods);
        store.setPods(r() < 0.8 ? pods : pods.map((p) => ({ jsonData: p })), null);
        const snap = store.getSnapshot();
        const gpuNodes = filterAmdGpuNodes(nodes);
        const gpuPods = filterGpuRequestingPods(pods);
        expect(snap.gpuPods.map((p) => p.metadata.uid)).toEqual(gpuPods.map((p) => p.metadata.uid));
        expect(plainIndex(snap.index)).toEqual(plainIndex(buildClusterIndex(gpuNodes, snap.gpuPods)));
        if (snap.index !== prevIdx) patched++;
      }
      expect(patched).toBeGreaterThan(20);
      // Most of those were delta patches, not rebuilds.
      expect(store.counters().indexPatches).toBeGreaterThan(store.counters().indexBuilds);
    }
  });

  it('stays equal to buildClusterIndex when node events (cordon, uncordon, resize, leave, join) interleave with pod events', () => {
    for (let seed = 21; seed <= 24; seed++) {
      const r = rng(seed);
      let nodes = NODES.map((n) => versioned(makeGpuNode(n, { gpus: 8 })));
      nodes.push(versioned(makeNode('cpu-0')));
      let pods = initialPods(r);
      const store = createClusterStore({ request: () => Promise.resolve({ kind: 'List', items: [] }) });
      store.setNodes(nodes, null);
      store.setPods(pods, null);
      let cordonedSeen = 0;
      for (let e = 0; e < 120; e++) {
        if (r() < 0.3) {
          nodes = nodes.slice();
          const i = Math.floor(r() * nodes.length);
          const y = r();
          if (y < 0.5) {
            nodes[i] = bump(nodes[i], function (c) { c.spec = Object.assign({}, c.spec, { unschedulable: !(c.spec && c.spec.unschedulable) }); });
          } else if (y < 0.75) {
            const n = 2 + Math.floor(r() * 7);
            nodes[i] = bump(nodes[i], function (c) {
              if (c.status && c.status.allocatable && c.status.allocatable['amd.com/gpu'] !== undefined) c.status.allocatable['amd.com/gpu'] = String(n);
            });
          } else if (y < 0.87 && nodes.length > 2) {
            nodes.splice(i, 1);
          } else {
            const name = NODES[Math.floor(r() * NODES.length)];
            if (!nodes.some((x) => x.metadata.name === name)) nodes.push(versioned(makeGpuNode(name, { gpus: 8 })));
          }
          store.setNodes(r() < 0.7 ? nodes : nodes.map((x) => ({ jsonData: x })), null);
        } else {
          pods = step(r, pods);
          store.setPods(pods, null);
        }
        const snap = store.getSnapshot();
        expect(plainIndex(snap.index)).toEqual(plainIndex(buildClusterIndex(filterAmdGpuNodes(nodes), snap.gpuPods)));
        cordonedSeen += snap.index.totals.cordonedNodes > 0 ? 1 : 0;
      }
      expect(cordonedSeen).toBeGreaterThan(0);
    }
  });

  it('patches only the nodes an event touched (others keep their identity)', () => {
    const nodes = NODES.map((n) => versioned(makeGpuNode(n)));
    const pods = NODES.map((n, i) => versioned(makeGpuPod('t' + i, { node: n })));
    const store = createClusterStore({ request: () => Promise.resolve({ kind: 'List', items: [] }) });
    store.setNodes(nodes, null);
    store.setPods(pods, null);
    const a = store.getSnapshot().index;
    const next = pods.slice();
    next[2] = bump(next[2], function (c) { c.status.phase = 'Succeeded'; });
    store.setPods(next, null);
    const b = store.getSnapshot().index;
    expect(b).not.toBe(a);
    expect(b.podsByNode.get('g0')).toBe(a.podsByNode.get('g0'));
    expect(b.nodeStats.get('g1')).toBe(a.nodeStats.get('g1'));
    expect(b.nodeStats.get('g2')).not.toBe(a.nodeStats.get('g2'));
    expect(b.nodeStats.get('g2').inUse).toBe(0);
    expect(b.totals.inUse).toBe(3);
    expect(b.phases.Succeeded).toBe(1);
  });

  it('patchClusterIndex gives up (null) on a delta that does not match the index', () => {
    const n = makeGpuNode('g0');
    const p = versioned(makeGpuPod('a', { node: 'g0' }));
    const idx = buildClusterIndex([n], [p]);
    const stranger = versioned(makeGpuPod('b', { node: 'g0' }));
    expect(patchClusterIndex(idx, { replaced: [], removed: [stranger], added: [] }, () => 0)).toBe(null);
  });
});
