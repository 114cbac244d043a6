/**
 * Native-view integration specs: Node detail section (reference
 * NodeDetailSection.test.tsx, 8 cases), Pod detail section
 * (PodDetailSection.test.tsx, 10 cases), the Nodes-table columns (untested in
 * the reference) and the topology model (new).
 */
import {
  formatEnergy,
  nodeColumns,
  nodeDetailView,
  podDetailView,
  seriesEnergyJoules,
} from '../../src/view/pages/details.js';
import { findSection, firstBlock, matrixCaption, matrixSummary, rowNames, rowValue, text } from '../../src/view/ir.js';
import { buildGpuSlots, buildXgmiMatrix, isFullMesh, placeThroughput } from '../../src/api/topology.js';
import { matrixBlock, nodesView } from '../../src/view/pages/nodes.js';
import { renderPage, renderSection } from '../../src/view/html.js';
import { renderText } from '../../src/view/text.js';
import { NOW, makeContext, makeGpuNode, makeGpuPod, makeNode, makePlainPod } from './fixtures.js';
import { getNodeGpuCount, getNodePhysicalGpuCount, partitionsPerGpu } from '../../src/api/amdNodes.js';
import { getPodGpuCount } from '../../src/api/amdPods.js';
import { buildClusterIndex } from '../../src/api/clusterIndex.js';
import { MI355X } from '../../src/api/k8sCore.js';

describe('nodeDetailView', () => {
  const node = makeGpuNode('g0');
  const ctx = makeContext({
    nodes: [node],
    pods: [makeGpuPod('a', { node: 'g0', gpus: 6 }), makeGpuPod('b', { node: 'g0', gpus: 1, phase: 'Succeeded' }), makeGpuPod('c', { node: 'other' })],
  });

  it('returns null for non-GPU nodes', () => {
    expect(nodeDetailView(makeNode('cpu'), ctx)).toBeNull();
  });
  it('returns null for label-only nodes without AMD resources', () => {
    expect(nodeDetailView(makeGpuNode('x', { capacity: false }), ctx)).toBeNull();
  });
  it('accepts a Headlamp KubeObject wrapper', () => {
    expect(nodeDetailView({ jsonData: node }, ctx)).not.toBeNull();
  });
  it('renders the AMD GPU section with capacity and allocatable rows', () => {
    const s = nodeDetailView(node, ctx);
    expect(s.title).toBe('AMD GPU');
    expect(rowValue(s, 'GPU (capacity)')).toBe('8');
    expect(rowValue(s, 'GPU (allocatable)')).toBe('8');
    expect(rowValue(s, 'GPU Model')).toBe('AMD Instinct MI355X');
    expect(rowValue(s, 'HBM')).toBe('2.25 TiB');
  });
  it('computes allocation from pods on this node with threshold status', () => {
    const s = nodeDetailView(node, ctx);
    expect(rowValue(s, 'GPU Allocation')).toEqual({ t: 'status', status: 'warning', text: '6/8 (75%)' });
  });
  it('pods seeded from an earlier store list are marked as being refreshed, not shown as current', () => {
    const s = nodeDetailView(node, Object.assign({}, ctx, { podsSeeded: true }));
    expect(rowValue(s, 'GPU Workload Pods')).toBe('a, b (from an earlier pod list; refreshing…)');
    expect(rowValue(s, 'GPU Allocation').text).toBe('6/8 (75%) (from an earlier pod list; refreshing…)');
    const none = makeContext({ nodes: [node], pods: [] });
    expect(rowValue(nodeDetailView(node, Object.assign({}, none, { podsSeeded: true })), 'GPU Workload Pods'))
      .toBe('None (from an earlier pod list; refreshing…)');
    expect(rowValue(nodeDetailView(node, ctx), 'GPU Workload Pods')).toBe('a, b');
  });
  it('escalates to error at 90%', () => {
    const c2 = makeContext({ nodes: [node], pods: [makeGpuPod('a', { node: 'g0', gpus: 8 })] });
    expect(rowValue(nodeDetailView(node, c2), 'GPU Allocation').status).toBe('error');
  });
  it('counts GPU init containers (reference quirk Q3)', () => {
    const c2 = makeContext({ nodes: [node], pods: [makeGpuPod('a', { node: 'g0', gpus: 1, init: 4 })] });
    expect(text(rowValue(nodeDetailView(node, c2), 'GPU Allocation'))).toBe('4/8 (50%)');
  });
  it('lists workload pods on the node', () => {
    expect(rowValue(nodeDetailView(node, ctx), 'GPU Workload Pods')).toBe('a, b');
  });
  it('shows Loading… while the store loads', () => {
    const c2 = makeContext({ loading: true, lastUpdated: null });
    expect(rowValue(nodeDetailView(node, c2), 'GPU Workload Pods')).toBe('Loading…');
  });
  it('shows None when no pods use the node', () => {
    expect(rowValue(nodeDetailView(node, makeContext({ nodes: [node] })), 'GPU Workload Pods')).toBe('None');
  });
  it('omits allocation when nothing is allocatable', () => {
    const n = makeGpuNode('g0', { allocatable: 0 });
    expect(rowNames(nodeDetailView(n, ctx))).not.toContain('GPU Allocation');
  });
  it('includes the per-GPU strip and xGMI matrix', () => {
    const s = nodeDetailView(node, ctx);
    expect(firstBlock(s, 'slots').slots).toHaveLength(8);
    expect(firstBlock(s, 'matrix').fullMesh).toBe(true);
  });
});

describe('podDetailView: GPU power history', () => {
  const series = { rangeSec: 1800, stepSec: 30, power: [[0, 1000], [30, 1200], [60, 1400]] };
  it('adds peak / average / energy over the window and a sparkline row for the pod', () => {
    const s = podDetailView(makeGpuPod('train-p', { gpus: 2 }), { series });
    expect(rowValue(s, 'Peak GPU Power (30 min)')).toBe('1400.0 W');
    expect(rowValue(s, 'Average GPU Power (30 min)')).toBe('1200.0 W');
    // 3 samples × 30 s steps: (1000 + 1200 + 1400) W × 30 s = 108 kJ = 30 Wh
    expect(rowValue(s, 'GPU Energy (30 min)')).toBe('30.0 Wh');
    const blk = s.blocks.filter((b) => b.t === 'series')[0];
    expect(blk.label).toBe('Pod');
    expect(Object.keys(blk.power)).toEqual(['train-p']);
    expect(blk.avgPower['train-p']).toBe(1200);
  });
  it('no history (empty or absent) leaves the section as it was', () => {
    const plain = podDetailView(makeGpuPod('train-q'));
    expect(podDetailView(makeGpuPod('train-q'), { series: { rangeSec: 1800, power: [] } }).blocks).toHaveLength(plain.blocks.length);
    expect(rowValue(plain, 'Peak GPU Power (30 min)')).toBeUndefined();
  });
  it('a window of non-numeric samples adds nothing (and does not throw)', () => {
    const plain = podDetailView(makeGpuPod('train-z'));
    const s = podDetailView(makeGpuPod('train-z'), { series: { rangeSec: 1800, power: [[0, NaN], [30, null]] } });
    expect(s.blocks).toHaveLength(plain.blocks.length);
  });
  it('energy helpers', () => {
    // fewer than 2 samples: unknown, shown as a dash (not "0.0 Wh" next to a non-zero peak)
    expect(seriesEnergyJoules([[0, 100]])).toBe(null);
    expect(formatEnergy(seriesEnergyJoules([[0, 100]]))).toBe('—');
    // with the query step each sample holds one step
    expect(seriesEnergyJoules([[0, 100], [60, 100]], 60)).toBe(12000);
    // a gap Prometheus left adds nothing (the old first-to-last guess stretched the step to 150 s: 45 kJ)
    expect(seriesEnergyJoules([[0, 100], [30, 100], [300, 100]], 30)).toBe(9000);
    // no step: trapezoid over the real timestamps
    expect(seriesEnergyJoules([[0, 100], [60, 200]])).toBe(9000);
    expect(formatEnergy(3600 * 1500)).toBe('1.50 kWh');
    expect(formatEnergy(3600 * 2)).toBe('2.0 Wh');
  });
});

describe('nodeDetailView: GPU power history', () => {
  it('adds the node\'s peak / average / energy and a Node sparkline row after the matrix', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('mi355x-7')] });
    const series = { rangeSec: 1800, power: [[0, 8000], [30, 9000]] };
    const s = nodeDetailView(makeGpuNode('mi355x-7'), ctx, { series });
    expect(rowValue(s, 'Peak GPU Power (30 min)')).toBe('9000.0 W');
    const kinds = s.blocks.map((b) => b.t);
    expect(kinds.slice(-2)).toEqual(['kv', 'series']);
    expect(kinds.indexOf('matrix')).toBeLessThan(kinds.indexOf('series'));
    expect(s.blocks[s.blocks.length - 1].label).toBe('Node');
    expect(nodeDetailView(makeGpuNode('mi355x-7'), ctx, {}).blocks.filter((b) => b.t === 'series')).toHaveLength(0);
  });
});

describe('podDetailView', () => {
  it('returns null for CPU pods', () => {
    expect(podDetailView(makePlainPod('x'))).toBeNull();
  });
  it('returns null for non-objects', () => {
    expect(podDetailView(null)).toBeNull();
  });
  it('accepts a KubeObject wrapper', () => {
    expect(podDetailView({ jsonData: makeGpuPod('p') })).not.toBeNull();
  });
  it('renders phase, node and container count', () => {
    const s = podDetailView(makeGpuPod('p', { gpus: 2 }));
    expect(s.title).toBe('AMD GPU Resources');
    expect(rowValue(s, 'Phase')).toEqual({ t: 'status', status: 'success', text: 'Running' });
    expect(rowValue(s, 'Scheduled Node')).toBe('mi355x-0');
    expect(rowValue(s, 'GPU Containers')).toBe('1');
    expect(rowValue(s, 'GPUs (effective)')).toBe('2 × MI355X (576 GiB HBM)');
  });
  it('shows request rows and omits equal limits', () => {
    const s = podDetailView(makeGpuPod('p', { gpus: 2 }));
    expect(rowValue(s, 'trainer → GPU request')).toBe('2');
    expect(rowNames(s)).not.toContain('trainer → GPU limit');
  });
  it('shows a limit row when it differs', () => {
    const p = makeGpuPod('p', { gpus: 1 });
    p.spec.containers[0].resources.limits['amd.com/gpu'] = '2';
    expect(rowValue(podDetailView(p), 'trainer → GPU limit')).toBe('2');
  });
  it('shows — for a limits-only request', () => {
    const s = podDetailView(makeGpuPod('p', { limitsOnly: true, gpus: 2 }));
    expect(rowValue(s, 'trainer → GPU request')).toBe('—');
    expect(rowValue(s, 'trainer → GPU limit')).toBe('2');
  });
  it('renders init-only GPU pods (reference quirk Q3)', () => {
    const s = podDetailView(makeGpuPod('p', { gpus: 0, init: 1 }));
    expect(s).not.toBeNull();
    expect(rowValue(s, 'warmup (init) → GPU request')).toBe('1');
  });
  it('maps Pending to warning and unknown phases to error', () => {
    expect(rowValue(podDetailView(makeGpuPod('p', { phase: 'Pending' })), 'Phase').status).toBe('warning');
    expect(rowValue(podDetailView(makeGpuPod('p', { phase: 'Failed' })), 'Phase').status).toBe('error');
    const p = makeGpuPod('p');
    delete p.status.phase;
    expect(rowValue(podDetailView(p), 'Phase')).toEqual({ t: 'status', status: 'error', text: 'Unknown' });
  });
  it('shows — for unscheduled pods', () => {
    expect(rowValue(podDetailView(makeGpuPod('p', { node: null, phase: 'Pending' })), 'Scheduled Node')).toBe('—');
  });
  it('lists partition resources with their display name', () => {
    const s = podDetailView(makeGpuPod('p', { resource: 'amd.com/cpx_nps4', gpus: 2 }));
    expect(rowValue(s, 'trainer → GPU partition (CPX/NPS4) request')).toBe('2');
  });
});

describe('nodeColumns', () => {
  const cols = nodeColumns();
  it('declares GPU Model, GPU Devices and GPU HBM', () => {
    expect(cols.map((c) => c.label)).toEqual(['GPU Model', 'GPU Devices', 'GPU HBM']);
  });
  it('returns dashes for CPU nodes', () => {
    const n = makeNode('c');
    expect(cols.map((c) => c.getter(n))).toEqual(['—', '—', '—']);
  });
  it('renders the model as a success status', () => {
    expect(cols[0].getter(makeGpuNode('g'))).toEqual({ t: 'status', status: 'success', text: 'MI355X' });
  });
  it('counts devices and HBM from KubeObject wrappers', () => {
    const w = { jsonData: makeGpuNode('g', { gpus: 4 }) };
    expect(cols[1].getter(w)).toBe('4');
    expect(cols[2].getter(w)).toBe('1.12 TiB');
  });
  it('shows — devices for label-only nodes', () => {
    expect(cols[1].getter(makeGpuNode('g', { capacity: false }))).toBe('—');
  });
  it('classifies each row once across columns', () => {
    const n = makeGpuNode('g');
    cols[0].getter(n);
    n.metadata.labels = {};
    n.status.capacity = {};
    // Cached classification from the first getter is reused.
    expect(cols[1].getter(n)).toBe('8');
  });
});

describe('topology', () => {
  it('builds a full 8×8 xGMI mesh with 7 links per GPU', () => {
    const m = buildXgmiMatrix(8);
    expect(m.size).toBe(8);
    expect(m.linksPerGpu).toBe(7);
    expect(m.perGpuPeakGBs).toBe(7 * 153);
    expect(m.ringBusGBs).toBe(153);
    expect(isFullMesh(m)).toBe(true);
    expect(m.cells[3][3].kind).toBe('self');
  });
  it('overlays measured throughput', () => {
    const m = buildXgmiMatrix(8, { '0-1': 42.5 });
    expect(m.cells[0][1].measuredGBs).toBe(42.5);
    expect(m.cells[1][0].measuredGBs).toBeNull();
  });
  it('detects a non-mesh from probed link types', () => {
    const m = buildXgmiMatrix(2, null, { '0-1': { type: 'PCIE', hops: 2 }, '1-0': { type: 'PCIE', hops: 2 } });
    expect(isFullMesh(m)).toBe(false);
    expect(m.cells[0][1].kind).toBe('pcie');
  });
  it('treats pairs missing from a measured topology as unconnected', () => {
    const m = buildXgmiMatrix(3, null, { '0-1': { type: 'XGMI', hops: 1 }, '1-0': { type: 'XGMI', hops: 1 } });
    expect(m.cells[0][2].kind).toBe('none');
    expect(m.linksPerGpu).toBe(1);
    expect(isFullMesh(m)).toBe(false);
  });
  it('xGMI throughput sits on a link only where a series pins neighbour k to its peer; else only per GPU', () => {
    // stock exporter rows: GPU 0 neighbours 0 and 1, GPU 1 neighbour 0 — which peers, no series says
    const measured = { '0>0': 10, '0>1': 20, '1>0': 5 };
    const unpinned = matrixBlock(8, measured, null, true);
    expect(unpinned.measuredThroughput).toBe(false);
    expect(unpinned.throughputPerGpu).toBe(true);
    expect(matrixCaption(unpinned)).not.toContain('link throughput measured');
    expect(matrixCaption(unpinned)).toContain('xGMI throughput measured per GPU, neighbour order not reported');
    expect(matrixSummary(unpinned)).toBe(' · measured per GPU: max 30, mean 18 GB/s over 2 GPUs');
    const ug = unpinned.matrix;
    ug.cells.forEach((row, i) => row.forEach((c, j) => { if (i !== j) expect(c.measuredGBs).toBeNull(); }));
    expect([ug.cells[0][0].measuredGBs, ug.cells[1][1].measuredGBs, ug.cells[2][2].measuredGBs]).toEqual([30, 5, null]);
    // this repo's exporter: link series with the KFD neighbour order (GPU 0's listed in reverse)
    const probed = {};
    for (let i = 0; i < 8; i++) {
      const peers = [];
      for (let j = 0; j < 8; j++) if (j !== i) peers.push(j);
      if (i === 0) peers.reverse();
      peers.forEach((j, k) => { probed[i + '-' + j] = { type: 'XGMI', hops: 1, neighbor: k }; });
    }
    const pinned = matrixBlock(8, measured, probed, true);
    expect(pinned.measuredThroughput).toBe(true);
    expect(matrixCaption(pinned)).toBe('xGMI topology (measured; link throughput measured) — full mesh, 7 links/GPU · 7× 153 GB/s per GPU · ' +
      'ring collectives bound at 153 GB/s per link');
    expect(matrixSummary(pinned)).toBe(' · measured: max 20, mean 12 GB/s over 3 links');
    const pg = pinned.matrix;
    expect([pg.cells[0][7].measuredGBs, pg.cells[0][6].measuredGBs, pg.cells[1][0].measuredGBs, pg.cells[0][1].measuredGBs]).toEqual([10, 20, 5, null]);
    expect(pg.cells[0][0].measuredGBs).toBe(30);
    // a link series without the order pins nothing
    const noOrder = {};
    Object.keys(probed).forEach((k) => { noOrder[k] = { type: 'XGMI', hops: 1 }; });
    expect(placeThroughput(measured, noOrder).pinned).toBe(false);
    expect(matrixCaption(matrixBlock(8, measured, noOrder, false))).toBe('xGMI topology (measured; xGMI throughput measured per GPU, ' +
      'neighbour order not reported) — full mesh, 7 links/GPU · 7× 153 GB/s per GPU · ring collectives bound at 153 GB/s per link');
    // a row that names its own peer is placed as named
    expect(placeThroughput({ '5-1': 7 }, null).map).toEqual({ '5-1': 7, '5-5': 7 });
  });
  it('a matrix block goes through JSON (amd-gpu-dash --json) with its grid and without the link maps', () => {
    const b = matrixBlock(8, { '0>0': 10, '2-3': 4 }, null, false);
    const j = JSON.parse(JSON.stringify(b));
    expect(Object.keys(j).sort()).toEqual(['fullMesh', 'gpuStats', 'linkGBs', 'linkStats', 'linksPerGpu', 'matrix', 'measuredThroughput',
      'measuredTopology', 'open', 'ringBusGBs', 'size', 't', 'throughputPerGpu']);
    expect(j.matrix.cells[2][3].measuredGBs).toBe(4);
    expect(j.matrix.cells[0][0].measuredGBs).toBe(10);
    expect(renderSection({ title: 'n', blocks: [j] })).toBe(renderSection({ title: 'n', blocks: [b] }));
    const open = JSON.parse(JSON.stringify(matrixBlock(8, { '0>0': 10 }, null, true)));
    expect(renderText({ title: 'x', actions: null, items: [{ title: 'n', blocks: [open] }] })).toContain('S10');
  });
  it('a GPU Nodes and a Node detail view-model render the same after a JSON round trip', () => {
    const nodes = [makeGpuNode('g0'), makeGpuNode('g1')];
    const ctx = makeContext({ nodes: nodes, pods: [makeGpuPod('a', { node: 'g0', gpus: 4 })] });
    const metrics = { source: 'amd-exporter', gpus: [], xgmi: { g0: { '0>0': 12, '1>3': 7 } }, links: {}, fetchedAt: new Date(NOW).toISOString() };
    const vm = nodesView(ctx, { now: NOW, metrics: metrics });
    const back = JSON.parse(JSON.stringify(vm));
    expect(renderPage(back)).toBe(renderPage(vm));
    expect(renderText(back)).toBe(renderText(vm));
    const card = back.items.find((x) => x.title === 'g0');
    expect(firstBlock(card, 'matrix').matrix.cells).toHaveLength(8);
    const sec = nodeDetailView(nodes[0], ctx, { now: NOW, metrics: metrics });
    const sback = JSON.parse(JSON.stringify(sec));
    expect(renderSection(sback)).toBe(renderSection(sec));
  });
  it('a single GPU is not a mesh', () => {
    expect(isFullMesh(buildXgmiMatrix(1))).toBe(false);
  });
  it('fills inferred slots in pod order, skipping finished pods', () => {
    const node = makeGpuNode('g', { gpus: 8 });
    const s = buildGpuSlots(node, [makeGpuPod('a', { gpus: 2 }), makeGpuPod('done', { gpus: 4, phase: 'Succeeded' }), makeGpuPod('b', { gpus: 1 })]);
    expect(s.exact).toBe(false);
    expect(s.slots.map((x) => x.pod)).toEqual(['a', 'a', 'b', null, null, null, null, null]);
    expect(s.slots[0].inferred).toBe(true);
  });
  it('never over-fills slots', () => {
    const s = buildGpuSlots(makeGpuNode('g', { gpus: 2 }), [makeGpuPod('a', { gpus: 8 })]);
    expect(s.slots).toHaveLength(2);
  });
  it('uses exporter owners when present', () => {
    const s = buildGpuSlots(makeGpuNode('g'), [], [{ gpu: '7', pod: 'x', namespace: 'ns' }, { gpu: '9', pod: 'bad' }]);
    expect(s.exact).toBe(true);
    expect(s.slots[7]).toEqual({ index: 7, board: 7, partition: null, pod: 'x', namespace: 'ns', inferred: false });
  });
});

void NOW;
void findSection;

describe('partitioned MI355X nodes (CPX: 8 devices per board)', () => {
  function cpxNode(name) {
    const n = makeGpuNode(name, { partition: 'cpx/nps2' });
    n.status.capacity['amd.com/gpu'] = '64';
    n.status.allocatable['amd.com/gpu'] = '64';
    return n;
  }
  it('counts boards, not partitions, for HBM and the xGMI matrix', () => {
    const n = cpxNode('c0');
    expect(getNodeGpuCount(n)).toBe(64);
    expect(partitionsPerGpu(n)).toBe(8);
    expect(getNodePhysicalGpuCount(n)).toBe(8);
    const s = nodeDetailView(n, makeContext({ nodes: [n] }));
    expect(rowValue(s, 'HBM')).toBe('2.25 TiB');
    const m = s.blocks.find((b) => b.t === 'matrix');
    expect(m.matrix.size).toBe(8);
  });
  it('labels each partition slot with its board', () => {
    const n = cpxNode('c1');
    const slots = buildGpuSlots(n, [], []).slots;
    expect(slots).toHaveLength(64);
    expect(slots[9].board).toBe(1);
    expect(slots[9].partition).toBe(1);
  });
  it('accounts HBM allocated per partition share', () => {
    const n = cpxNode('c2');
    const pod = makeGpuPod('p', { node: 'c2', gpus: 4 });
    const idx = buildClusterIndex([n], [pod]);
    expect(idx.totals.physicalGpus).toBe(8);
    expect(idx.totals.hbmAllocatedBytes).toBe((4 * MI355X.hbmBytes) / 8);
  });
  it('counts mixed-strategy partition resources as devices', () => {
    const n = makeGpuNode('m0', { partition: 'cpx/nps4' });
    delete n.status.capacity['amd.com/gpu'];
    n.status.capacity['amd.com/cpx_nps4'] = '16';
    expect(getNodeGpuCount(n)).toBe(16);
    expect(getNodePhysicalGpuCount(n)).toBe(2);
    expect(getPodGpuCount(makeGpuPod('q', { resource: 'amd.com/cpx_nps4', gpus: 3 }))).toBe(3);
  });
});
