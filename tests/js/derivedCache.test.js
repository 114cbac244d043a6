/**
 * What a cold mount pays for (api/derivedCache.js) and what the data layer
 * derived on arrival (api/nodeSummaries.js, clusterIndex.js facts): the view
 * memo's reset (clearViewMemo — a cluster switch, tests, the render
 * comparison's first-render-of-a-session mount) empties the first; the second
 * stays with its objects.
 */
import { derivedCache, resetDerivedCaches } from '../../src/api/derivedCache.js';
import { buildClusterIndex, nodeFacts, podContainerLines } from '../../src/api/clusterIndex.js';
import { nodePowerKeys, ownersByNode, podGpuAssignments, primeSnapshot } from '../../src/api/nodeSummaries.js';
import { deviceConfigFacts, operatorPodFacts } from '../../src/api/operatorFacts.js';
import { linkFacts } from '../../src/api/topology.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { nodeReadyCell } from '../../src/view/pages/nodes.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makePluginPod } from './fixtures.js';

function snapshot() {
  const gpus = [];
  for (let i = 0; i < 8; i++) {
    gpus.push({ nodeName: 'n1', gpu: String(i), powerWatts: 1000 + i, powerCapWatts: 1400, tempC: 60 + i, pod: i < 2 ? 'train' : null, namespace: 'ml' });
  }
  const xgmi = { n1: {} };
  for (let i = 0; i < 8; i++) for (let j = 0; j < 8; j++) if (i !== j) xgmi.n1[i + '-' + j] = 10;
  return { gpus: gpus, xgmi: xgmi, links: {} };
}

describe('derivedCache', () => {
  it('resetDerivedCaches empties every registered cache and runs its reset hook', () => {
    const c = derivedCache();
    let hook = 0;
    c.onReset = () => { hook++; };
    const k = {};
    expect(c.set(k, 1)).toBe(1);
    expect(c.has(k)).toBe(true);
    resetDerivedCaches();
    expect(c.has(k)).toBe(false);
    expect(hook).toBe(1);
  });

  it('clearViewMemo drops first-use view facts: a pod\'s container lines', () => {
    const pod = makeGpuPod('a', { gpus: 2 });
    const lines = podContainerLines(pod);
    expect(podContainerLines(pod)).toBe(lines);
    clearViewMemo();
    expect(podContainerLines(pod)).not.toBe(lines);
    expect(podContainerLines(pod)).toEqual(lines);
  });

  it('facts derived on arrival stay: node facts, and a primed snapshot\'s summaries and link facts', () => {
    const node = makeGpuNode('n1');
    const f = nodeFacts(node);
    const ready = nodeReadyCell(node);
    const m = primeSnapshot(snapshot());
    const power = nodePowerKeys(m);
    const owners = ownersByNode(m);
    const assign = podGpuAssignments(m);
    const links = linkFacts(8, m.xgmi.n1, null);
    clearViewMemo();
    expect(nodeFacts(node)).toBe(f);
    expect(nodeReadyCell(node)).toBe(ready); // one cell per wording, from the node's facts
    expect(f.card.after).toEqual([{ name: 'OS / Kernel / Kubelet / amdgpu', value: f.osText + ' · amdgpu ' + f.driverVersion }]);
    expect(nodePowerKeys(m)).toBe(power);
    expect(ownersByNode(m)).toBe(owners);
    expect(podGpuAssignments(m)).toBe(assign);
    expect(linkFacts(8, m.xgmi.n1, null)).toBe(links);
    expect(power.byNode.n1).toBe('8028|11200');
    expect(owners.n1.map((o) => o.gpu)).toEqual(['0', '1']);
    expect(assign['ml/train']).toHaveLength(2);
    expect(links).toEqual({ fullMesh: true, linksPerGpu: 7, stats: { links: 56, meanGBs: 10, maxGBs: 10 }, gpuStats: { gpus: 8, meanGBs: 70, maxGBs: 70 } });
  });

  it('the index derives every node\'s accounting with the list, display facts only for the first page in name order', () => {
    const nodes = [];
    for (let i = 0; i < 20; i++) nodes.push(makeGpuNode('node-' + String(19 - i).padStart(2, '0')));
    buildClusterIndex(nodes, []);
    const primed = nodes.filter((n) => nodeFacts(n).shown !== null).map((n) => n.metadata.name).sort();
    expect(primed).toEqual(['node-00', 'node-01', 'node-02', 'node-03', 'node-04', 'node-05', 'node-06', 'node-07']);
    expect(nodes.every((n) => nodeFacts(n).capacity === 8)).toBe(true);
    // any other node's display facts on first read, kept with its object (not reset with the memo)
    const late = nodes.find((n) => n.metadata.name === 'node-15');
    expect(nodeFacts(late).modelText).toBe('MI355X');
    const shown = nodeFacts(late).shown;
    clearViewMemo();
    expect(nodeFacts(late).shown).toBe(shown);
    // a small cluster: every node
    const few = [makeGpuNode('b'), makeGpuNode('a')];
    buildClusterIndex(few, []);
    expect(few.every((n) => nodeFacts(n).shown !== null)).toBe(true);
  });

  it('the store derives the DeviceConfigs\' facts when it takes their list; an operator pod\'s when a row reads them', async () => {
    const { createClusterStore } = await import('../../src/api/clusterStore.js');
    const dc = makeDeviceConfig('gpu-operator');
    const op = makePluginPod('dp-0');
    const store = createClusterStore({ request: (path) => Promise.resolve({ kind: 'List', items: path.indexOf('deviceconfigs') >= 0 ? [dc] : [op] }) });
    store.setNodes([], null);
    store.setPods([op], null);
    await store.refresh();
    const ctx = store.getSnapshot();
    expect(ctx.deviceConfigs).toEqual([dc]);
    const f = deviceConfigFacts(ctx.deviceConfigs[0]);
    const pf = operatorPodFacts(op);
    expect(operatorPodFacts(makePluginPod('dp-1'))).not.toBe(pf);
    clearViewMemo();
    expect(deviceConfigFacts(ctx.deviceConfigs[0])).toBe(f);
    expect(operatorPodFacts(op)).toBe(pf);
    expect(f.metricsExporter).toEqual({ enabled: true, level: 'success', text: 'Enabled — port 5000 · 2/2 ready' });
    expect(pf.ready).toBe(true);
  });
});

describe('arrival facts change no output', () => {
  it('a page built from a primed snapshot equals one built from fresh, unprimed copies of the same data', async () => {
    const { nodesView } = await import('../../src/view/pages/nodes.js');
    const { podsView } = await import('../../src/view/pages/pods.js');
    const { makeContext } = await import('./fixtures.js');
    const nodes = [makeGpuNode('n1'), makeGpuNode('n2')];
    const pods = [makeGpuPod('train', { node: 'n1', gpus: 2 }), makeGpuPod('eval', { node: 'n2', gpus: 1 })];
    const now = Date.parse('2026-10-16T00:00:00Z');
    function metrics() {
      const m = snapshot();
      m.gpus.forEach((g, i) => { if (i < 2) g.pod = 'train'; });
      return m;
    }
    const primed = primeSnapshot(metrics());
    const a = [nodesView(makeContext({ nodes, pods }), { metrics: primed, now }), podsView(makeContext({ nodes, pods }), { metrics: primed, now })];
    clearViewMemo();
    const copy = (x) => JSON.parse(JSON.stringify(x));
    const fresh = metrics(); // never primed: every summary derived on first read
    const b = [nodesView(makeContext({ nodes: copy(nodes), pods: copy(pods) }), { metrics: fresh, now }),
      podsView(makeContext({ nodes: copy(nodes), pods: copy(pods) }), { metrics: fresh, now })];
    expect(JSON.stringify(b)).toBe(JSON.stringify(a));
  });
});
