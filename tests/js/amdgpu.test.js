/**
 * Domain-model specs (analog of reference src/api/k8s.test.ts, 48 cases).
 */
import {
  countsToStatus,
  countsToText,
  deviceConfigStatus,
  deviceConfigStatusText,
  filterAmdGpuNodes,
  formatGpuModel,
  formatSelector,
  getGpuResources,
  getNodeGpuAllocatable,
  getNodeGpuCount,
  getNodeGpuModel,
  getNodePartitionCount,
  isAmdGpuNode,
  isDeviceConfig,
  isNodeReady,
  operandEnabled,
  operandStatus,
  shortProductName,
} from '../../src/api/amdNodes.js';
import {
  containerGpuEntries,
  dedupePods,
  filterAmdGpuPluginPods,
  filterGpuRequestingPods,
  formatPodGpuRequests,
  getPodGpuCount,
  getPodGpuDemand,
  getPodGpuRequests,
  getPodRestarts,
  isAmdGpuPluginPod,
  isGpuRequestingPod,
  isPodReady,
  phaseToStatus,
  pluginPodComponent,
  podWaitingMessage,
  podWaitingReason,
} from '../../src/api/amdPods.js';
import { buildClusterIndex } from '../../src/api/clusterIndex.js';
import {
  AMD_GPU_RESOURCE,
  DEVICE_CONFIG_LIST_PATH,
  formatAge,
  formatBytes,
  formatGpuResourceName,
  formatPercent,
  formatWatts,
  isKubeList,
  isNamedObject,
  MI355X,
  nextAgeChange,
  parseCount,
  pct,
  pctToColor,
  pctToStatus,
  PLUGIN_POD_QUERIES,
  unwrapAll,
  unwrapKubeObject,
} from '../../src/api/k8sCore.js';
import { NOW, ago, makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from './fixtures.js';

describe('constants', () => {
  it('targets the AMD GPU Operator DeviceConfig CRD', () => {
    expect(DEVICE_CONFIG_LIST_PATH).toBe('/apis/amd.com/v1alpha1/deviceconfigs');
  });
  it('uses amd.com/gpu as the whole-GPU resource', () => {
    expect(AMD_GPU_RESOURCE).toBe('amd.com/gpu');
  });
  it('describes an MI355X with 288 GB HBM and an 8-GPU xGMI mesh', () => {
    expect(MI355X.hbmBytes).toBe(294896 * 1024 * 1024); // device-reported: tests/fixtures/mi355x
    expect(formatBytes(MI355X.hbmBytes)).toBe('288 GiB');
    expect(MI355X.gpusPerNode).toBe(8);
    expect(MI355X.xgmiLinksPerGpu).toBe(MI355X.gpusPerNode - 1);
    expect(MI355X.computeUnits).toBe(256);
  });
  it('encodes the set-based plugin-pod selector', () => {
    expect(decodeURIComponent(PLUGIN_POD_QUERIES[0])).toContain('name in (amdgpu-dp-ds,amdgpu-labeller-ds)');
    // disjoint from the namespace request: the operator namespace is left out of the selector's answer
    expect(decodeURIComponent(PLUGIN_POD_QUERIES[0])).toContain('&fieldSelector=metadata.namespace!=kube-amd-gpu');
    expect(PLUGIN_POD_QUERIES[1]).toBe('/api/v1/namespaces/kube-amd-gpu/pods');
  });
});

describe('isAmdGpuNode', () => {
  it('detects a node by the NFD amd-gpu label alone', () => {
    expect(isAmdGpuNode(makeGpuNode('a', { labels: false, capacity: false }))).toBe(true);
  });
  it('detects a node by node-labeller labels alone', () => {
    expect(isAmdGpuNode(makeGpuNode('a', { nfd: false, capacity: false }))).toBe(true);
  });
  it('detects a node by legacy beta.amd.com labels', () => {
    const n = makeNode('a');
    n.metadata.labels['beta.amd.com/gpu.family'] = 'AI';
    expect(isAmdGpuNode(n)).toBe(true);
  });
  it('detects a node by amd.com/gpu capacity alone', () => {
    expect(isAmdGpuNode(makeGpuNode('a', { labels: false, nfd: false }))).toBe(true);
  });
  it('detects partition resources in capacity', () => {
    const n = makeNode('a');
    n.status.capacity['amd.com/cpx_nps4'] = '64';
    expect(isAmdGpuNode(n)).toBe(true);
  });
  it('rejects a CPU node', () => {
    expect(isAmdGpuNode(makeNode('cpu'))).toBe(false);
  });
  it('rejects an NFD label that is not "true"', () => {
    const n = makeNode('a');
    n.metadata.labels['feature.node.kubernetes.io/amd-gpu'] = 'false';
    expect(isAmdGpuNode(n)).toBe(false);
  });
  it('rejects non-objects and objects without metadata', () => {
    expect(isAmdGpuNode(null)).toBe(false);
    expect(isAmdGpuNode('node')).toBe(false);
    expect(isAmdGpuNode({ status: { capacity: { 'amd.com/gpu': '8' } } })).toBe(false);
  });
  it('filterAmdGpuNodes keeps only GPU nodes', () => {
    const out = filterAmdGpuNodes([makeNode('c1'), makeGpuNode('g1'), makeNode('c2'), makeGpuNode('g2')]);
    expect(out.map((n) => n.metadata.name)).toEqual(['g1', 'g2']);
  });
  it('filterAmdGpuNodes tolerates a non-array', () => {
    expect(filterAmdGpuNodes(undefined)).toEqual([]);
  });
});

describe('node resources', () => {
  it('getGpuResources returns only amd.com/* keys', () => {
    const n = makeGpuNode('g');
    n.status.capacity['amd.com/cpx_nps4'] = '0';
    expect(getGpuResources(n.status.capacity)).toEqual({ 'amd.com/gpu': '8', 'amd.com/cpx_nps4': '0' });
  });
  it('getGpuResources of undefined is empty', () => {
    expect(getGpuResources(undefined)).toEqual({});
  });
  it('getNodeGpuCount reads amd.com/gpu capacity', () => {
    expect(getNodeGpuCount(makeGpuNode('g', { gpus: 8 }))).toBe(8);
    expect(getNodeGpuCount(makeGpuNode('g', { gpus: 1 }))).toBe(1);
  });
  it('getNodeGpuCount is 0 for a label-only node', () => {
    expect(getNodeGpuCount(makeGpuNode('g', { capacity: false }))).toBe(0);
  });
  it('getNodeGpuAllocatable reads allocatable separately from capacity', () => {
    expect(getNodeGpuAllocatable(makeGpuNode('g', { gpus: 8, allocatable: 7 }))).toBe(7);
  });
  it('getNodePartitionCount sums partition resources', () => {
    const n = makeGpuNode('g');
    n.status.capacity['amd.com/cpx_nps4'] = '32';
    n.status.capacity['amd.com/dpx_nps1'] = '4';
    expect(getNodePartitionCount(n)).toBe(36);
  });
  it('parseCount ignores junk and negatives', () => {
    expect(parseCount('8')).toBe(8);
    expect(parseCount('x')).toBe(0);
    expect(parseCount('-2')).toBe(0);
    expect(parseCount(undefined)).toBe(0);
  });
  it('isNodeReady reads the Ready condition', () => {
    expect(isNodeReady(makeGpuNode('g'))).toBe(true);
    expect(isNodeReady(makeGpuNode('g', { ready: false }))).toBe(false);
    expect(isNodeReady({ metadata: { name: 'x' } })).toBe(false);
  });
});

describe('GPU model', () => {
  it('reads the product from the node labeller', () => {
    const m = getNodeGpuModel(makeGpuNode('g'));
    expect(m.product).toBe('AMD Instinct MI355X');
    expect(m.fromLabels).toBe(true);
    expect(m.cuCount).toBe(256);
  });
  it('defaults to MI355X without labeller labels', () => {
    const m = getNodeGpuModel(makeGpuNode('g', { labels: false }));
    expect(m.product).toBe(MI355X.product);
    expect(m.fromLabels).toBe(false);
    expect(m.vram).toBe('288 GB HBM3E');
  });
  it('formats SPX nodes as the short name', () => {
    expect(formatGpuModel(getNodeGpuModel(makeGpuNode('g')))).toBe('MI355X');
  });
  it('formats partitioned nodes with their modes', () => {
    expect(formatGpuModel(getNodeGpuModel(makeGpuNode('g', { partition: 'cpx/nps4' })))).toBe('MI355X (CPX/NPS4)');
  });
  it('names the product from the device id amd-smi reports for MI355X', () => {
    // tests/fixtures/mi355x/amd_smi_static.json: device_id 0x75a3, market name "AMD Instinct MI355 OAM"
    expect(shortProductName('0x75a3', 'AMD Instinct MI355 OAM')).toBe('MI355X');
    expect(shortProductName('75A3', null)).toBe('MI355X');
  });
  it('falls back to the product string, then to MI355X', () => {
    expect(shortProductName(null, 'AMD_Instinct_MI300X')).toBe('MI300X');
    expect(shortProductName('74b5', 'AMD_Instinct_MI300X')).toBe('MI300X');
    expect(shortProductName(null, null)).toBe('MI355X');
  });
  it('uses the labeller product for a non-MI355X node', () => {
    const n = makeGpuNode('g');
    n.metadata.labels['amd.com/gpu.product-name'] = 'AMD_Instinct_MI325X';
    expect(formatGpuModel(getNodeGpuModel(n))).toBe('MI325X');
  });
});

describe('isGpuRequestingPod', () => {
  it('detects amd.com/gpu requests', () => {
    expect(isGpuRequestingPod(makeGpuPod('p'))).toBe(true);
  });
  it('detects limits-only GPU pods', () => {
    expect(isGpuRequestingPod(makeGpuPod('p', { limitsOnly: true }))).toBe(true);
  });
  it('detects partition resource requests', () => {
    expect(isGpuRequestingPod(makeGpuPod('p', { resource: 'amd.com/cpx_nps4' }))).toBe(true);
  });
  it('detects GPU init containers', () => {
    expect(isGpuRequestingPod(makeGpuPod('p', { gpus: 0, init: 1 }))).toBe(true);
  });
  it('rejects CPU-only pods', () => {
    expect(isGpuRequestingPod(makePlainPod('p'))).toBe(false);
  });
  it('rejects non-objects', () => {
    expect(isGpuRequestingPod(null)).toBe(false);
    expect(isGpuRequestingPod(42)).toBe(false);
  });
  it('filterGpuRequestingPods keeps only GPU pods', () => {
    expect(filterGpuRequestingPods([makePlainPod('a'), makeGpuPod('b')]).map((p) => p.metadata.name)).toEqual(['b']);
  });
});

describe('pod GPU demand', () => {
  it('sums regular containers', () => {
    const p = makeGpuPod('p', { gpus: 2 });
    p.spec.containers.push({ name: 'b', resources: { requests: { 'amd.com/gpu': '3' } } });
    expect(getPodGpuDemand(p)).toEqual({ 'amd.com/gpu': 5 });
  });
  it('falls back to limits for extended resources', () => {
    expect(getPodGpuCount(makeGpuPod('p', { gpus: 4, limitsOnly: true }))).toBe(4);
  });
  it('uses max(init, regular), not their sum', () => {
    expect(getPodGpuCount(makeGpuPod('p', { gpus: 2, init: 4 }))).toBe(4);
    expect(getPodGpuCount(makeGpuPod('p', { gpus: 4, init: 2 }))).toBe(4);
  });
  it('adds restartable sidecar init containers to the steady state', () => {
    const p = makeGpuPod('p', { gpus: 2 });
    p.spec.initContainers = [{ name: 'side', restartPolicy: 'Always', resources: { limits: { 'amd.com/gpu': '1' } } }];
    expect(getPodGpuCount(p)).toBe(3);
  });
  it('getPodGpuRequests returns strings', () => {
    expect(getPodGpuRequests(makeGpuPod('p', { gpus: 8 }))).toEqual({ 'amd.com/gpu': '8' });
  });
  it('containerGpuEntries reports request, limit and effective', () => {
    const c = { name: 'c', resources: { requests: { 'amd.com/gpu': '1' }, limits: { 'amd.com/gpu': '2' } } };
    expect(containerGpuEntries(c)).toEqual([{ key: 'amd.com/gpu', request: '1', limit: '2', effective: 1 }]);
  });
  it('formatPodGpuRequests renders display names', () => {
    expect(formatPodGpuRequests(makeGpuPod('p', { gpus: 2 }))).toBe('GPU: 2');
    expect(formatPodGpuRequests(makePlainPod('p'))).toBe('—');
  });
});

describe('pod status helpers', () => {
  it('isPodReady reads the Ready condition', () => {
    expect(isPodReady(makeGpuPod('p'))).toBe(true);
    expect(isPodReady(makeGpuPod('p', { phase: 'Pending' }))).toBe(false);
  });
  it('getPodRestarts sums container restarts', () => {
    const p = makeGpuPod('p', { restarts: 2 });
    p.status.containerStatuses.push({ name: 'x', ready: true, restartCount: 3 });
    expect(getPodRestarts(p)).toBe(5);
  });
  it('getPodRestarts is 0 without statuses', () => {
    expect(getPodRestarts({ metadata: { name: 'x' } })).toBe(0);
  });
  it('podWaitingReason reads container waiting state', () => {
    expect(podWaitingReason(makeGpuPod('p', { phase: 'Pending', waiting: 'ContainerCreating' }))).toBe('ContainerCreating');
  });
  it('podWaitingReason falls back to the scheduler condition', () => {
    const p = makeGpuPod('p', { phase: 'Pending', node: null });
    p.status.containerStatuses = [];
    p.status.conditions = [{ type: 'PodScheduled', status: 'False', reason: 'Unschedulable' }];
    expect(podWaitingReason(p)).toBe('Unschedulable');
  });
  it('podWaitingMessage: the scheduler\'s explanation, or the waiting container\'s message', () => {
    const p = makeGpuPod('p', { phase: 'Pending', node: null });
    p.status.containerStatuses = [];
    p.status.conditions = [{ type: 'PodScheduled', status: 'False', reason: 'Unschedulable', message: '0/8 nodes are available: 8 Insufficient amd.com/gpu.' }];
    expect(podWaitingMessage(p)).toBe('0/8 nodes are available: 8 Insufficient amd.com/gpu.');
    const q = makeGpuPod('q', { phase: 'Pending', waiting: 'ImagePullBackOff' });
    q.status.containerStatuses[0].state.waiting.message = 'Back-off pulling image "rocm/pytorch:bad"';
    expect(podWaitingMessage(q)).toBe('Back-off pulling image "rocm/pytorch:bad"');
    expect(podWaitingMessage(makeGpuPod('r'))).toBeNull();
  });
  it('phaseToStatus maps phases', () => {
    expect(phaseToStatus('Running')).toBe('success');
    expect(phaseToStatus('Succeeded')).toBe('success');
    expect(phaseToStatus('Pending')).toBe('warning');
    expect(phaseToStatus('Failed')).toBe('error');
    expect(phaseToStatus('Unknown')).toBe('warning');
  });
});

describe('plugin pods', () => {
  it('classifies the standalone device-plugin DaemonSet', () => {
    expect(pluginPodComponent(makePluginPod('dp'))).toBe('device-plugin');
  });
  it('classifies the standalone labeller DaemonSet', () => {
    expect(pluginPodComponent(makePluginPod('lb', { label: 'amdgpu-labeller-ds' }))).toBe('node-labeller');
  });
  it('classifies operator operands by namespace and name', () => {
    const mk = (n) => makePluginPod(n, { label: null, ns: 'kube-amd-gpu' });
    expect(pluginPodComponent(mk('gpu-operator-device-plugin-abcde'))).toBe('device-plugin');
    expect(pluginPodComponent(mk('gpu-operator-node-labeller-abcde'))).toBe('node-labeller');
    expect(pluginPodComponent(mk('gpu-operator-metrics-exporter-abcde'))).toBe('metrics-exporter');
    expect(pluginPodComponent(mk('amd-gpu-operator-controller-manager-1'))).toBe('operator');
  });
  it('ignores unrelated pods in other namespaces', () => {
    expect(isAmdGpuPluginPod(makePluginPod('x', { label: 'nginx' }))).toBe(false);
    expect(isAmdGpuPluginPod(makePluginPod('device-plugin-x', { label: null, ns: 'default' }))).toBe(false);
  });
  it('filterAmdGpuPluginPods filters', () => {
    expect(filterAmdGpuPluginPods([makePluginPod('a'), makePlainPod('b')])).toHaveLength(1);
  });
  it('dedupePods keeps uid-less pods by namespace/name', () => {
    const a = makePluginPod('a', { uid: '' });
    const b = makePluginPod('a', { uid: '' });
    const c = makePluginPod('c');
    expect(dedupePods([a, b, c, c])).toHaveLength(2);
  });
});

describe('DeviceConfig', () => {
  it('isDeviceConfig checks the kind', () => {
    expect(isDeviceConfig(makeDeviceConfig())).toBe(true);
    expect(isDeviceConfig({ kind: 'GpuDevicePlugin', metadata: {} })).toBe(false);
    expect(isDeviceConfig(null)).toBe(false);
  });
  it('operandEnabled follows the spec', () => {
    const dc = makeDeviceConfig('x', { exporter: false, labeller: true });
    expect(operandEnabled(dc, 'devicePlugin')).toBe(true);
    expect(operandEnabled(dc, 'metricsExporter')).toBe(false);
    expect(operandEnabled(dc, 'nodeLabeller')).toBe(true);
    expect(operandEnabled(dc, 'driver')).toBe(false);
  });
  it('operandStatus derives unavailable', () => {
    expect(operandStatus(makeDeviceConfig('x', { desired: 4, available: 1 }), 'devicePlugin')).toEqual({
      desired: 4, available: 1, unavailable: 3, matching: 4,
    });
  });
  it('countsToStatus covers every branch', () => {
    expect(countsToStatus(0, 0)).toBe('warning');
    expect(countsToStatus(4, 4)).toBe('success');
    expect(countsToStatus(4, 2)).toBe('warning');
    expect(countsToStatus(4, 0)).toBe('error');
  });
  it('countsToText', () => {
    expect(countsToText(0, 0)).toBe('No nodes scheduled');
    expect(countsToText(8, 7)).toBe('7/8 ready');
  });
  it('deviceConfigStatus is the worst enabled operand', () => {
    expect(deviceConfigStatus(makeDeviceConfig())).toBe('success');
    expect(deviceConfigStatus(makeDeviceConfig('x', { available: 0 }))).toBe('error');
    const dc = makeDeviceConfig();
    dc.status.metricsExporter.availableNumber = 1;
    expect(deviceConfigStatus(dc)).toBe('warning');
  });
  it('deviceConfigStatusText reports device-plugin readiness', () => {
    expect(deviceConfigStatusText(makeDeviceConfig('x', { desired: 4, available: 3 }))).toBe('3/4 ready');
  });
  it('formatSelector renders k=v pairs', () => {
    expect(formatSelector({ a: '1', b: '2' })).toBe('a=1, b=2');
    expect(formatSelector({})).toBe('—');
    expect(formatSelector(undefined)).toBe('—');
  });
});

describe('isKubeList / unwrap', () => {
  it('isKubeList accepts item arrays only', () => {
    expect(isKubeList({ items: [] })).toBe(true);
    expect(isKubeList({ items: 'x' })).toBe(false);
    expect(isKubeList(null)).toBe(false);
  });
  it('unwrapKubeObject returns jsonData', () => {
    const raw = makeGpuNode('g');
    expect(unwrapKubeObject({ jsonData: raw })).toBe(raw);
    expect(unwrapKubeObject(raw)).toBe(raw);
  });
  it('unwrapAll maps lists and tolerates null', () => {
    expect(unwrapAll([{ jsonData: 1 }, 2])).toEqual([{ jsonData: 1 }, 2]);
    expect(unwrapAll(null)).toEqual([]);
  });
});

describe('buildClusterIndex', () => {
  const nodes = [makeGpuNode('n0'), makeGpuNode('n1', { allocatable: 7 })];
  const pods = [
    makeGpuPod('a', { node: 'n0', gpus: 4 }),
    makeGpuPod('b', { node: 'n0', gpus: 2, phase: 'Pending' }),
    makeGpuPod('c', { node: 'n1', gpus: 8, phase: 'Succeeded' }),
    makeGpuPod('d', { node: null, phase: 'Pending' }),
  ];
  const idx = buildClusterIndex(nodes, pods);
  it('sums capacity and allocatable', () => {
    expect(idx.totals.capacity).toBe(16);
    expect(idx.totals.allocatable).toBe(15);
  });
  it('counts GPUs held by bound non-terminal pods', () => {
    expect(idx.nodeStats.get('n0').inUse).toBe(6);
    expect(idx.nodeStats.get('n1').inUse).toBe(0);
    expect(idx.totals.inUse).toBe(6);
  });
  it('indexes pods by node', () => {
    expect(idx.podsByNode.get('n0').map((p) => p.metadata.name)).toEqual(['a', 'b']);
    expect(idx.nodeStats.get('n1').pods).toBe(1);
  });
  it('counts phases including unbound pods', () => {
    expect(idx.phases).toEqual({ Running: 1, Pending: 2, Succeeded: 1, Failed: 0, Other: 0 });
  });
  it('clamps free at zero when over-committed', () => {
    const i2 = buildClusterIndex([makeGpuNode('x', { gpus: 2 })], [makeGpuPod('p', { node: 'x', gpus: 4 })]);
    expect(i2.totals.free).toBe(0);
  });
  it('computes utilisation percent', () => {
    expect(idx.totals.utilizationPct).toBe(40);
  });
});

describe('formatters', () => {
  it('formatAge covers s/m/h/d', () => {
    expect(formatAge(ago(30), NOW)).toBe('30s');
    expect(formatAge(ago(5 * 60), NOW)).toBe('5m');
    expect(formatAge(ago(3 * 3600), NOW)).toBe('3h');
    expect(formatAge(ago(2 * 86400), NOW)).toBe('2d');
  });
  it('formatAge with missing or bad timestamps', () => {
    expect(formatAge(undefined, NOW)).toBe('unknown');
    expect(formatAge('not-a-date', NOW)).toBe('unknown');
  });
  it('formatAge uses Date.now by default', () => {
    expect(formatAge(new Date(Date.now() - 10000).toISOString())).toMatch(/^(9|10|11)s$/);
  });
  it('formatGpuResourceName maps AMD resources', () => {
    expect(formatGpuResourceName('amd.com/gpu')).toBe('GPU');
    expect(formatGpuResourceName('amd.com/cpx_nps4')).toBe('GPU partition (CPX/NPS4)');
    expect(formatGpuResourceName('amd.com/other')).toBe('other');
    expect(formatGpuResourceName('nvidia.com/gpu')).toBe('nvidia.com/gpu');
  });
  it('formatBytes uses decimal units', () => {
    expect(formatBytes(288 * 1024 ** 3)).toBe('288 GiB');
    expect(formatBytes(8 * 288 * 1024 ** 3)).toBe('2.25 TiB');
    expect(formatBytes(512)).toBe('512 B');
    expect(formatBytes(null)).toBe('—');
  });
  it('formatWatts / formatPercent', () => {
    expect(formatWatts(1234.56)).toBe('1234.6 W');
    expect(formatPercent(50, 200)).toBe('25%');
    expect(formatPercent(5, 0)).toBe('—');
  });
  it('pct / pctToStatus / pctToColor thresholds', () => {
    expect(pct(1, 3)).toBe(33);
    expect(pct(1, 0)).toBe(0);
    expect(pctToStatus(69)).toBe('success');
    expect(pctToStatus(70)).toBe('warning');
    expect(pctToStatus(90)).toBe('error');
    expect(pctToColor(95)).toBe('#d32f2f');
    expect(pctToColor(75)).toBe('#f57c00');
  });
});

describe('nextAgeChange', () => {
  it('is the first instant at which formatAge shows a different label', () => {
    let a = 7;
    const r = () => {
      a = (a * 1103515245 + 12345) % 2147483648;
      return a / 2147483648;
    };
    const t0 = Date.UTC(2026, 0, 1);
    for (let i = 0; i < 2000; i++) {
      const ts = new Date(t0 + Math.floor(r() * 1e9)).toISOString();
      // ages from "in the future" (clock skew) to ~40 days
      const now = t0 + Math.floor(r() * 1e9) + Math.floor((r() - 0.05) * 40 * 86400000);
      const next = nextAgeChange(ts, now);
      expect(next).toBeGreaterThan(now);
      expect(formatAge(ts, next - 1)).toBe(formatAge(ts, now));
      expect(formatAge(ts, next)).not.toBe(formatAge(ts, now));
    }
  });
  it('never changes for a missing or unparseable timestamp', () => {
    expect(nextAgeChange(undefined, 0)).toBe(Infinity);
    expect(nextAgeChange('not a time', 0)).toBe(Infinity);
  });
});

describe('isNamedObject: what the views can name', () => {
  it('needs a non-empty string name; namespace and uid are strings when present', () => {
    expect(isNamedObject(makeGpuNode('g0'))).toBe(true);
    expect(isNamedObject(makeGpuPod('p'))).toBe(true);
    expect(isNamedObject({ metadata: { name: 'x', namespace: null, uid: undefined } })).toBe(true);
    for (const name of [undefined, null, '', 7, {}, { a: 1 }, [], ['x'], true]) {
      expect(isNamedObject({ metadata: { name } })).toBe(false);
    }
    expect(isNamedObject({ metadata: { name: 'x', namespace: { a: 1 } } })).toBe(false);
    expect(isNamedObject({ metadata: { name: 'x', uid: 3 } })).toBe(false);
    expect(isNamedObject(null)).toBe(false);
    expect(isNamedObject({ metadata: [] })).toBe(false);
  });

  it('an AMD node, GPU pod, operator pod or DeviceConfig without a usable name is not classified as one', () => {
    const node = makeGpuNode('g0');
    const pod = makeGpuPod('p');
    const dp = makePluginPod('dp');
    const dc = makeDeviceConfig();
    const unnamed = (o) => Object.assign({}, o, { metadata: Object.assign({}, o.metadata, { name: { a: 1 } }) });
    expect(isAmdGpuNode(node) && !isAmdGpuNode(unnamed(node))).toBe(true);
    expect(isGpuRequestingPod(pod) && !isGpuRequestingPod(unnamed(pod))).toBe(true);
    expect(isAmdGpuPluginPod(dp) && !isAmdGpuPluginPod(unnamed(dp))).toBe(true);
    expect(isDeviceConfig(dc) && !isDeviceConfig(unnamed(dc))).toBe(true);
  });
});
