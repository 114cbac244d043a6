/**
 * Page view-model specs — the analog of the reference's component tests
 * (OverviewPage.test.tsx 9, DevicePluginsPage.test.tsx 6, NodesPage.test.tsx 5,
 * PodsPage.test.tsx 6, MetricsPage.test.tsx 9). Assertions target section
 * titles, row labels, status values and refresh aria-labels, as there.
 */
import { allocationBar, eccCell, formatWindow, hbmBar, localTimeText, powerBar, tempCell } from '../../src/view/pages/common.js';
import { nodeDetailView, podDetailView } from '../../src/view/pages/details.js';
import { devicePluginsView } from '../../src/view/pages/devicePlugins.js';
import { metricsView } from '../../src/view/pages/metricsPage.js';
import { formatTaints, nodePowerKeys, nodeReadyCell, nodesView, nodeTempKeys } from '../../src/view/pages/nodes.js';
import { ACTIVE_PODS_LIMIT, overviewView } from '../../src/view/pages/overview.js';
import { gpuContainerLines, podGpuAssignments, podsView } from '../../src/view/pages/pods.js';
import { countRows, findSection, firstBlock, firstTable, loaders, rowNames, rowValue, sectionTitles, text } from '../../src/view/ir.js';
import { renderPage, textContent } from '../../src/view/html.js';
import { SERIES } from '../../src/api/series.js';
import { clusterPowerStats, joinExporterResults } from '../../src/api/telemetry.js';
import { NOW, makeContext, makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from './fixtures.js';
import { MI355X } from '../../src/api/k8sCore.js';
import { assignedLines } from '../../src/view/pages/pods.js';

const opts = { now: NOW };

// ---------------------------------------------------------------------------
describe('overviewView', () => {
  it('shows only the loader on first load', () => {
    const vm = overviewView(makeContext({ loading: true, lastUpdated: null }), opts);
    expect(loaders(vm)).toEqual(['Loading AMD GPU data...']);
    expect(vm.title).toBeNull();
  });

  it('keeps content visible during a refresh (no loader swap)', () => {
    // The store keeps `loading` false once everything settled; a refresh only sets `refreshing`.
    const vm = overviewView(makeContext({ loading: false, refreshing: true, nodes: [makeGpuNode('g')] }), opts);
    expect(loaders(vm)).toEqual([]);
    expect(vm.refresh.label).toBe('Refreshing…');
    expect(vm.refresh.disabled).toBe(true);
  });

  it('shows the loader while a list is still in flight even if the CRD answered', () => {
    const vm = overviewView(makeContext({ loading: true, lastUpdated: 1, nodes: [makeGpuNode('g')] }), opts);
    expect(loaders(vm)).toEqual(['Loading AMD GPU data...']);
  });

  it('has the page header and refresh aria-label', () => {
    const vm = overviewView(makeContext(), opts);
    expect(vm.title).toBe('AMD GPU — Overview');
    expect(vm.refresh.ariaLabel).toBe('Refresh AMD GPU data');
  });

  it('shows "Plugin Not Detected" with install instructions when nothing is installed', () => {
    const vm = overviewView(makeContext(), opts);
    const s = findSection(vm, 'Plugin Not Detected');
    expect(s).not.toBeNull();
    expect(text(rowValue(s, 'Install (Helm)'))).toContain('gpu-operator-charts');
    expect(rowValue(s, 'Status').status).toBe('warning');
  });

  it('shows the CRD notice when plugin pods exist without the CRD', () => {
    const vm = overviewView(makeContext({ pluginPods: [makePluginPod('dp')] }), opts);
    expect(sectionTitles(vm)).toContain('Notice');
    expect(sectionTitles(vm)).not.toContain('Plugin Not Detected');
  });

  it('renders the DeviceConfig status table when the CRD exists', () => {
    const vm = overviewView(makeContext({ crdAvailable: true, deviceConfigs: [makeDeviceConfig('cfg', { desired: 4, available: 3 })] }), opts);
    const t = firstTable(findSection(vm, 'Device Config Status'));
    expect(t.columns).toEqual(['Name', 'Namespace', 'Status', 'Metrics Exporter', 'Node Labeller', 'Selector', 'Age']);
    expect(t.rows[0][0]).toBe('cfg');
    expect(t.rows[0][2]).toEqual({ t: 'status', status: 'warning', text: '3/4 ready' });
    expect(t.rows[0][6]).toBe('3d');
  });

  it('lists plugin daemon pods with their component', () => {
    const vm = overviewView(makeContext({ pluginPods: [makePluginPod('dp-0'), makePluginPod('lb-0', { label: 'amdgpu-labeller-ds', ready: false })] }), opts);
    const t = firstTable(findSection(vm, 'Plugin Daemon Pods'));
    expect(t.rows.map((r) => r[2])).toEqual(['Device Plugin', 'Node Labeller']);
    expect(t.rows[1][4].status).toBe('warning');
  });

  it('summarises GPU nodes with MI355X model and HBM', () => {
    const vm = overviewView(makeContext({ nodes: [makeGpuNode('a'), makeGpuNode('b', { ready: false })] }), opts);
    const s = findSection(vm, 'GPU Nodes');
    expect(rowValue(s, 'Total GPU Nodes')).toEqual({ t: 'status', status: 'success', text: '2' });
    expect(rowValue(s, 'Ready Nodes')).toBe('1');
    expect(rowValue(s, 'Total GPU Devices')).toBe('16');
    expect(rowValue(s, 'Total HBM')).toContain('4.5 TiB');
    expect(text(rowValue(s, 'GPU Model'))).toContain('MI355X');
  });

  it('shows the partition-mode distribution of GPU nodes', () => {
    const vm = overviewView(makeContext({ nodes: [makeGpuNode('a'), makeGpuNode('b', { partition: 'cpx/nps4' }), makeGpuNode('c')] }), opts);
    const bars = findSection(vm, 'GPU Nodes').blocks.filter((b) => b.t === 'pctbar');
    const modes = bars.find((b) => b.label === 'GPU Partition Modes');
    expect(modes.data.map((d) => [d.name, d.value])).toEqual([['SPX/NPS1', 2], ['CPX/NPS4', 1]]);
    expect(modes.total).toBe(3);
  });

  it('warns when there are zero GPU nodes', () => {
    const vm = overviewView(makeContext({ nodes: [makeNode('cpu')] }), opts);
    expect(rowValue(findSection(vm, 'GPU Nodes'), 'Total GPU Nodes').status).toBe('warning');
    expect(findSection(vm, 'GPU Allocation')).toBeNull();
  });

  it('computes allocation from GPUs held', () => {
    const ctx = makeContext({
      nodes: [makeGpuNode('g0')],
      pods: [makeGpuPod('a', { node: 'g0', gpus: 4 }), makeGpuPod('b', { node: 'g0', gpus: 2, phase: 'Succeeded' })],
    });
    const s = findSection(overviewView(ctx, opts), 'GPU Allocation');
    expect(rowValue(s, 'In Use')).toBe('4');
    expect(rowValue(s, 'Free')).toEqual({ t: 'status', status: 'success', text: '4' });
    expect(firstBlock(s, 'pctbar').label).toBe('GPU Allocation (50%)');
  });

  it('warns when no GPU is free', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0', { gpus: 1 })], pods: [makeGpuPod('a', { node: 'g0', gpus: 1 })] });
    expect(rowValue(findSection(overviewView(ctx, opts), 'GPU Allocation'), 'Free').status).toBe('warning');
  });

  it('counts workload phases', () => {
    const ctx = makeContext({
      nodes: [makeGpuNode('g0')],
      pods: [makeGpuPod('a'), makeGpuPod('b', { phase: 'Pending' }), makeGpuPod('c', { phase: 'Failed' })],
    });
    const s = findSection(overviewView(ctx, opts), 'GPU Workloads');
    expect(rowNames(s)).toEqual(['Total GPU Pods', 'Running', 'Pending', 'Failed']);
    expect(rowValue(s, 'Failed').status).toBe('error');
  });

  it('caps Active GPU Pods at the first 10 running', () => {
    const pods = [];
    for (let i = 0; i < 15; i++) pods.push(makeGpuPod('p' + i));
    pods.push(makeGpuPod('pending', { phase: 'Pending' }));
    const t = firstTable(findSection(overviewView(makeContext({ nodes: [makeGpuNode('mi355x-0')], pods }), opts), 'Active GPU Pods'));
    expect(t.rows).toHaveLength(ACTIVE_PODS_LIMIT);
    expect(t.rows[0][3]).toBe('GPU: 1');
  });

  it('surfaces the aggregated error', () => {
    const vm = overviewView(makeContext({ error: 'nodes forbidden' }), opts);
    expect(rowValue(findSection(vm, 'Error'), 'Status')).toEqual({ t: 'status', status: 'error', text: 'nodes forbidden' });
  });
});

// ---------------------------------------------------------------------------
describe('devicePluginsView', () => {
  it('a forbidden DeviceConfig list says which permission is missing, not "not installed"', () => {
    const vm = devicePluginsView(makeContext({ crdAvailable: false, crdForbidden: true }), opts);
    const s = findSection(vm, 'CRD Not Available');
    expect(rowValue(s, 'Status').text).toBe('DeviceConfig list forbidden for this user (HTTP 403)');
    expect(rowValue(s, 'Note')).toContain('deviceconfigs.amd.com');
    const absent = findSection(devicePluginsView(makeContext({ crdAvailable: false }), opts), 'CRD Not Available');
    expect(rowValue(absent, 'Status').text).toContain('not installed');
  });
  it('test runner / config manager operands show when the DeviceConfig names them, pods when its status counts them', () => {
    const dc = makeDeviceConfig('gpu-operator');
    dc.spec.testRunner = { enable: true };
    dc.spec.configManager = { enable: false };
    dc.status.testRunner = { nodesMatchingSelectorNumber: 2, desiredNumber: 2, availableNumber: 1 };
    const s = findSection(devicePluginsView(makeContext({ deviceConfigs: [dc] }), opts), 'DeviceConfig: gpu-operator');
    expect(rowValue(s, 'Test Runner')).toEqual({ t: 'status', status: 'warning', text: 'Enabled · 1/2 ready' });
    expect(rowValue(s, 'Config Manager')).toEqual({ t: 'status', status: 'warning', text: 'Disabled' });
    // a new object (the store's objects are immutable snapshots; their facts are derived once)
    const dc2 = JSON.parse(JSON.stringify(dc));
    delete dc2.status.testRunner;
    const uncounted = findSection(devicePluginsView(makeContext({ deviceConfigs: [dc2] }), opts), 'DeviceConfig: gpu-operator');
    expect(rowValue(uncounted, 'Test Runner')).toEqual({ t: 'status', status: 'success', text: 'Enabled' });
    const plain = findSection(devicePluginsView(makeContext({ deviceConfigs: [makeDeviceConfig('gpu-operator')] }), opts), 'DeviceConfig: gpu-operator');
    expect(rowValue(plain, 'Test Runner')).toBeUndefined();
  });
  it('shows the loader on first load', () => {
    expect(loaders(devicePluginsView(makeContext({ loading: true, lastUpdated: null }), opts))).toEqual(['Loading device plugin data...']);
  });
  it('has header and aria-label', () => {
    const vm = devicePluginsView(makeContext(), opts);
    expect(vm.title).toBe('AMD GPU — Device Plugins');
    expect(vm.refresh.ariaLabel).toBe('Refresh device plugin data');
  });
  it('shows "CRD Not Available" without the CRD', () => {
    const s = findSection(devicePluginsView(makeContext(), opts), 'CRD Not Available');
    expect(text(rowValue(s, 'Status'))).toContain('amd.com/v1alpha1');
  });
  it('shows "No Device Configs" when the CRD exists but is empty', () => {
    const vm = devicePluginsView(makeContext({ crdAvailable: true }), opts);
    expect(sectionTitles(vm)).toContain('No Device Configs');
    expect(sectionTitles(vm)).not.toContain('CRD Not Available');
  });
  it('renders one card per DeviceConfig with operand rows', () => {
    const vm = devicePluginsView(makeContext({ crdAvailable: true, deviceConfigs: [makeDeviceConfig('a'), makeDeviceConfig('b', { exporter: false })] }), opts);
    const a = findSection(vm, 'DeviceConfig: a');
    expect(rowValue(a, 'Status')).toEqual({ t: 'status', status: 'success', text: '2/2 ready' });
    // the operand and its DaemonSet's pods in one row
    expect(rowValue(a, 'Metrics Exporter')).toEqual({ t: 'status', status: 'success', text: 'Enabled — port 5000 · 2/2 ready' });
    expect(rowNames(a).filter((n) => / Pods$/.test(n))).toEqual([]);
    expect(rowValue(findSection(vm, 'DeviceConfig: b'), 'Metrics Exporter').status).toBe('warning');
    expect(rowValue(a, 'Node Selector')).toBe('feature.node.kubernetes.io/amd-gpu=true');
  });
  it('shows Unavailable Nodes only when some are unavailable', () => {
    const vm = devicePluginsView(makeContext({ crdAvailable: true, deviceConfigs: [makeDeviceConfig('a', { desired: 4, available: 1 })] }), opts);
    expect(rowValue(findSection(vm, 'DeviceConfig: a'), 'Unavailable Nodes')).toEqual({ t: 'status', status: 'error', text: '3' });
    const vm2 = devicePluginsView(makeContext({ crdAvailable: true, deviceConfigs: [makeDeviceConfig('a')] }), opts);
    expect(rowNames(findSection(vm2, 'DeviceConfig: a'))).not.toContain('Unavailable Nodes');
  });
  it('lists daemon pods with restarts flagged', () => {
    const vm = devicePluginsView(makeContext({ pluginPods: [makePluginPod('dp-0', { restarts: 3 }), makePluginPod('dp-1')] }), opts);
    const t = firstTable(findSection(vm, 'Plugin Daemon Pods'));
    expect(t.columns).toEqual(['Name', 'Namespace', 'Component', 'Node', 'Ready', 'Restarts', 'Age']);
    expect(t.rows[0][5]).toEqual({ t: 'status', status: 'warning', text: '3' });
    expect(t.rows[1][5]).toBe('0');
  });
  it('surfaces errors', () => {
    expect(sectionTitles(devicePluginsView(makeContext({ error: 'x' }), opts))[0]).toBe('Error');
  });
});

// ---------------------------------------------------------------------------
describe('overview: cordoned nodes', () => {
  it('counts cordoned nodes and the free GPUs new pods can still get', () => {
    const a = makeGpuNode('g0');
    const b = makeGpuNode('g1');
    b.spec = { unschedulable: true };
    const ctx = makeContext({ nodes: [a, b], pods: [makeGpuPod('x', { node: 'g0', gpus: 6 })] });
    const vm = overviewView(ctx, opts);
    expect(rowValue(findSection(vm, 'GPU Nodes'), 'Cordoned Nodes').text).toBe('1 (SchedulingDisabled)');
    const alloc = findSection(vm, 'GPU Allocation');
    expect(rowValue(alloc, 'Free').text).toBe('10');
    expect(rowValue(alloc, 'Free on Schedulable Nodes').text).toBe('2');
    // no cordon: no extra rows
    const plain = overviewView(makeContext({ nodes: [makeGpuNode('g0')] }), opts);
    expect(rowValue(findSection(plain, 'GPU Allocation'), 'Free on Schedulable Nodes')).toBeUndefined();
    expect(rowValue(findSection(plain, 'GPU Nodes'), 'Cordoned Nodes')).toBeUndefined();
  });
});

describe('nodesView: live node power', () => {
  it('adds a Power column (GPUs summed against their caps) when telemetry is there, whole watts', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0'), makeGpuNode('g1')] });
    const g = (node, i, w) => ({ nodeName: node, gpu: String(i), powerWatts: w, powerCapWatts: 1400 });
    const metrics = { source: 'amd-exporter', gpus: [g('g0', 0, 700.4), g('g0', 1, 699.8), g('g1', 0, NaN)], xgmi: {}, links: {} };
    const t = firstTable(findSection(nodesView(ctx, { now: NOW, metrics }), 'GPU Node Summary'));
    const col = t.columns.indexOf('Power');
    expect(col).toBe(t.columns.length - 2); // before Age
    expect(t.rows[0][col].text).toBe('1400.0 W / 2800.0 W (50%)');
    expect(t.rows[1][col]).toBe('—');
    expect(nodePowerKeys(metrics).byNode).toEqual({ g0: '1400|2800' });
    const plain = firstTable(findSection(nodesView(ctx, { now: NOW }), 'GPU Node Summary'));
    expect(plain.columns).not.toContain('Power');
  });
});

describe('nodesView: hottest GPU', () => {
  it('adds a Hottest GPU column (max junction °C per node, coloured against its throttle limit) when temperatures are there', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0'), makeGpuNode('g1')] });
    const g = (node, i, t) => ({ nodeName: node, gpu: String(i), powerWatts: 700, powerCapWatts: 1400, tempC: t, tempSlowdownC: 100 });
    const metrics = { source: 'amd-exporter', gpus: [g('g0', 0, 61.2), g('g0', 1, 93.6), g('g1', 0, null)], xgmi: {}, links: {} };
    const t = firstTable(findSection(nodesView(ctx, { now: NOW, metrics }), 'GPU Node Summary'));
    const col = t.columns.indexOf('Hottest GPU');
    expect(col).toBe(t.columns.length - 2); // after Power, before Age
    expect(t.rows[0][col]).toEqual({ t: 'status', status: 'warning', text: '94 °C' });
    expect(t.rows[1][col]).toBe('—');
    expect(nodeTempKeys(metrics).byNode).toEqual({ g0: '94|100|warning' });
    const plain = firstTable(findSection(nodesView(ctx, { now: NOW }), 'GPU Node Summary'));
    expect(plain.columns).not.toContain('Hottest GPU');
  });

  it('classifies the hottest GPU from its unrounded reading, as the Metrics page does (99.6 °C under 100 °C is a warning)', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0'), makeGpuNode('g1'), makeGpuNode('g2')] });
    const g = (node, t) => ({ nodeName: node, gpu: '0', powerWatts: 700, powerCapWatts: 1400, tempC: t, tempSlowdownC: 100 });
    const metrics = { source: 'amd-exporter', gpus: [g('g0', 99.6), g('g1', 100), g('g2', 89.5)], xgmi: {}, links: {} };
    const t = firstTable(findSection(nodesView(ctx, { now: NOW, metrics }), 'GPU Node Summary'));
    const col = t.columns.indexOf('Hottest GPU');
    expect(t.rows[0][col]).toEqual({ t: 'status', status: 'warning', text: '100 °C' });
    expect(tempCell(metrics.gpus[0])).toEqual({ t: 'status', status: 'warning', text: '100 °C' });
    expect(t.rows[1][col]).toEqual({ t: 'status', status: 'error', text: '100 °C (throttling at 100 °C)' });
    expect(t.rows[2][col]).toBe('90 °C'); // 89.5 is below the warning band, though it rounds to 90
  });
});

describe('nodesView', () => {
  it('a cordoned GPU node reads "Ready, SchedulingDisabled" (warning) and its card lists the taints', () => {
    const n = makeGpuNode('g0');
    n.spec = { unschedulable: true, taints: [{ key: 'amd.com/gpu', value: 'present', effect: 'NoSchedule' }, { key: 'node.kubernetes.io/unschedulable', effect: 'NoSchedule' }] };
    const vm = nodesView(makeContext({ nodes: [n] }), opts);
    const t = firstTable(findSection(vm, 'GPU Node Summary'));
    expect(t.rows[0][1]).toEqual({ t: 'status', status: 'warning', text: 'Ready, SchedulingDisabled' });
    const card = findSection(vm, 'g0');
    expect(rowValue(card, 'Taints')).toBe('amd.com/gpu=present:NoSchedule, node.kubernetes.io/unschedulable:NoSchedule');
    // readiness, model and age are the summary row's, not repeated on the card
    expect(rowValue(card, 'Status')).toBeUndefined();
    expect(rowValue(card, 'GPU Model')).toBeUndefined();
    // an untainted, schedulable node: plain "Ready", no Taints row
    const plain = nodesView(makeContext({ nodes: [makeGpuNode('g1')] }), opts);
    expect(rowValue(findSection(plain, 'g1'), 'Taints')).toBeUndefined();
    expect(nodeReadyCell(makeGpuNode('g1'))).toEqual({ t: 'status', status: 'success', text: 'Ready' });
    expect(formatTaints({ spec: {} })).toBeNull();
  });
  it('shows the loader on first load', () => {
    expect(loaders(nodesView(makeContext({ loading: true, lastUpdated: null }), opts))).toEqual(['Loading GPU node data...']);
  });
  it('shows "No GPU Nodes Found" on a CPU cluster', () => {
    const vm = nodesView(makeContext({ nodes: [makeNode('c')] }), opts);
    expect(sectionTitles(vm)).toEqual(['No GPU Nodes Found']);
    expect(vm.refresh.ariaLabel).toBe('Refresh node data');
  });
  it('renders the summary table with GPU-based allocation', () => {
    const ctx = makeContext({
      nodes: [makeGpuNode('g0'), makeGpuNode('g1')],
      pods: [makeGpuPod('a', { node: 'g0', gpus: 6 }), makeGpuPod('b', { node: 'g0', gpus: 1 }), makeGpuPod('c', { node: 'g1', gpus: 1 })],
    });
    const t = firstTable(findSection(nodesView(ctx, opts), 'GPU Node Summary'));
    expect(t.columns).toEqual(['Node', 'Ready', 'GPU Model', 'GPU Devices', 'Allocation', 'GPU Pods', 'Age']);
    expect(t.rows[0][4].text).toBe('7/8 (88%)');
    expect(t.rows[0][4].color).toBe('#f57c00');
    expect(t.rows[0][5]).toBe('2');
    expect(t.rows[1][4].text).toBe('1/8 (13%)');
  });
  it('renders one card per node with HBM and workload pods', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0', gpus: 2 })] });
    const s = findSection(nodesView(ctx, opts), 'g0');
    // one amd.com/gpu resource: capacity and allocatable on the device row; OS, kernel and kubelet on one row
    expect(rowValue(s, 'GPU Devices (amd.com/gpu) · HBM')).toBe('8 · capacity 8, allocatable 8 · HBM 2.25 TiB (8 × 288G)');
    expect(rowValue(s, 'GPU Workload Pods')).toBe('a');
    expect(rowValue(s, 'GPU (capacity)')).toBeUndefined();
    expect(rowValue(s, 'OS / Kernel / Kubelet / amdgpu')).toBe('Ubuntu 24.04 LTS · 6.8.0-45-generic · v1.31.2 · amdgpu 6.12.12');
  });
  it('adds per-GPU slots and the xGMI matrix to each card', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0', gpus: 3 })] });
    const s = findSection(nodesView(ctx, opts), 'g0');
    const slots = firstBlock(s, 'slots');
    expect(slots.slots.filter((x) => x.pod === 'a')).toHaveLength(3);
    expect(slots.exact).toBe(false);
    const m = firstBlock(s, 'matrix');
    expect(m.matrix.size).toBe(8);
    expect(m.fullMesh).toBe(true);
  });
  it('a single-GPU node has slots but no xGMI matrix (no peers), on its card and its detail section', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g1', { gpus: 1 })], pods: [makeGpuPod('a', { node: 'g1', gpus: 1 })] });
    const s = findSection(nodesView(ctx, opts), 'g1');
    expect(firstBlock(s, 'slots').slots).toHaveLength(1);
    expect(firstBlock(s, 'matrix')).toBeFalsy();
    const d = nodeDetailView(makeGpuNode('g1', { gpus: 1 }), ctx);
    expect(firstBlock(d, 'slots')).toBeTruthy();
    expect(firstBlock(d, 'matrix')).toBeFalsy();
    expect(renderPage(nodesView(ctx, opts))).not.toContain('xgmi-matrix');
  });
  it('the Node detail section shows its GPUs\' live telemetry from the node-scoped snapshot, and no table without one', () => {
    const E = SERIES.exporter;
    const r = {};
    r[E.power] = [0, 1].map((g) => ({ metric: { hostname: 'g0', gpu_id: String(g) }, value: [0, String(700 + g)] }));
    r[E.temp] = [0, 1].map((g) => ({ metric: { hostname: 'g0', gpu_id: String(g) }, value: [0, '66'] }));
    const metrics = joinExporterResults(r);
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [] });
    const d = nodeDetailView(makeGpuNode('g0'), ctx, { metrics: metrics });
    const t = firstBlock(d, 'table');
    expect(t.columns.slice(0, 2)).toEqual(['GPU', 'Power']);
    expect(t.rows.map((x) => [x[0], text(x[5])])).toEqual([['GPU 0', '66 °C'], ['GPU 1', '66 °C']]);
    expect(firstBlock(nodeDetailView(makeGpuNode('g0'), ctx), 'table')).toBeFalsy();
  });
  it('uses exporter pod labels for exact slots when metrics are given', () => {
    const E = SERIES.exporter;
    const r = {};
    r[E.power] = [{ metric: { hostname: 'g0', gpu_id: '5', pod: 'a', namespace: 'ml' }, value: [0, '700'] }];
    const metrics = joinExporterResults(r);
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0', gpus: 1 })] });
    const slots = firstBlock(findSection(nodesView(ctx, { now: NOW, metrics }), 'g0'), 'slots');
    expect(slots.exact).toBe(true);
    expect(slots.slots[5].pod).toBe('a');
    expect(slots.slots[0].pod).toBeNull();
  });
  it('marks not-ready nodes', () => {
    const t = firstTable(findSection(nodesView(makeContext({ nodes: [makeGpuNode('g', { ready: false })] }), opts), 'GPU Node Summary'));
    expect(t.rows[0][1]).toEqual({ t: 'status', status: 'error', text: 'Not Ready' });
  });
  it('shows partition mode on partitioned nodes', () => {
    const s = findSection(nodesView(makeContext({ nodes: [makeGpuNode('g', { partition: 'cpx/nps4' })] }), opts), 'g');
    expect(rowValue(s, 'Partition Mode')).toBe('MI355X (CPX/NPS4)');
  });
});

// ---------------------------------------------------------------------------
describe('podsView', () => {
  it('shows the loader on first load', () => {
    expect(loaders(podsView(makeContext({ loading: true, lastUpdated: null }), opts))).toEqual(['Loading GPU pod data...']);
  });
  it('shows "No GPU Pods Found"', () => {
    const vm = podsView(makeContext({ pods: [makePlainPod('x')] }), opts);
    expect(sectionTitles(vm)).toEqual(['No GPU Pods Found']);
    expect(vm.refresh.ariaLabel).toBe('Refresh pod data');
  });
  it('summarises phases and GPUs held', () => {
    const ctx = makeContext({
      pods: [makeGpuPod('a', { gpus: 8 }), makeGpuPod('b', { phase: 'Pending', gpus: 2 }), makeGpuPod('c', { phase: 'Failed', gpus: 4 })],
    });
    const s = findSection(podsView(ctx, opts), 'Summary');
    expect(rowValue(s, 'Total GPU Pods')).toBe('3');
    expect(rowValue(s, 'Running').status).toBe('success');
    expect(rowValue(s, 'GPUs Held')).toBe('10');
  });
  it('lists all GPU pods with phase status and restarts', () => {
    const ctx = makeContext({ pods: [makeGpuPod('a', { restarts: 2 }), makeGpuPod('b', { phase: 'Failed' })] });
    const t = firstTable(findSection(podsView(ctx, opts), 'All GPU Pods'));
    expect(t.columns).toEqual(['Name', 'Namespace', 'Node', 'Phase', 'GPU Resources', 'Restarts', 'Age']);
    expect(t.rows[0][3]).toEqual({ t: 'status', status: 'success', text: 'Running' });
    expect(t.rows[1][3].status).toBe('error');
    expect(t.rows[0][5].status).toBe('warning');
    expect(text(t.rows[0][4])).toBe('trainer: GPU: 1');
  });
  it('shows the pending attention table with waiting reasons', () => {
    const ctx = makeContext({ pods: [makeGpuPod('a'), makeGpuPod('b', { phase: 'Pending', waiting: 'ImagePullBackOff', gpus: 4 })] });
    const t = firstTable(findSection(podsView(ctx, opts), 'Attention: Pending GPU Pods'));
    expect(t.rows).toHaveLength(1);
    expect(t.rows[0][2]).toBe('GPU: 4');
    expect(t.rows[0][3]).toBe('ImagePullBackOff');
    expect(t.columns).toEqual(['Name', 'Namespace', 'GPU Resources', 'Waiting Reason', 'Message', 'Age']);
    expect(t.rows[0][4]).toBe('—'); // no message on this fixture
  });
  it('omits the pending table when nothing is pending', () => {
    expect(sectionTitles(podsView(makeContext({ pods: [makeGpuPod('a')] }), opts))).not.toContain('Attention: Pending GPU Pods');
  });
  it('gpuContainerLines shows req/lim when they differ and marks init containers', () => {
    const p = makeGpuPod('p', { gpus: 1, init: 2 });
    p.spec.containers[0].resources.limits['amd.com/gpu'] = '2';
    expect(text(gpuContainerLines(p))).toBe('warmup (init): GPU: 2\ntrainer: GPU: req=1 lim=2');
  });
  it('gpuContainerLines handles limits-only containers', () => {
    expect(text(gpuContainerLines(makeGpuPod('p', { limitsOnly: true, gpus: 2 })))).toBe('trainer: GPU: req=— lim=2');
  });
});

// ---------------------------------------------------------------------------
describe('temperature against the throttle threshold', () => {
  it('is plain text when cool, warning within 10 °C, error at the threshold', () => {
    expect(tempCell({ tempC: 60, tempSlowdownC: 100 })).toBe('60 °C');
    expect(tempCell({ tempC: 93, tempSlowdownC: 100 })).toEqual({ t: 'status', status: 'warning', text: '93 °C' });
    expect(tempCell({ tempC: 101, tempSlowdownC: 100 }).status).toBe('error');
    expect(tempCell({ tempC: null })).toBe('—');
  });
  it('falls back to the MI355X threshold without exporter data', () => {
    expect(MI355X.junctionSlowdownC).toBe(100);
    expect(tempCell({ tempC: 95, tempSlowdownC: null }).status).toBe('warning');
  });
});

describe('RAS error cell', () => {
  it('is OK when clean, a warning for corrected and an error for uncorrected errors', () => {
    expect(eccCell({ eccCorrectable: 0, eccUncorrectable: 0 })).toBe('OK');
    expect(eccCell({ eccCorrectable: 3, eccUncorrectable: 0 })).toEqual({ t: 'status', status: 'warning', text: '3 corrected' });
    expect(eccCell({ eccCorrectable: 3, eccUncorrectable: 1 })).toEqual({
      t: 'status', status: 'error', text: '1 uncorrected, 3 corrected' });
    expect(eccCell({ eccCorrectable: null, eccUncorrectable: null })).toBe('—');
  });
  it('adds an ECC column per GPU and a cluster RAS row on the Metrics page', () => {
    const E = SERIES.exporter;
    const r = {};
    r[E.power] = [0, 1].map((i) => ({ metric: { hostname: 'g0', gpu_id: String(i) }, value: [0, '900'] }));
    r[E.eccCorrect] = [0, 1].map((i) => ({ metric: { hostname: 'g0', gpu_id: String(i) }, value: [0, String(i * 2)] }));
    r[E.eccUncorrect] = [0, 1].map((i) => ({ metric: { hostname: 'g0', gpu_id: String(i) }, value: [0, '0'] }));
    const m = Object.assign(joinExporterResults(r), { source: 'amd-exporter', fetchedAt: NOW, prometheusPath: '/p' });
    const vm = metricsView(makeContext({ nodes: [makeGpuNode('g0')] }), { metrics: m, series: null, fetching: false }, {});
    const t = firstTable(findSection(vm, 'g0 — 2 × ' + MI355X.shortName));
    expect(t.columns).toContain('ECC');
    const col = t.columns.indexOf('ECC');
    expect(t.rows.map((row) => text(row[col]))).toEqual(['OK', '2 corrected']);
    expect(text(rowValue(findSection(vm, 'GPU Power Summary'), 'RAS Errors'))).toBe('2 corrected');
  });
});

describe('pod → GPU assignment (exporter pod labels)', () => {
  const pods = [makeGpuPod('train', { node: 'g0', gpus: 2 }), makeGpuPod('idle', { node: 'g0', gpus: 1 })];
  const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods });
  const gpu = (i, pod) => ({ nodeName: 'g0', gpu: String(i), pod, namespace: pod ? 'ml' : null, powerWatts: 1000 + i,
    gfxActivityPct: 90, vramUsedBytes: 64 * 1024 ** 3 });
  const metrics = { source: 'amd-exporter', gpus: [gpu(0, 'train'), gpu(1, 'train'), gpu(2, null)], xgmi: {}, links: {} };
  it('adds an Assigned GPUs column when the exporter labels pods', () => {
    const t = firstTable(findSection(podsView(ctx, { now: NOW, metrics }), 'All GPU Pods'));
    expect(t.columns).toContain('Assigned GPUs');
    const col = t.columns.indexOf('Assigned GPUs');
    const trainRow = t.rows.find((r) => r[0] === 'train');
    expect(trainRow[col]).toBe('g0: GPU 0, 1');
    expect(t.rows.find((r) => r[0] === 'idle')[col]).toBe('—');
    // GPU Power: the held GPUs' live power, summed (1000 W + 1001 W)
    const pw = t.columns.indexOf('GPU Power');
    expect(pw).toBe(col + 1);
    expect(trainRow[pw]).toBe('2001.0 W');
    expect(t.rows.find((r) => r[0] === 'idle')[pw]).toBe('—');
  });
  it('keeps the reference columns without exporter data', () => {
    const t = firstTable(findSection(podsView(ctx, { now: NOW }), 'All GPU Pods'));
    expect(t.columns).toEqual(['Name', 'Namespace', 'Node', 'Phase', 'GPU Resources', 'Restarts', 'Age']);
  });
  it('shows live telemetry of the held GPUs on the pod detail section', () => {
    const s = podDetailView(pods[0], { metrics });
    const v = rowValue(s, 'Assigned GPUs');
    expect(v.t).toBe('lines');
    expect(v.lines[0]).toEqual({ label: 'g0 GPU 0', text: '1000.0 W, 90% GFX, 64 GiB HBM' });
    expect(assignedLines([Object.assign({}, metrics.gpus[0], { tempC: 81.6 })]).lines[0].text).toBe('1000.0 W, 90% GFX, 64 GiB HBM, 82 °C');
    expect(rowValue(podDetailView(pods[1], { metrics }), 'Assigned GPUs')).toBeUndefined();
  });
  it('keeps assignment identity across snapshots with unchanged ownership', () => {
    const a = podGpuAssignments(metrics);
    const b = podGpuAssignments(Object.assign({}, metrics, { gpus: metrics.gpus.slice() }));
    expect(b).toBe(a);
  });
});

describe('metricsView', () => {
  const E = SERIES.exporter;
  function metrics(nodes, gpusPer) {
    const r = {};
    r[E.power] = [];
    r[E.vramUsed] = [];
    r[E.vramTotal] = [];
    nodes.forEach((n) => {
      for (let g = 0; g < gpusPer; g++) {
        const m = { hostname: n, gpu_id: String(g) };
        r[E.power].push({ metric: m, value: [0, String(1300)] });
        r[E.vramUsed].push({ metric: m, value: [0, String(100 * 1024)] });
        r[E.vramTotal].push({ metric: m, value: [0, String(274658)] });
      }
    });
    const j = joinExporterResults(r);
    return { source: 'amd-exporter', gpus: j.gpus, xgmi: j.xgmi, fetchedAt: new Date(NOW).toISOString(), prometheusPath: '/p' };
  }
  const ctx = makeContext({ nodes: [makeGpuNode('n0')] });

  it('always shows the availability box and header', () => {
    const vm = metricsView(ctx, { metrics: null, fetchError: null, fetching: false }, opts);
    expect(vm.title).toBe('AMD GPU — Metrics');
    expect(sectionTitles(vm)).toEqual(['Metric Availability']);
    expect(vm.refresh.ariaLabel).toBe('Refresh metrics');
  });
  it('availability says what the answering source reports: node-exporter has no HBM activity, xGMI or pod owner', () => {
    const g = { nodeName: 'n0', gpu: '0', powerWatts: 900, powerCapWatts: 1400, vramUsedBytes: 1, vramTotalBytes: 2,
      gfxActivityPct: 50, memActivityPct: null, tempC: 70, tempSlowdownC: 100, pod: null };
    const cell = (m, name) => {
      const sec = findSection(metricsView(ctx, { metrics: m, fetchError: null, fetching: false }, opts), 'Metric Availability');
      return sec.blocks[0].rows.filter((r) => r.name === name)[0].value;
    };
    const ne = { source: 'node-exporter', gpus: [g], xgmi: {}, fetchedAt: new Date(NOW).toISOString(), prometheusPath: '/p' };
    expect(cell(ne, 'Junction temperature').status).toBe('success');
    expect(cell(ne, 'Junction temperature').text).toContain('"junction"');
    expect(cell(ne, 'HBM controller activity (%)')).toEqual({ t: 'status', status: 'warning',
      text: 'Not available from node-exporter — the AMD Device Metrics Exporter reports gpu_umc_activity' });
    expect(cell(ne, 'xGMI link throughput').status).toBe('warning');
    const ex = { source: 'amd-exporter', gpus: [Object.assign({}, g, { memActivityPct: 30 })], xgmi: { n0: { 0: [50e9] } },
      fetchedAt: new Date(NOW).toISOString(), prometheusPath: '/p' };
    expect(cell(ex, 'HBM controller activity (%)').text).toBe('Reporting — gpu_umc_activity');
    expect(cell(ex, 'xGMI link throughput').status).toBe('success');
    expect(cell(ex, 'Per-GPU pod owner').text).toBe('Not reported on this page — pod / namespace labels (exporter pod association)');
    // The Metrics page's own snapshot ('gauges') asks for no link throughput: it points to GPU Nodes instead.
    expect(text(cell(Object.assign({}, ex, { view: 'gauges', xgmi: {} }), 'xGMI link throughput'))).toContain('On GPU Nodes');
    // Before an answer: what each source offers.
    expect(text(cell(null, 'Power (W)'))).toContain('Available — gpu_power_usage');
  });
  it('shows the context loader while the store loads', () => {
    const vm = metricsView(makeContext({ loading: true, lastUpdated: null }), { metrics: null, fetchError: null, fetching: false }, opts);
    expect(loaders(vm)).toEqual(['Loading AMD GPU data...']);
    expect(vm.refresh.disabled).toBe(true);
  });
  it('shows the query loader while fetching the first time', () => {
    const vm = metricsView(ctx, { metrics: null, fetchError: null, fetching: true }, opts);
    expect(loaders(vm)).toEqual(['Querying Prometheus for GPU metrics...']);
    expect(vm.refresh.label).toBe('Refreshing…');
  });
  it('shows "Prometheus Unreachable" with the checked services', () => {
    const vm = metricsView(ctx, { metrics: null, fetchError: 'Could not reach Prometheus', fetching: false }, opts);
    const s = findSection(vm, 'Prometheus Unreachable');
    expect(rowValue(s, 'Error').status).toBe('error');
    expect(rowValue(s, 'Checked services')).toContain('kube-prometheus-stack-prometheus:9090');
  });
  it('shows "No AMD GPU Metrics" with the GPU node list', () => {
    const vm = metricsView(ctx, { metrics: { source: null, gpus: [], xgmi: {}, fetchedAt: new Date(NOW).toISOString() }, fetchError: null, fetching: false }, opts);
    expect(rowValue(findSection(vm, 'No AMD GPU Metrics in Prometheus'), 'GPU Nodes')).toBe('n0');
  });
  it('summarises power and HBM', () => {
    const vm = metricsView(ctx, { metrics: metrics(['n0'], 8), fetchError: null, fetching: false }, opts);
    const s = findSection(vm, 'GPU Power Summary');
    expect(rowValue(s, 'GPUs Monitored')).toBe('8');
    expect(rowValue(s, 'Total Power').text).toBe('10400.0 W / 11200.0 W (93%)');
    expect(rowValue(s, 'Total Power').color).toBe('#d32f2f');
    expect(rowValue(s, 'Source')).toBe('AMD Device Metrics Exporter');
  });
  it('shows Last Fetched in browser-local time and the PromQL it ran (reference MetricsPage.tsx:336-343)', () => {
    const m = Object.assign(metrics(['n0'], 1), { query: 'max by (hostname, gpu_id) ({__name__=~"gpu_power_usage"})' });
    const s = findSection(metricsView(ctx, { metrics: m, fetchError: null, fetching: false }, opts), 'GPU Power Summary');
    expect(rowValue(s, 'Last Fetched')).toBe(new Date(NOW).toLocaleTimeString());
    expect(rowValue(s, 'Query')).toBe(m.query);
    const stale = findSection(metricsView(ctx, { metrics: Object.assign({}, m, { stale: true }), fetchError: null, fetching: false }, opts), 'GPU Power Summary');
    expect(rowValue(stale, 'Last Fetched').text).toBe(new Date(NOW).toLocaleTimeString() + ' (stale: the latest refresh failed)');
  });
  it('renders one card per node with a per-GPU table', () => {
    const vm = metricsView(ctx, { metrics: metrics(['n0', 'n1'], 8), fetchError: null, fetching: false }, opts);
    const s = findSection(vm, 'n1 — 8 × MI355X');
    expect(firstTable(s).rows).toHaveLength(8);
    expect(firstTable(s).rows[0][0]).toBe('GPU 0');
  });
  it('adds the time-series section when range data exists', () => {
    const vm = metricsView(ctx, { metrics: metrics(['n0'], 1), fetchError: null, fetching: false, series: { power: { n0: [[1, 2]] }, vram: {} } }, opts);
    expect(sectionTitles(vm)).toContain('Power & HBM (last 30 min)');
  });
  it('shows cluster peak and average power over the window (per-step sums over nodes)', () => {
    const series = { power: { n0: [[30, 100], [60, 300], [90, 200]], n1: [[30, 50], [60, 50], [90, 400]] }, vram: {} };
    const vm = metricsView(ctx, { metrics: metrics(['n0', 'n1'], 1), fetchError: null, fetching: false, series }, opts);
    const s = findSection(vm, 'Power & HBM (last 30 min)');
    expect(rowValue(s, 'Peak Power (30 min)').text).toContain('600.0 W');
    expect(rowValue(s, 'Average Power (30 min)').text).toContain('366.7 W');
    // no samples in the window: no stat rows, the series block alone
    const empty = findSection(metricsView(ctx, { metrics: metrics(['n0'], 1), fetchError: null, fetching: false, series: { power: {}, vram: {} } }, opts), 'Power & HBM (last 30 min)');
    expect(rowValue(empty, 'Peak Power (30 min)')).toBeUndefined();
  });
  it('series block carries the per-node mean; summary counts the nodes reporting', () => {
    const series = { power: { n0: [[30, 100], [60, 300]], n1: [] }, vram: {} };
    const vm = metricsView(ctx, { metrics: metrics(['n0'], 1), fetchError: null, fetching: false, series }, opts);
    const blk = findSection(vm, 'Power & HBM (last 30 min)').blocks.filter((b) => b.t === 'series')[0];
    // the cluster line (summed over the nodes) first, then the nodes of the page
    expect(blk.avgPower).toEqual({ 'All GPU nodes': 200, n0: 200 });
    expect(Object.keys(blk.power)).toEqual(['All GPU nodes', 'n0']);
    expect(rowValue(findSection(vm, 'GPU Power Summary'), 'Nodes Reporting')).toBe('1 / 1 GPU nodes');
    const two = makeContext({ nodes: [makeGpuNode('n0'), makeGpuNode('n9')] });
    const vm2 = metricsView(two, { metrics: metrics(['n0'], 1), fetchError: null, fetching: false }, opts);
    const rep = rowValue(findSection(vm2, 'GPU Power Summary'), 'Nodes Reporting');
    expect(rep.status).toBe('warning');
    expect(rep.text).toBe('1 / 2 GPU nodes (1 without telemetry)');
  });
  it('clusterPowerStats ignores non-numbers and reports the peak instant', () => {
    expect(clusterPowerStats({})).toBeNull();
    expect(clusterPowerStats({ a: [[10, 5], [20, NaN]], b: [[10, 1], [20, 7]] })).toEqual({ peakWatts: 7, peakAt: 20, avgWatts: 6.5, steps: 2 });
  });
  it('titles the time-series section with the configured window', () => {
    const series = { rangeSec: 6 * 3600, power: { n0: [[1, 2]] }, vram: {} };
    const vm = metricsView(ctx, { metrics: metrics(['n0'], 1), fetchError: null, fetching: false, series }, opts);
    expect(sectionTitles(vm)).toContain('Power & HBM (last 6 h)');
    expect(formatWindow(90)).toBe('90 s');
    expect(formatWindow(900)).toBe('15 min');
  });
  it('"Last Fetched" reads as toLocaleTimeString() does, through one cached formatter', () => {
    const t0 = Date.parse('2026-10-16T13:04:05Z');
    for (let i = 0; i < 48; i++) {
      const t = t0 + i * 3599 * 1000;
      expect(localTimeText(t)).toBe(new Date(t).toLocaleTimeString());
      expect(localTimeText(new Date(t).toISOString())).toBe(new Date(t).toLocaleTimeString());
    }
  });
  it('powerBar without a cap shows watts only', () => {
    expect(powerBar(512.25, null).text).toBe('512.3 W');
    expect(powerBar(512.25, null).pct).toBeNull();
  });
  it('hbmBar formats used/total', () => {
    expect(hbmBar(144 * 1024 ** 3, 288 * 1024 ** 3).text).toBe('144 GiB / 288 GiB (50%)');
    expect(hbmBar(null, 288e9)).toBe('—');
  });
});

// ---------------------------------------------------------------------------
describe('allocationBar', () => {
  it('returns a dash without allocatable GPUs', () => {
    expect(allocationBar(1, 0)).toBe('—');
  });
  it('caps at 100% and colours by threshold', () => {
    expect(allocationBar(10, 8).pct).toBe(100);
    expect(allocationBar(10, 8).color).toBe('#d32f2f');
    expect(allocationBar(1, 8).color).toBe('#ed1c24');
  });
});

// ---------------------------------------------------------------------------
describe('html rendering', () => {
  it('renders sections, tables and status labels semantically', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0' })] });
    const html = renderPage(nodesView(ctx, opts));
    expect(html).toContain('<h1>AMD GPU — Nodes</h1>');
    expect(html).toContain('<button aria-label="Refresh node data">Refresh</button>');
    expect(html).toContain('<h2>GPU Node Summary</h2>');
    expect(html).toContain('<span data-status="success">Ready</span>');
    expect(html).toContain('data-testid="xgmi-matrix" data-full-mesh="true"');
  });
  it('escapes user-controlled strings', () => {
    const n = makeGpuNode('<script>');
    const html = renderPage(nodesView(makeContext({ nodes: [n] }), opts));
    expect(html).not.toContain('<script>');
    expect(html).toContain('&lt;script&gt;');
  });
  it('textContent strips markup', () => {
    const html = renderPage(overviewView(makeContext({ loading: true, lastUpdated: null }), opts));
    expect(textContent(html)).toBe('Loading AMD GPU data...');
  });
  it('countRows counts table rows and GPU cells', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0'), makeGpuNode('g1')], pods: [makeGpuPod('a', { node: 'g0' })] });
    const c = countRows(nodesView(ctx, opts));
    expect(c.tableRows).toBe(2);
    expect(c.gpuCells).toBe(2 * (8 + 64));
  });
});
