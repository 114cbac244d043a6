/**
 * node-exporter as the telemetry source (the reference's only one,
 * src/api/metrics.ts:101-116): node-exporter's GPU series carry `instance`,
 * not the node name, so the paged views select a page through
 * node_uname_info, take the cluster totals from server-side aggregates and
 * let Prometheus rank nodes by power — O(page) as on the exporter
 * (promql.js nodeExporterScopedQuery / nodeExporterSummaryQuery /
 * rankedHwQuery, scopedSnapshots.js hwScoped / hwRanked).
 */
import { createMetricsSource } from '../../src/api/metrics.js';
import { SERIES } from '../../src/api/series.js';
import { summarizeMetrics } from '../../src/api/telemetry.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { metricsView } from '../../src/view/pages/metricsPage.js';
import { sectionTitles } from '../../src/view/ir.js';
import { makeContext, makeGpuNode, makeGpuPod } from './fixtures.js';
import { exporterData, prom, vec } from './promFake.js';

const names = (n) => Array.from({ length: n }, (_, i) => 'mi355x-' + String(i).padStart(3, '0'));
const ctxOf = (n) => makeContext({ nodes: names(n).map((x) => makeGpuNode(x)), pods: [makeGpuPod('train-0', { node: 'mi355x-000' })] });
const cards = (vm) => sectionTitles(vm).filter((t) => /^mi355x-/.test(t));
const source = (fake) => createMetricsSource({ request: fake });
const rank = (page, filter) => ({ by: 'power', page: page, per: 8, filter: filter || '' });

beforeEach(() => {
  clearViewMemo();
});

describe('node-exporter source: paged, totalled and ranked by Prometheus', () => {
  it('a node-exporter Prometheus is ranked too: each node\'s amdgpu chips summed through node_uname_info', async () => {
    const ne = { node_uname_info: [] };
    ne[SERIES.nodeExporter.chips] = [];
    ne.node_hwmon_power_input_watt = [];
    const watts = [300, 900, 600];
    ['mi355x-000', 'mi355x-001', 'mi355x-002'].forEach((n, k) => {
      const inst = 'i' + k;
      ne.node_uname_info.push({ metric: { __name__: 'node_uname_info', instance: inst, nodename: n }, value: [0, '1'] });
      ne[SERIES.nodeExporter.chips].push({ metric: { __name__: 'node_hwmon_chip_names', chip_name: 'amdgpu', instance: inst, chip: '0000:05:00_0' }, value: [0, '1'] });
      ne.node_hwmon_power_input_watt.push({ metric: { __name__: 'node_hwmon_power_input_watt', instance: inst, chip: '0000:05:00_0' }, value: [0, String(watts[k])] });
    });
    const request = prom({ data: {}, ne: ne });
    const s = createMetricsSource({ request: request });
    // the first ranked fetch finds no exporter: the cluster-wide answer names node-exporter, which is then ranked
    const m = await s.fetchGpuMetrics('gauges', { rank: Object.assign(rank(0), { per: 2 }), summary: true });
    expect(m.source).toBe('node-exporter');
    expect(m.scope).toEqual(['mi355x-001', 'mi355x-002']);
    expect(m.rank.count).toBe(3);
    expect(m.rank.watts).toEqual({ 'mi355x-001': 900, 'mi355x-002': 600 });
    expect(m.gpus.map((g) => g.nodeName)).toEqual(['mi355x-001', 'mi355x-002']);
    expect(m.totals.powerWatts).toBe(1800);
    const n = request.mock.calls.length;
    const p2 = await s.fetchGpuMetrics('gauges', { rank: Object.assign(rank(1), { per: 2 }), summary: true });
    expect(request.mock.calls.length).toBe(n + 1); // one request per ranked page from then on
    expect(p2.scope).toEqual(['mi355x-000']);
    const vm = metricsView(ctxOf(3), { metrics: m, series: null, fetchError: null, fetching: false }, { pager: { sort: 'power' } });
    expect(sectionTitles(vm)).not.toContain('No AMD GPU Metrics in Prometheus');
    expect(cards(vm)).toEqual(['mi355x-001 — 1 × MI355X', 'mi355x-002 — 1 × MI355X']);
  });
  it('falls back to the cluster-wide snapshot cut to the scope for a node-exporter source', async () => {
    const ne = { node_uname_info: [{ metric: { __name__: 'node_uname_info', instance: 'i0', nodename: 'mi355x-000' }, value: [0, '1'] }] };
    ne[SERIES.nodeExporter.chips] = [{ metric: { __name__: 'node_hwmon_chip_names', chip_name: 'amdgpu', instance: 'i0', chip: '0000:05:00_0' }, value: [0, '1'] }];
    const fake = prom({ data: {}, ne: ne });
    const s = source(fake);
    const m = await s.fetchGpuMetrics('gauges', { scope: ['mi355x-000'], summary: true });
    expect(m.source).toBe('node-exporter');
    expect(m.gpus.map((g) => g.nodeName)).toEqual(['mi355x-000']);
    expect(m.totals.gpus).toBe(1);
  });
  it('a Node detail opened first (source unknown) reads its node in ONE request on node-exporter, and on a Prometheus with no GPU series', async () => {
    const ne = { node_uname_info: [] };
    ne[SERIES.nodeExporter.chips] = [];
    ['mi355x-000', 'mi355x-001'].forEach((n, k) => {
      ne.node_uname_info.push({ metric: { __name__: 'node_uname_info', instance: 'i' + k, nodename: n }, value: [0, '1'] });
      ne[SERIES.nodeExporter.chips].push({ metric: { __name__: 'node_hwmon_chip_names', chip_name: 'amdgpu', instance: 'i' + k, chip: '0000:05:00_0' }, value: [0, '1'] });
    });
    const fake = prom({ data: {}, ne: ne });
    const s = source(fake);
    const m = await s.fetchNodeMetrics('mi355x-001');
    expect(m.source).toBe('node-exporter');
    expect(m.gpus.map((g) => g.nodeName)).toEqual(['mi355x-001']);
    const queries = fake.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('/api/v1/query') >= 0);
    expect(queries).toHaveLength(1);
    expect(s.source()).toBe('node-exporter');

    const none = prom({ data: {} });
    const s2 = source(none);
    const m2 = await s2.fetchNodeMetrics('mi355x-000');
    expect(m2).not.toBeNull();
    expect(m2.gpus).toEqual([]);
    expect(none.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('/api/v1/query') >= 0)).toHaveLength(1);
  });

  it('a cold Node detail on an exporter cluster never asks node-exporter for its history (the node query decides first)', async () => {
    const fake = prom({ data: exporterData(['mi355x-000']) });
    const s = source(fake);
    const r = await Promise.all([s.fetchNodeMetrics('mi355x-000'), s.fetchNodeSeries('mi355x-000', 1800, 30)]);
    expect(r[0].source).toBe('amd-exporter');
    const ranges = fake.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('/query_range') >= 0);
    expect(ranges).toHaveLength(1);
    expect(ranges[0]).not.toContain('node_hwmon');
  });

  it('junction temperature and its throttle limit come from the amdgpu hwmon sensor labelled "junction" (not mem, not the CPU)', async () => {
    const i = '10.0.0.1:9100';
    const chip = '0000:05:00_0';
    const cpu = 'platform_coretemp_0';
    const t = (name, c, sensor, v) => vec({ __name__: name, instance: i, chip: c, sensor: sensor }, v);
    const lab = (c, sensor, label) => vec({ __name__: 'node_hwmon_sensor_label', instance: i, chip: c, sensor: sensor, label: label }, 1);
    const ne = {
      node_uname_info: [vec({ __name__: 'node_uname_info', instance: i, nodename: 'mi355x-000' }, 1)],
      chips: [vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: chip, chip_name: 'amdgpu' }, 1),
        vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: cpu, chip_name: 'coretemp' }, 1)],
      power: [vec({ __name__: 'node_hwmon_power_input_watt', instance: i, chip: chip, sensor: 'power1' }, 900)],
      temps: [t('node_hwmon_temp_celsius', chip, 'temp2', 71), t('node_hwmon_temp_crit_celsius', chip, 'temp2', 100),
        t('node_hwmon_temp_celsius', chip, 'temp3', 64), t('node_hwmon_temp_crit_celsius', chip, 'temp3', 95),
        t('node_hwmon_temp_celsius', cpu, 'temp1', 47)],
      labels: [lab(chip, 'temp2', 'junction'), lab(chip, 'temp3', 'mem'), lab(cpu, 'temp1', 'Package id 0')],
    };
    // Cluster-wide, paged and single-node reads all carry it.
    const m = await source(prom({ data: {}, ne: ne })).fetchGpuMetrics();
    expect(m.source).toBe('node-exporter');
    expect(m.gpus.map((g) => [g.nodeName, g.tempC, g.tempSlowdownC, g.powerWatts])).toEqual([['mi355x-000', 71, 100, 900]]);
    const p = await source(prom({ data: {}, ne: ne })).fetchGpuMetrics('gauges', { scope: ['mi355x-000'], summary: true });
    expect(p.gpus.map((g) => g.tempC)).toEqual([71]);
    const d = await source(prom({ data: {}, ne: ne })).fetchNodeMetrics('mi355x-000');
    expect(d.gpus.map((g) => [g.tempC, g.tempSlowdownC])).toEqual([[71, 100]]);
  });

  it('node-exporter source, small-cluster fetch before the node list: every GPU of a small cluster, the page of a larger one', async () => {
    function neData(nodes) {
      const ne = { node_uname_info: [] };
      ne[SERIES.nodeExporter.chips] = [];
      nodes.forEach((n, k) => {
        ne.node_uname_info.push({ metric: { __name__: 'node_uname_info', instance: 'i' + k, nodename: n }, value: [0, '1'] });
        for (let c = 0; c < 8; c++) {
          const chip = '0000:' + (5 + c * 16).toString(16).padStart(2, '0') + ':00_0';
          ne[SERIES.nodeExporter.chips].push({ metric: { __name__: 'node_hwmon_chip_names', chip_name: 'amdgpu', instance: 'i' + k, chip: chip }, value: [0, '1'] });
        }
      });
      return ne;
    }
    // 2 nodes (16 chips): the first answer (no names yet) holds the whole cluster, so the names arriving need no refetch.
    let request = prom({ data: {}, ne: neData(names(2)) });
    let s = createMetricsSource({ request });
    let m = await s.fetchGpuMetrics('gauges', { scope: [], summary: true, small: true });
    expect(m.source).toBe('node-exporter');
    expect(Array.from(new Set(m.gpus.map((g) => g.nodeName)))).toEqual(names(2));
    expect(m.small).toEqual({ count: 16, limit: 64, exceeded: false });
    expect([m.totals.gpus, m.totals.nodes]).toEqual([16, 2]);
    expect(request.mock.calls).toHaveLength(1);
    // 12 nodes (96 chips): more than a page — only the scope's, flagged so the caller's key follows the names.
    request = prom({ data: {}, ne: neData(names(12)) });
    s = createMetricsSource({ request });
    m = await s.fetchGpuMetrics('gauges', { scope: [], summary: true, small: true });
    expect(m.gpus).toHaveLength(0);
    expect(m.small.exceeded).toBe(true);
    expect([m.totals.gpus, m.totals.nodes]).toEqual([96, 12]);
    m = await s.fetchGpuMetrics('gauges', { scope: names(8), summary: true, small: true });
    expect(Array.from(new Set(m.gpus.map((g) => g.nodeName)))).toEqual(names(8));
    expect(m.gpus).toHaveLength(64);
    expect(m.totals.gpus).toBe(96);
    // the probe (with the totals), then the page through node_uname_info
    const qs = request.mock.calls.map((c) => decodeURIComponent(c[0]));
    expect(qs).toHaveLength(2);
    expect(qs[1]).toContain('and on(instance) node_uname_info{nodename=~"mi355x-000|');
  });
  it('node-exporter: the page\'s totals from server-side aggregates equal the cluster-wide join\'s', async () => {
    const ne = { node_uname_info: [] };
    ['node_hwmon_chip_names', 'node_hwmon_power_input_watt', 'node_hwmon_power_average_watt', 'node_hwmon_power_cap_watt',
      'node_drm_gpu_busy_percent', 'node_drm_memory_vram_used_bytes', 'node_drm_memory_vram_size_bytes'].forEach((n) => (ne[n] = []));
    names(10).forEach((n, k) => {
      const inst = '10.0.1.' + k + ':9100';
      ne.node_uname_info.push(vec({ __name__: 'node_uname_info', instance: inst, nodename: n }, 1));
      ne.node_hwmon_chip_names.push(vec({ __name__: 'node_hwmon_chip_names', instance: inst, chip: 'platform_coretemp_0', chip_name: 'coretemp' }, 1));
      for (let c = 0; c < 8; c++) {
        const chip = '0000:' + String(10 + c) + ':00_0';
        ne.node_hwmon_chip_names.push(vec({ __name__: 'node_hwmon_chip_names', instance: inst, chip: chip, chip_name: 'amdgpu' }, 1));
        ne.node_hwmon_power_input_watt.push(vec({ __name__: 'node_hwmon_power_input_watt', instance: inst, chip: chip }, 500 + k + c));
        // some chips also report an average: it wins
        if (c % 3 === 0) ne.node_hwmon_power_average_watt.push(vec({ __name__: 'node_hwmon_power_average_watt', instance: inst, chip: chip }, 700 + c));
        if (k % 2 === 0) ne.node_hwmon_power_cap_watt.push(vec({ __name__: 'node_hwmon_power_cap_watt', instance: inst, chip: chip }, 1400));
        ne.node_drm_gpu_busy_percent.push(vec({ __name__: 'node_drm_gpu_busy_percent', instance: inst, card: 'card' + c }, 10 * c));
        ne.node_drm_memory_vram_used_bytes.push(vec({ __name__: 'node_drm_memory_vram_used_bytes', instance: inst, card: 'card' + c }, 1e9 * (c + 1)));
        ne.node_drm_memory_vram_size_bytes.push(vec({ __name__: 'node_drm_memory_vram_size_bytes', instance: inst, card: 'card' + c }, 288e9));
      }
    });
    const wide = await createMetricsSource({ request: prom({ data: {}, ne: ne }) }).fetchGpuMetrics();
    const expected = Object.assign(summarizeMetrics(wide), { nodes: 10 });
    const paged = await createMetricsSource({ request: prom({ data: {}, ne: ne }) })
      .fetchGpuMetrics('gauges', { scope: names(10).slice(0, 8), summary: true });
    expect(paged.source).toBe('node-exporter');
    expect(Array.from(new Set(paged.gpus.map((g) => g.nodeName)))).toEqual(names(8));
    Object.keys(expected).forEach((k) => expect([k, paged.totals[k]]).toEqual([k, expected[k]]));
  });
});
