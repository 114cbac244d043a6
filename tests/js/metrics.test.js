/**
 * Metrics-client specs. The reference has NO direct tests for
 * src/api/metrics.ts (SURVEY.md §4 gaps); these cover discovery, the
 * exporter and node-exporter joins, the per-(node, gpu) key, caching and
 * range queries.
 */
import { createMetricsSource } from '../../src/api/metrics.js';
import { exporterNodeQuery, exporterQuery, mergedQuery, NODE_GAUGE_LABELS } from '../../src/api/promql.js';
import {
  EXPORTER_JOIN_LABELS,
  EXPORTER_LEAN_LABELS,
  METRIC_VIEWS,
  PROMETHEUS_SERVICES,
  SERIES,
  STALE_FAILURES,
} from '../../src/api/series.js';
import { applyStatics, keyedByHostname, shareGpus, shareMap, splitByName, staticsOf } from '../../src/api/telemetry.js';

import fs from 'fs';
import { BASE0, BASE1, exporterData, ok, prom, vec } from './promFake.js';

describe('discovery', () => {
  it('probes all candidate services in parallel', async () => {
    const request = prom();
    const src = createMetricsSource({ request });
    await src.discover();
    const probes = request.mock.calls.filter((c) => c[0].indexOf('query=1') >= 0);
    expect(probes).toHaveLength(PROMETHEUS_SERVICES.length);
  });
  it('prefers the highest-priority reachable service', async () => {
    const src = createMetricsSource({ request: prom({ up: [BASE1, BASE0] }) });
    expect(await src.discover()).toBe(BASE0);
  });
  it('falls back to a lower-priority service', async () => {
    const src = createMetricsSource({ request: prom({ up: [BASE1] }) });
    expect(await src.discover()).toBe(BASE1);
  });
  it('returns null when nothing answers', async () => {
    const src = createMetricsSource({ request: prom({ up: [] }) });
    expect(await src.discover()).toBeNull();
  });
  it('caches the discovered path', async () => {
    const request = prom();
    const src = createMetricsSource({ request });
    await src.discover();
    const n = request.mock.calls.length;
    await src.discover();
    expect(request.mock.calls.length).toBe(n);
  });
  it('re-discovers after the TTL', async () => {
    let now = 0;
    const request = prom();
    const src = createMetricsSource({
      request, discoveryTtlMs: 1000,
      clock: { setTimeout, clearTimeout, now: () => now },
    });
    await src.discover();
    const n = request.mock.calls.length;
    now = 5000;
    await src.discover();
    expect(request.mock.calls.length).toBe(n + PROMETHEUS_SERVICES.length);
  });
  it('times out a hanging probe', async () => {
    vi.useFakeTimers();
    const request = vi.fn(() => new Promise(() => {}));
    const src = createMetricsSource({ request, timeoutMs: 2000 });
    const p = src.discover();
    await vi.advanceTimersByTimeAsync(2000);
    expect(await p).toBeNull();
    vi.useRealTimers();
  });
});

describe('fetchGpuMetrics', () => {
  it('returns null when Prometheus is unreachable', async () => {
    const src = createMetricsSource({ request: prom({ up: [] }) });
    expect(await src.fetchGpuMetrics()).toBeNull();
  });
  it('joins exporter series per (node, gpu)', async () => {
    const src = createMetricsSource({ request: prom({ data: exporterData(['n0', 'n1']) }) });
    const m = await src.fetchGpuMetrics();
    expect(m.source).toBe('amd-exporter');
    expect(m.gpus).toHaveLength(16);
    const g = m.gpus.find((x) => x.nodeName === 'n1' && x.gpu === '3');
    expect(g.powerWatts).toBe(703);
    expect(g.gfxActivityPct).toBe(50);
    expect(g.vramUsedBytes).toBe(4 * 1024 * 1024 * 1024);
  });
  it('does not collide identical GPU ids across nodes (reference quirk Q1)', async () => {
    const d = exporterData(['a', 'b']);
    d[SERIES.exporter.power].forEach((r) => {
      if (r.metric.hostname === 'b') r.value[1] = '111';
    });
    const src = createMetricsSource({ request: prom({ data: d }) });
    const m = await src.fetchGpuMetrics();
    expect(m.gpus.find((x) => x.nodeName === 'a' && x.gpu === '5').powerWatts).toBe(705);
    expect(m.gpus.find((x) => x.nodeName === 'b' && x.gpu === '5').powerWatts).toBe(111);
  });
  it('records the PromQL it sent with the snapshot (Metrics page "Query" row)', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    const m = await src.fetchGpuMetrics();
    const sent = request.mock.calls.map((c) => c[0]).filter((u) => u.indexOf('/api/v1/query?query=') >= 0 && !/query=1$/.test(u));
    expect(sent.map((u) => decodeURIComponent(u.split('query=')[1]))).toContain(m.query);
    expect(m.query).toContain('gpu_power_usage');
  });
  it('captures pod ownership labels', async () => {
    const src = createMetricsSource({ request: prom() });
    const m = await src.fetchGpuMetrics();
    expect(m.gpus[0].pod).toBe('train-0');
    expect(m.gpus[0].namespace).toBe('ml');
    expect(m.gpus[4].pod).toBeNull();
  });
  it('keeps xGMI neighbour series per neighbour: no series says which peer neighbour k is', async () => {
    const src = createMetricsSource({ request: prom() });
    const m = await src.fetchGpuMetrics();
    expect(m.xgmi.n0['0>0']).toBe(50);
    expect(m.xgmi.n0['3>0']).toBe(50);
    expect(m.xgmi.n0['0-1']).toBeUndefined();
  });
  it('places a neighbour row on the peer its own peer_gpu_id label names', async () => {
    const d = exporterData(['n0']);
    d.__xgmi = [vec({ __name__: 'xgmi_neighbor_2_tx_throughput', hostname: 'n0', gpu_id: '5', peer_gpu_id: '1' }, 30e9)];
    const m = await createMetricsSource({ request: prom({ data: d }) }).fetchGpuMetrics();
    expect(m.xgmi.n0).toEqual({ '5-1': 30 });
  });
  it('reads the neighbour order of the native exporter\'s link series', async () => {
    const d = exporterData(['n0']);
    d.gpu_xgmi_link_hops = [vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n0', gpu_id: '0', peer_gpu_id: '6', neighbor: '0' }, 1),
      vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n0', gpu_id: '0', peer_gpu_id: '1', neighbor: 'x' }, 1)];
    const m = await createMetricsSource({ request: prom({ data: d }) }).fetchGpuMetrics();
    expect(m.links.n0).toEqual({ '0-6': { type: 'XGMI', hops: 1, neighbor: 0 }, '0-1': { type: 'XGMI', hops: 1 } });
  });
  it('reads measured xGMI link hops from the native exporter', async () => {
    const d = exporterData(['n0']);
    d.gpu_xgmi_link_hops = [
      vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n0', gpu_id: '0', peer_gpu_id: '1' }, 1),
      vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n0', gpu_id: '1', peer_gpu_id: '0' }, 1),
    ];
    const src = createMetricsSource({ request: prom({ data: d }) });
    const m = await src.fetchGpuMetrics();
    expect(m.links.n0).toEqual({ '0-1': { type: 'XGMI', hops: 1 }, '1-0': { type: 'XGMI', hops: 1 } });
  });
  it('serves the last snapshot marked stale through transient failures, then reports unreachable', async () => {
    let up = true;
    const ok = prom();
    const request = vi.fn((path) => (up ? ok(path) : Promise.reject(Object.assign(new Error('503'), { status: 503 }))));
    const src = createMetricsSource({ request });
    const a = await src.fetchGpuMetrics();
    up = false;
    const b = await src.fetchGpuMetrics();
    expect(b.stale).toBe(true);
    expect(b.gpus).toBe(a.gpus);
    const c = await src.fetchGpuMetrics();
    expect(c.stale).toBe(true);
    expect(await src.fetchGpuMetrics()).toBeNull(); // STALE_FAILURES in a row
    up = true;
    const d = await src.fetchGpuMetrics();
    expect(d.stale).toBeUndefined();
    expect(d.gpus.length).toBe(a.gpus.length);
  });
  it('paged, node and owner fetches re-discover a Prometheus that moved, once they report it unreachable', async () => {
    const fetches = {
      paged: (src) => src.fetchGpuMetrics('gauges', { scope: ['n0'], summary: true }),
      node: (src) => src.fetchNodeMetrics('n0'),
      owners: (src) => src.fetchGpuOwners({ pods: ['ml/train-0'] }),
    };
    for (const name of Object.keys(fetches)) {
      const fetch = fetches[name];
      let at = BASE0;
      const inner = prom({ up: [BASE0, BASE1], data: exporterData(['n0']) });
      const request = vi.fn((path) => (path.indexOf(at) === 0 ? inner(path) : Promise.reject(Object.assign(new Error('503'), { status: 503 }))));
      const src = createMetricsSource({ request });
      expect((await fetch(src)).prometheusPath).toBe(BASE0);
      at = BASE1; // the service moved
      let r;
      for (let i = 0; i < STALE_FAILURES; i++) r = await fetch(src);
      expect(r).toBeNull();
      r = await fetch(src);
      expect(r === null ? name + ': still unreachable' : r.prometheusPath).toBe(BASE1);
    }
  });
  it('reuses unchanged GPU objects and maps across refreshes (structural sharing)', async () => {
    const d = exporterData(['n0', 'n1']);
    const request = prom({ data: d });
    const src = createMetricsSource({ request });
    const a = await src.fetchGpuMetrics();
    const b = await src.fetchGpuMetrics();
    expect(b.gpus).toBe(a.gpus);
    expect(b.xgmi).toBe(a.xgmi);
    // One GPU's power changes: a new list, every other GPU object reused.
    d[SERIES.exporter.power][0].value = [1760000001, '999'];
    const c = await src.fetchGpuMetrics();
    expect(c.gpus).not.toBe(b.gpus);
    const changed = c.gpus.filter((g, i) => g !== b.gpus[i]);
    expect(changed).toHaveLength(1);
    expect(changed[0].powerWatts).toBe(999);
  });
  it('shareMap keeps equal entries and returns prev when nothing changed', () => {
    const prev = { n0: { '0-1': 1 }, n1: { '0-1': 2 } };
    expect(shareMap(prev, { n0: { '0-1': 1 }, n1: { '0-1': 2 } })).toBe(prev);
    const next = shareMap(prev, { n0: { '0-1': 1 }, n1: { '0-1': 3 } });
    expect(next).not.toBe(prev);
    expect(next.n0).toBe(prev.n0);
    expect(next.n1).toEqual({ '0-1': 3 });
    expect(shareGpus(null, [1])).toEqual([1]);
  });
  it('projects exporter series onto the labels the join reads', () => {
    const q = exporterQuery();
    expect(q.indexOf('max by (__name__, hostname,')).toBe(0);
    EXPORTER_JOIN_LABELS.forEach((l) => expect(q).toContain(l));
    expect(q).not.toContain('serial_number');
  });
  it('asks for the static link topology only when its cached copy is stale', async () => {
    const d = exporterData(['n0']);
    d.gpu_xgmi_link_hops = [vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n0', gpu_id: '0', peer_gpu_id: '1' }, 1)];
    const request = prom({ data: d });
    let now = 1000000;
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    const asked = () =>
      request.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('gpu_power_usage') >= 0);
    await src.fetchGpuMetrics();
    now += 1000;
    const m = await src.fetchGpuMetrics();
    expect(asked()[0]).toContain('gpu_xgmi_link_hops');
    expect(asked()[1]).not.toContain('gpu_xgmi_link_hops');
    expect(m.links.n0).toEqual({ '0-1': { type: 'XGMI', hops: 1 } }); // served from the cache
    now += 10 * 60 * 1000;
    await src.fetchGpuMetrics();
    expect(asked()[asked().length - 1]).toContain('gpu_xgmi_link_hops');
  });
  it('fetches static per-GPU series with the topology and serves them from the copy in between', async () => {
    const E = SERIES.exporter;
    const d = exporterData(['n0']);
    d[E.powerCap] = [vec({ __name__: E.powerCap, hostname: 'n0', gpu_id: '0' }, 1200)];
    const request = prom({ data: d });
    let now = 1000000;
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    const a = await src.fetchGpuMetrics();
    now += 1000;
    const b = await src.fetchGpuMetrics();
    const second = decodeURIComponent(request.mock.calls[1][0]);
    [E.powerCap, E.vramTotal, E.tempSlowdown].forEach((n) => expect(second).not.toContain(n));
    expect(b.gpus[0].powerCapWatts).toBe(1200);
    expect(b.gpus[0].vramTotalBytes).toBe(a.gpus[0].vramTotalBytes);
    expect(b.gpus).toBe(a.gpus); // nothing changed: the same objects
  });
  it('drops the fallback keys from live-only queries once every exporter series carries hostname', async () => {
    const E = SERIES.exporter;
    // The fake answers with the labels the `max by (...)` projection keeps, as Prometheus does.
    const inner = prom({ data: exporterData(['n0', 'n1']), ne: { [SERIES.nodeExporter.power]: [vec({ __name__: SERIES.nodeExporter.power, instance: 'x:9100' }, 5)] } });
    const request = vi.fn((p) => inner(p).then((r) => {
      const q = decodeURIComponent((p.split('query=')[1] || '').split('&')[0]);
      const by = /^max by \(([^)]*)\)/.exec(q);
      if (!by || !r.data) return r;
      const keep = by[1].split(', ');
      const result = r.data.result.map((row) => {
        const m = {};
        keep.forEach((k) => { if (row.metric[k] !== undefined) m[k] = row.metric[k]; });
        return { metric: m, value: row.value };
      });
      return ok(result);
    }));
    let now = 1000000;
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    const a = await src.fetchGpuMetrics(); // merged discovery query: full projection, node-exporter rows ignored
    now += 1000;
    const b = await src.fetchGpuMetrics();
    const asked = request.mock.calls.map((x) => decodeURIComponent(x[0]));
    expect(asked[0]).toContain('instance');
    expect(/max by \(([^)]*)\)/.exec(asked[1])[1]).toBe(EXPORTER_LEAN_LABELS.join(', '));
    expect(b.gpus.map((g) => g.instance)).toEqual(a.gpus.map((g) => g.instance));
    expect(b.gpus[9]).toMatchObject({ nodeName: 'n1', gpu: '1', instance: 'n1:5000', powerWatts: 701 });
    expect(b.gpus).toBe(a.gpus); // same content: structural sharing still hits
    expect(exporterQuery(true, true)).toBe(exporterQuery(true)); // static queries keep the fallback keys
  });
  it('keeps the fallback keys when an exporter series has no hostname', async () => {
    const d = exporterData(['n0']);
    d[SERIES.exporter.temp].push(vec({ __name__: SERIES.exporter.temp, instance: '10.0.0.9:5000', gpu_id: '0' }, 70));
    expect(keyedByHostname(d)).toBe(false);
    expect(keyedByHostname(exporterData(['n0']))).toBe(true);
    expect(keyedByHostname({})).toBe(false);
    const request = prom({ data: d });
    let now = 1000000;
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    await src.fetchGpuMetrics();
    now += 1000;
    await src.fetchGpuMetrics();
    expect(/max by \(([^)]*)\)/.exec(decodeURIComponent(request.mock.calls[1][0]))[1]).toBe(EXPORTER_JOIN_LABELS.join(', '));
  });
  it('projects one node\'s gauges onto what the detail pages read: no hostname (the matcher), no instance', () => {
    [true, false].forEach((withStatic) => {
      const q = exporterNodeQuery('n0', withStatic);
      expect(q.indexOf('max by (' + NODE_GAUGE_LABELS.join(', ') + ') ({__name__=~"gpu_power_usage|')).toBe(0);
      expect(q).not.toContain('max by (' + EXPORTER_JOIN_LABELS.join(', ') + ')');
      expect(q).not.toContain('max by (' + EXPORTER_LEAN_LABELS.join(', ') + ')');
      // xGMI throughput comes placed (or summed per GPU), never as per-neighbour rows
      expect(q).toContain('"__name__", "' + SERIES.nodeShaped.xgmiLink + '"');
      expect(q).toContain('"__name__", "' + SERIES.nodeShaped.xgmiGpu + '"');
      // the topology only with the static series
      expect(q.indexOf(SERIES.nodeShaped.oneHopLinks) >= 0).toBe(withStatic);
    });
    expect(NODE_GAUGE_LABELS).toEqual(['__name__', 'gpu_id', 'pod', 'namespace']);
  });
  it('one node\'s answer: gauges keyed by the asked node, throughput placed by the link series, the mesh from its counts', async () => {
    const d = exporterData(['n0', 'n1']);
    // n1 GPU 0's neighbour 0 is GPU 5 (this repo's exporter says so); the others have no link series
    d.gpu_xgmi_link_hops = [vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n1', gpu_id: '0', peer_gpu_id: '5', neighbor: '0' }, 1)];
    for (let p = 1; p < 8; p++) if (p !== 5) d.gpu_xgmi_link_hops.push(vec({ __name__: 'gpu_xgmi_link_hops', hostname: 'n1', gpu_id: '0', peer_gpu_id: String(p), neighbor: String(p) }, 1));
    const m = await createMetricsSource({ request: prom({ data: d }) }).fetchNodeMetrics('n1');
    expect(m.gpus.map((g) => g.nodeName)).toEqual(Array(8).fill('n1'));
    expect(m.xgmi.n1['0-5']).toBe(50);
    expect(m.xgmi.n1['3>*']).toBe(50); // GPU 3: no link series, its total only
    expect(m.xgmi.n1['0>*']).toBeUndefined();
    // GPU 0 has its 7 one-hop links: counted by Prometheus, expanded here
    expect(Object.keys(m.links.n1).sort()).toEqual(['0-1', '0-2', '0-3', '0-4', '0-5', '0-6', '0-7']);
  });
  it('refetches the static series when a GPU appears that the copy does not know', async () => {
    const E = SERIES.exporter;
    let inner = prom({ data: exporterData(['n0']) });
    const request = vi.fn((p) => inner(p));
    let now = 1000000;
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    await src.fetchGpuMetrics();
    // A node joins: its live series arrive on the next refresh, without statics.
    inner = prom({ data: exporterData(['n0', 'n1']) });
    now += 1000;
    await src.fetchGpuMetrics();
    now += 1000;
    const c = await src.fetchGpuMetrics();
    const asked = request.mock.calls.map((x) => decodeURIComponent(x[0]));
    expect(asked[1]).not.toContain(E.vramTotal);
    expect(asked[2]).toContain(E.vramTotal);
    expect(c.gpus.find((g) => g.nodeName === 'n1').vramTotalBytes).toBeGreaterThan(0);
  });
  it('applyStatics reports GPUs missing from the copy', () => {
    const g = [{ nodeName: 'n', gpu: '0', powerCapWatts: null }, { nodeName: 'n', gpu: '1', powerCapWatts: null }];
    const st = staticsOf([{ nodeName: 'n', gpu: '0', powerCapWatts: 1400, vramTotalBytes: 1, tempSlowdownC: 100 }]);
    expect(applyStatics(g, st)).toBe(false);
    expect(g[0].powerCapWatts).toBe(1400);
    expect(g[1].powerCapWatts).toBeNull();
  });
  it('remembers the answering source and skips the other', async () => {
    const request = prom();
    const src = createMetricsSource({ request });
    await src.fetchGpuMetrics();
    const n = request.mock.calls.length;
    await src.fetchGpuMetrics();
    const second = request.mock.calls.slice(n).map((c) => decodeURIComponent(c[0]));
    expect(second.some((p) => p.indexOf('node_hwmon') >= 0)).toBe(false);
    expect(second).toHaveLength(1);
  });
  it('falls back to node-exporter amdgpu hwmon + DRM', async () => {
    const i = '10.0.0.1:9100';
    const ne = {
      chips: [
        vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: '0000:15:00_0', chip_name: 'amdgpu' }, 1),
        vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: '0000:05:00_0', chip_name: 'amdgpu' }, 1),
        vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: 'platform_coretemp_0', chip_name: 'coretemp' }, 1),
      ],
      power: [
        vec({ __name__: 'node_hwmon_power_average_watt', instance: i, chip: '0000:05:00_0' }, 650),
        vec({ __name__: 'node_hwmon_power_average_watt', instance: i, chip: '0000:15:00_0' }, 900),
      ],
      busy: [vec({ __name__: 'node_drm_gpu_busy_percent', instance: i, card: 'card1' }, 88)],
      uname: [vec({ __name__: 'node_uname_info', instance: i, nodename: 'mi355x-0' }, 1)],
    };
    const src = createMetricsSource({ request: prom({ data: null, ne }) });
    const m = await src.fetchGpuMetrics();
    expect(m.source).toBe('node-exporter');
    expect(m.gpus.map((g) => [g.nodeName, g.gpu, g.powerWatts])).toEqual([
      ['mi355x-0', '0', 650],
      ['mi355x-0', '1', 900],
    ]);
    expect(m.gpus[1].gfxActivityPct).toBe(88);
  });
  it('first fetch: one merged query straight to the preferred service, no discovery probes', async () => {
    const request = prom();
    const src = createMetricsSource({ request });
    const m = await src.fetchGpuMetrics();
    const paths = request.mock.calls.map((c) => decodeURIComponent(c[0]));
    expect(paths).toHaveLength(1);
    expect(paths[0].indexOf(BASE0)).toBe(0);
    expect(paths[0]).toContain('gpu_power_usage|gpu_used_vram');
    expect(paths[0]).toContain('gpu_power_cap|gpu_total_vram');
    expect(paths[0]).toContain('node_hwmon_chip_names|node_hwmon_power_average_watt');
    expect(m.source).toBe('amd-exporter');
    await src.fetchGpuMetrics();
    const second = decodeURIComponent(request.mock.calls[1][0]);
    expect(second).toContain('gpu_power_usage');
    expect(second).not.toContain('node_hwmon'); // only the exporter that answered
  });
  it('falls back to parallel discovery when the preferred service does not answer', async () => {
    const request = prom({ up: [BASE1] });
    const src = createMetricsSource({ request });
    const m = await src.fetchGpuMetrics();
    expect(m.prometheusPath).toBe(BASE1);
    const probes = request.mock.calls.filter((c) => c[0].indexOf('query=1') >= 0);
    expect(probes).toHaveLength(PROMETHEUS_SERVICES.length);
    expect(m.gpus.length).toBeGreaterThan(0);
  });
  it('the merged first query projects onto both joins\' labels', () => {
    const q = mergedQuery();
    ['hostname', 'gpu_id', 'pod', 'chip', 'card', 'nodename'].forEach((l) => expect(q).toContain(l));
    expect(q.indexOf('max by (')).toBe(0);
  });
  it('returns an empty GPU list when Prometheus has no AMD series', async () => {
    const src = createMetricsSource({ request: prom({ data: null }) });
    const m = await src.fetchGpuMetrics();
    expect(m.gpus).toHaveLength(0);
    expect(m.source).toBeNull();
  });
  it('fills the power cap with the MI355X board power when absent', async () => {
    const src = createMetricsSource({ request: prom() });
    const m = await src.fetchGpuMetrics();
    expect(m.gpus[0].powerCapWatts).toBe(1400);
  });
});

describe('page views (each page asks only for what it draws)', () => {
  const E = SERIES.exporter;
  const queried = (request) => request.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('max by') >= 0);

  it('lists the views', () => {
    expect(METRIC_VIEWS).toEqual(['all', 'gauges', 'topology']);
  });

  it("'gauges' (Metrics page) asks for every per-GPU gauge and no xGMI link", () => {
    const q = exporterQuery(false, true, 'gauges');
    [E.power, E.vramUsed, E.gfx, E.umc, E.temp, E.eccCorrect, E.eccUncorrect].forEach((n) => expect(q).toContain(n));
    expect(q).not.toContain('xgmi');
    expect(mergedQuery(true, 'gauges')).not.toContain(E.xgmiRe);
  });

  it("'topology' (GPU Nodes page) asks for the owner-bearing power gauge, the junction temperature and the xGMI links only", () => {
    const q = exporterQuery(false, true, 'topology');
    expect(q).toContain(E.power);
    expect(q).toContain(E.temp);
    expect(q).toContain(E.xgmiRe);
    [E.vramUsed, E.gfx, E.umc, E.eccCorrect].forEach((n) => expect(q).not.toContain(n));
    // static series (link hops, caps) still ride along when the cached copy is stale
    expect(exporterQuery(true, false, 'topology')).toContain(E.linkHops);
  });

  it("'all' is the union and the default", () => {
    expect(exporterQuery(false, true)).toBe(exporterQuery(false, true, 'all'));
    const all = exporterQuery(false, true, 'all');
    expect(all).toContain(E.xgmiRe);
    expect(all).toContain(E.gfx);
  });

  it('a gauges snapshot has the GPU gauges and no links; a topology snapshot has owners and links', async () => {
    const request = prom({ data: exporterData(['n0', 'n1']) });
    const src = createMetricsSource({ request });
    const g = await src.fetchGpuMetrics('gauges');
    expect(g.view).toBe('gauges');
    expect(g.gpus).toHaveLength(16);
    expect(g.gpus[3].gfxActivityPct).toBe(50);
    expect(Object.keys(g.xgmi)).toHaveLength(0);
    const t = await src.fetchGpuMetrics('topology');
    expect(t.view).toBe('topology');
    expect(Object.keys(t.xgmi).sort()).toEqual(['n0', 'n1']);
    expect(t.gpus.filter((x) => x.pod).map((x) => x.nodeName + '/' + x.pod)).toEqual(['n0/train-0', 'n0/train-1', 'n1/train-0', 'n1/train-1']);
    expect(t.gpus[0].gfxActivityPct).toBe(null);
    // the static copy fetched by the first query serves the second
    expect(t.gpus[0].vramTotalBytes).toBe(g.gpus[0].vramTotalBytes);
    const qs = queried(request);
    expect(qs.filter((q) => q.indexOf(E.xgmiRe) >= 0)).toHaveLength(1);
  });

  it('each view keeps its own previous snapshot for sharing and stale fallbacks', async () => {
    const src = createMetricsSource({ request: prom({ data: exporterData(['n0']) }) });
    const g1 = await src.fetchGpuMetrics('gauges');
    await src.fetchGpuMetrics('topology');
    const g2 = await src.fetchGpuMetrics('gauges');
    expect(g2.gpus).toBe(g1.gpus);
  });

  it('rejects an unknown view', async () => {
    const src = createMetricsSource({ request: prom() });
    let err = null;
    await src.fetchGpuMetrics('everything').catch((e) => { err = e; });
    expect(String(err)).toContain('unknown view');
  });

  it('a gauges refresh moves about half the bytes of the all-series refresh', async () => {
    const sizes = {};
    for (const v of ['all', 'gauges', 'topology']) {
      const request = prom({ data: exporterData(['n0', 'n1', 'n2', 'n3']) });
      const src = createMetricsSource({ request });
      await src.fetchGpuMetrics(v); // static copy
      const before = request.mock.calls.length;
      await src.fetchGpuMetrics(v);
      const res = await request.mock.results[before].value;
      sizes[v] = JSON.stringify(res).length;
    }
    expect(sizes.gauges).toBeLessThan(sizes.all);
    expect(sizes.topology).toBeLessThan(sizes.all);
  });
});

describe('in-flight sharing', () => {
  const live = (request) => request.mock.calls.filter((c) => decodeURIComponent(c[0]).indexOf('max by') >= 0).length;

  it('concurrent fetches of one view share one request and one answer', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    const [a, b] = await Promise.all([src.fetchGpuMetrics('gauges'), src.fetchGpuMetrics('gauges')]);
    expect(a).toBe(b);
    expect(live(request)).toBe(1);
  });

  it('different views, owners and nodes are separate requests', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    await src.fetchGpuMetrics('gauges');
    const n = live(request);
    await Promise.all([src.fetchGpuMetrics('gauges'), src.fetchGpuMetrics('topology'), src.fetchGpuOwners(), src.fetchNodeMetrics('n0'), src.fetchNodeMetrics('n0')]);
    expect(live(request) - n).toBe(4);
  });

  it('concurrent range fetches of one window share one query_range', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    const [a, b] = await Promise.all([src.fetchSeries(1800, 30), src.fetchSeries(1800, 30)]);
    expect(a).toBe(b);
    expect(request.mock.calls.filter((c) => c[0].indexOf('/query_range') >= 0)).toHaveLength(1);
  });

  it('a fetch after the previous one settled asks again', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    await src.fetchGpuMetrics();
    await src.fetchGpuMetrics();
    expect(live(request)).toBe(2);
  });
});

describe('hostile / malformed answers', () => {
  it('a series named "__proto__" is a plain key, not a prototype write', () => {
    const out = splitByName([{ metric: { __name__: '__proto__', hostname: 'n0' }, value: [0, '1'] }, null, { metric: 'x' }]);
    expect(Array.isArray(out.__proto__)).toBe(true);
    expect(Object.getPrototypeOf(out)).toBeNull();
    expect({}.push).toBeUndefined();
  });

  it('range answers with malformed rows and points are filtered, not thrown on', async () => {
    const request = vi.fn((path) => {
      if (path.indexOf('query=1') >= 0) return Promise.resolve(ok([{ metric: {}, value: [0, '1'] }]));
      return Promise.resolve({
        status: 'success',
        data: {
          resultType: 'matrix',
          result: [
            null,
            { metric: null, values: [] },
            { metric: { __name__: 'gpu_power_usage', hostname: 'n0' }, values: [[3000, '5'], 'bad', [3030]] },
            { metric: { __name__: 'gpu_power_usage', hostname: 'n1' }, values: 'nope' },
          ],
        },
      });
    });
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => 3600 * 1000 } });
    const sr = await src.fetchSeries(1800, 30);
    expect(Object.keys(sr.power)).toEqual(['n0']);
    expect(sr.power.n0).toEqual([[3000, 5]]);
    const ps = await src.fetchPodSeries('ml', 'p', 1800, 30);
    expect(ps.power).toEqual([[3000, 5]]);
  });
});

describe('failureReason (RBAC vs outage)', () => {
  it('"forbidden" when the service proxy answers 403, "unreachable" on 503, cleared by a success', async () => {
    let mode = 403;
    const request = vi.fn(() => (mode === 200
      ? Promise.resolve(ok([{ metric: {}, value: [0, '1'] }]))
      : Promise.reject(Object.assign(new Error('HTTP ' + mode), { status: mode }))));
    const src = createMetricsSource({ request });
    expect(await src.fetchGpuMetrics('gauges')).toBeNull();
    expect(src.failureReason()).toBe('forbidden');
    mode = 503;
    expect(await src.fetchGpuMetrics('gauges')).toBeNull();
    expect(src.failureReason()).toBe('unreachable');
    mode = 200;
    await src.discover();
    expect(src.failureReason()).toBe('unreachable'); // no failure pending: the default wording
  });
});

describe('answer shapes match src/api/types.ts (no tsc offline: this pins the drift)', () => {
  const types = fs.readFileSync(new URL('../../src/api/types.ts', import.meta.url), 'utf8');
  /** {required, optional} top-level field names of `export interface <name>`. */
  function fields(name) {
    const body = new RegExp('export interface ' + name + ' \\{([\\s\\S]*?)\\n\\}').exec(types)[1];
    const out = { required: [], optional: [] };
    body.split('\n').forEach((l) => {
      const m = /^\s{2}(\w+)(\??):/.exec(l);
      if (m) out[m[2] ? 'optional' : 'required'].push(m[1]);
    });
    return out;
  }
  function conforms(obj, name) {
    const f = fields(name);
    const keys = Object.keys(obj).filter((k) => obj[k] !== undefined);
    f.required.forEach((k) => expect([name, k, k in obj]).toEqual([name, k, true]));
    keys.forEach((k) => expect([name, k, f.required.concat(f.optional).indexOf(k) >= 0]).toEqual([name, k, true]));
  }
  it('GpuMetrics / GpuTelemetry / GpuTotals of a cluster-wide, a scoped and a summary answer', async () => {
    const src = createMetricsSource({ request: prom({ data: exporterData(['n0', 'n1']) }) });
    const all = await src.fetchGpuMetrics();
    conforms(all, 'GpuMetrics');
    all.gpus.forEach((g) => conforms(g, 'GpuTelemetry'));
    const scoped = await src.fetchGpuMetrics('gauges', { scope: ['n0'], summary: true });
    conforms(scoped, 'GpuMetrics');
    conforms(scoped.totals, 'GpuTotals');
    scoped.gpus.forEach((g) => conforms(g, 'GpuTelemetry'));
    const owners = await src.fetchGpuOwners();
    conforms(owners, 'GpuMetrics');
    const sr = await src.fetchSeries(1800, 30, ['n0']);
    conforms(sr, 'GpuSeries');
  });
  it('a node-exporter answer', async () => {
    const i = '10.0.0.1:9100';
    const ne = {
      chips: [vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: '0000:05:00_0', chip_name: 'amdgpu' }, 1)],
      power: [vec({ __name__: 'node_hwmon_power_average_watt', instance: i, chip: '0000:05:00_0' }, 650)],
      uname: [vec({ __name__: 'node_uname_info', instance: i, nodename: 'mi355x-0' }, 1)],
    };
    const m = await createMetricsSource({ request: prom({ data: null, ne }) }).fetchGpuMetrics();
    conforms(m, 'GpuMetrics');
    m.gpus.forEach((g) => conforms(g, 'GpuTelemetry'));
  });
});

describe('power / HBM series on either source', () => {
  const ne = () => ({
    chips: [vec({ __name__: 'node_hwmon_chip_names', instance: 'i0', chip: '0000:05:00_0', chip_name: 'amdgpu' }, 1)],
    power: [vec({ __name__: 'node_hwmon_power_input_watt', instance: 'i0', chip: '0000:05:00_0' }, 650)],
    uname: [vec({ __name__: 'node_uname_info', instance: 'i0', nodename: 'mi355x-0' }, 1)],
  });
  const ranges = (request) => request.mock.calls.map((c) => decodeURIComponent(c[0])).filter((p) => p.indexOf('/query_range') >= 0);
  it('before any answer says which exporter feeds Prometheus: the exporter\'s window, node-exporter\'s only if it finds nothing', async () => {
    // (the JS fake answers every range query with exporter-shaped rows unless told otherwise)
    const empty = vi.fn((path) => (path.indexOf('/query_range') >= 0 && path.indexOf('node_uname_info') < 0
      ? Promise.resolve({ status: 'success', data: { resultType: 'matrix', result: [] } }) : prom({ data: null, ne: ne() })(path)));
    // as the pages fetch: the telemetry (whose answer decides the source) next to the window
    const src = createMetricsSource({ request: empty });
    await Promise.all([src.fetchGpuMetrics('gauges', { scope: ['mi355x-0'], summary: true }), src.fetchSeries(1800, 30, ['mi355x-0'])]);
    const [first, second] = ranges(empty);
    expect(first).toContain('sum by (__name__, hostname) ({__name__=~"gpu_power_usage|gpu_used_vram", hostname=~"mi355x-0"})');
    expect(first).not.toContain('node_uname_info');
    expect(second).toContain('node_uname_info{nodename=~"mi355x-0"}');
    // an exporter cluster: one window, no node-exporter query
    const request = prom({ data: exporterData(['mi355x-0']) });
    await createMetricsSource({ request }).fetchSeries(1800, 30, ['mi355x-0']);
    expect(ranges(request)).toHaveLength(1);
    // no GPU telemetry at all: the empty window stands, nothing more is asked
    const none = vi.fn((path) => (path.indexOf('/query_range') >= 0
      ? Promise.resolve({ status: 'success', data: { resultType: 'matrix', result: [] } }) : prom({ data: {} })(path)));
    const s2 = createMetricsSource({ request: none });
    await Promise.all([s2.fetchGpuMetrics('gauges', { scope: ['mi355x-0'], summary: true }), s2.fetchSeries(1800, 30, ['mi355x-0'])]);
    expect(ranges(none)).toHaveLength(1);
  });
  it('on a node-exporter source: node-exporter\'s lines alone, through node_uname_info', async () => {
    const request = prom({ data: null, ne: ne() });
    const src = createMetricsSource({ request });
    await src.fetchGpuMetrics();
    await src.fetchSeries(1800, 30, ['mi355x-0']);
    await src.fetchNodeSeries('mi355x-0', 1800, 30);
    const [page, node] = ranges(request);
    expect(page).toContain('node_uname_info{nodename=~"mi355x-0"}');
    expect(page).not.toContain('hostname=~');
    expect(node).toContain('node_uname_info{nodename="mi355x-0"}');
    expect(node).not.toContain('hostname=');
  });
  it('on an exporter source: the exporter\'s lines alone', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    await src.fetchGpuMetrics();
    await src.fetchSeries(1800, 30, ['n0']);
    expect(ranges(request)[0]).not.toContain('node_uname_info');
  });
});
