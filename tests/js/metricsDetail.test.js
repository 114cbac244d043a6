/**
 * Metrics-client specs, second half: the detail pages' fetches (node
 * telemetry, pod and node power history), the GPU Pods page's attribution,
 * the exporter joins called directly, range series and the Metrics summary.
 * Discovery, the page views, sharing and failure handling are in
 * metrics.test.js.
 */
import { createMetricsSource } from '../../src/api/metrics.js';
import {
  exporterNodeQuery,
  exporterQuery,
  mergedQuery,
  nodePowerQuery,
  ownersQuery,
  podPowerQuery,
  promString,
} from '../../src/api/promql.js';
import { EXPORTER_JOIN_LABELS, SERIES } from '../../src/api/series.js';
import {
  joinExporterResults,
  joinNodeExporterResults,
  nodeSlice,
  stringLabels,
  summarizeMetrics,
} from '../../src/api/telemetry.js';

import { exporterData, flatten, ok, prom, vec } from './promFake.js';
import { nodeDetailView } from '../../src/view/pages/details.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { renderSection } from '../../src/view/html.js';
import { makeContext, makeGpuNode, makeGpuPod, NOW } from './fixtures.js';

describe('fetchPodSeries (Pod detail power history)', () => {
  it('asks for one pod\'s power, summed per step, with escaped matchers', () => {
    expect(podPowerQuery('ml', 'train-0')).toBe('sum by (__name__) ({__name__="gpu_power_usage", namespace="ml", pod="train-0"})');
    expect(podPowerQuery('a"b', 'c\\d')).toContain('namespace="a\\"b", pod="c\\\\d"');
  });

  it('returns the step-aligned total over the window (rows summed per step)', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => 1800 * 1000 * 1000 } });
    const sr = await src.fetchPodSeries('ml', 'train-0', 1800, 30);
    const q = decodeURIComponent(request.mock.calls.map((c) => c[0]).find((p) => p.indexOf('/query_range') >= 0));
    expect(q).toContain('pod="train-0"');
    expect(q).toContain('step=30');
    expect(sr.rangeSec).toBe(1800);
    // the fake answers two power points for one node
    expect(sr.power.map((p) => p[1])).toEqual([100, 200]);
    expect(sr.power[0][0]).toBeLessThan(sr.power[1][0]);
  });

  it('node history: hostname-scoped query; node and pod histories are separate requests', async () => {
    expect(nodePowerQuery('mi355x-0')).toBe('sum by (__name__) ({__name__="gpu_power_usage", hostname="mi355x-0"})');
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    const [n, p] = await Promise.all([src.fetchNodeSeries('n0', 1800, 30), src.fetchPodSeries('ml', 'n0', 1800, 30)]);
    expect(n.power.length).toBeGreaterThan(0);
    expect(n).not.toBe(p);
    expect(request.mock.calls.filter((c) => c[0].indexOf('/query_range') >= 0)).toHaveLength(2);
  });

  it('concurrent fetches of one pod share a request; unreachable Prometheus gives null', async () => {
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request });
    const [a, b] = await Promise.all([src.fetchPodSeries('ml', 'p', 1800, 30), src.fetchPodSeries('ml', 'p', 1800, 30)]);
    expect(a).toBe(b);
    expect(request.mock.calls.filter((c) => c[0].indexOf('/query_range') >= 0)).toHaveLength(1);
    const down = createMetricsSource({ request: prom({ up: [] }) });
    expect(await down.fetchPodSeries('ml', 'p', 1800, 30)).toBeNull();
  });
});

describe('fetchNodeMetrics (detail pages)', () => {
  const paths = (request, from) => request.mock.calls.slice(from || 0).map((c) => decodeURIComponent(c[0]));

  it('asks for one node only, with a hostname matcher, and returns that node\'s GPUs', async () => {
    const request = prom({ data: exporterData(['n0', 'n1', 'n2']) });
    const src = createMetricsSource({ request });
    const m = await src.fetchNodeMetrics('n1');
    expect(paths(request)).toHaveLength(1);
    expect(paths(request)[0]).toContain('hostname="n1"');
    expect(m.scope).toBe('n1');
    expect(m.gpus).toHaveLength(8);
    expect(m.gpus.every((g) => g.nodeName === 'n1')).toBe(true);
    expect(m.gpus[0].pod).toBe('train-0');
    expect(Object.keys(m.xgmi)).toEqual(['n1']);
  });
  it('escapes the node name inside the matcher', () => {
    expect(exporterNodeQuery('a"b\\c', false)).toContain('hostname="a\\"b\\\\c"');
    expect(promString('x"y')).toBe('x\\"y');
  });
  it('re-reads a node\'s static series only after the TTL', async () => {
    let now = 0;
    const request = prom({ data: exporterData(['n0']) });
    const src = createMetricsSource({ request, discoveryTtlMs: 1000, clock: { setTimeout, clearTimeout, now: () => now } });
    const a = await src.fetchNodeMetrics('n0');
    await src.fetchNodeMetrics('n0');
    now = 5000;
    await src.fetchNodeMetrics('n0');
    const qs = paths(request);
    expect(qs.map((q) => q.indexOf(SERIES.exporter.vramTotal) >= 0)).toEqual([true, false, true]);
    const b = await src.fetchNodeMetrics('n0');
    expect(b.gpus[0].vramTotalBytes).toBe(a.gpus[0].vramTotalBytes); // from the node's static copy
  });
  it('shares unchanged GPU objects between fetches of the same node', async () => {
    const src = createMetricsSource({ request: prom({ data: exporterData(['n0']) }) });
    const a = await src.fetchNodeMetrics('n0');
    const b = await src.fetchNodeMetrics('n0');
    expect(b.gpus).toBe(a.gpus);
  });
  it('falls back to the cluster-wide snapshot, cut to the node, when the exporter has no such hostname', async () => {
    const i = '10.0.0.1:9100';
    const ne = {
      chips: [vec({ __name__: 'node_hwmon_chip_names', instance: i, chip: '0000:05:00_0', chip_name: 'amdgpu' }, 1)],
      power: [vec({ __name__: 'node_hwmon_power_average_watt', instance: i, chip: '0000:05:00_0' }, 650)],
      uname: [vec({ __name__: 'node_uname_info', instance: i, nodename: 'mi355x-0' }, 1)],
    };
    const request = prom({ data: null, ne });
    const src = createMetricsSource({ request });
    const m = await src.fetchNodeMetrics('mi355x-0');
    expect(m.source).toBe('node-exporter');
    expect(m.gpus.map((g) => [g.nodeName, g.powerWatts])).toEqual([['mi355x-0', 650]]);
    // node-exporter is now the known source: later detail fetches skip the scoped query.
    const n = request.mock.calls.length;
    await src.fetchNodeMetrics('mi355x-0');
    expect(paths(request, n)).toHaveLength(1);
    expect(paths(request, n)[0]).not.toContain('hostname=');
    // ... and read that node alone, through node_uname_info
    expect(paths(request, n)[0]).toContain('and on(instance) node_uname_info{nodename=~"mi355x-0"}');
  });
  it('serves the node\'s last snapshot stale through a transient failure, then null', async () => {
    let up = true;
    const good = prom({ data: exporterData(['n0']) });
    const request = vi.fn((p) => (up ? good(p) : Promise.reject(Object.assign(new Error('503'), { status: 503 }))));
    const src = createMetricsSource({ request });
    const a = await src.fetchNodeMetrics('n0');
    up = false;
    const b = await src.fetchNodeMetrics('n0');
    expect(b.stale).toBe(true);
    expect(b.gpus).toBe(a.gpus);
    await src.fetchNodeMetrics('n0');
    expect(await src.fetchNodeMetrics('n0')).toBeNull();
  });
  it('returns null when Prometheus is unreachable', async () => {
    const src = createMetricsSource({ request: prom({ up: [] }) });
    expect(await src.fetchNodeMetrics('n0')).toBeNull();
  });
  it('nodeSlice keeps the node\'s GPUs, xGMI and links and shares their objects', () => {
    const m = {
      source: 'amd-exporter', fetchedAt: 'x', prometheusPath: 'p',
      gpus: [{ nodeName: 'a', gpu: '0' }, { nodeName: 'b', gpu: '0' }],
      xgmi: { a: { '0-1': 1 }, b: { '0-1': 2 } }, links: { b: { '0-1': { type: 'XGMI', hops: 1 } } },
    };
    const s = nodeSlice(m, 'b');
    expect(s.gpus).toEqual([m.gpus[1]]);
    expect(s.gpus[0]).toBe(m.gpus[1]);
    expect(s.xgmi).toEqual({ b: { '0-1': 2 } });
    expect(s.links.b).toBe(m.links.b);
    expect(s.source).toBe('amd-exporter');
  });
});

describe('fetchGpuOwners (Pods page)', () => {
  it('asks for the power gauge of pod-attributed GPUs only', async () => {
    const request = prom({ data: exporterData(['n0', 'n1']) });
    const src = createMetricsSource({ request });
    const m = await src.fetchGpuOwners();
    const q = decodeURIComponent(request.mock.calls[0][0]);
    expect(request.mock.calls).toHaveLength(1);
    expect(q).toContain('pod!=""');
    expect(q).not.toContain('xgmi');
    expect(m.scope).toBe('owners');
    expect(m.gpus.map((g) => [g.nodeName, g.gpu, g.pod])).toEqual([
      ['n0', '0', 'train-0'], ['n0', '1', 'train-1'], ['n1', '0', 'train-0'], ['n1', '1', 'train-1'],
    ]);
    expect(m.gpus[0].powerWatts).toBe(700);
  });
  it('an empty answer means no attribution, not an unreachable Prometheus', async () => {
    const src = createMetricsSource({ request: prom({ data: null }) });
    const m = await src.fetchGpuOwners();
    expect(m).not.toBeNull();
    expect(m.gpus).toEqual([]);
  });
  it('serves the last attribution stale through a transient failure', async () => {
    let up = true;
    const good = prom();
    const request = vi.fn((p) => (up ? good(p) : Promise.reject(Object.assign(new Error('503'), { status: 503 }))));
    const src = createMetricsSource({ request });
    const a = await src.fetchGpuOwners();
    up = false;
    const b = await src.fetchGpuOwners();
    expect(b.stale).toBe(true);
    expect(b.gpus).toBe(a.gpus);
  });
  it('projects onto the join labels', () => {
    expect(ownersQuery()).toBe('max by (' + EXPORTER_JOIN_LABELS.join(', ') + ') ({__name__="gpu_power_usage", pod!=""})');
  });
});

describe('joins (direct)', () => {
  it('joinExporterResults tolerates malformed rows', () => {
    const r = {};
    r[SERIES.exporter.power] = [null, { metric: 'x' }, vec({ hostname: 'n', gpu_id: '0' }, 'NaN')];
    const j = joinExporterResults(r);
    expect(j.gpus).toHaveLength(1);
    expect(j.gpus[0].powerWatts).toBeNull();
  });
  it('reads hwmon power1_input where power1_average does not exist (MI355X), preferring the average', () => {
    const N = SERIES.nodeExporter;
    const r = {};
    r[N.chips] = [vec({ instance: 'i', chip: 'c0', chip_name: 'amdgpu' }, 1), vec({ instance: 'i', chip: 'c1', chip_name: 'amdgpu' }, 1)];
    r[N.powerInput] = [vec({ instance: 'i', chip: 'c0' }, 700), vec({ instance: 'i', chip: 'c1' }, 800)];
    r[N.power] = [vec({ instance: 'i', chip: 'c1' }, 810)];
    const g = joinNodeExporterResults(r).gpus;
    expect(g[0].powerWatts).toBe(700);
    expect(g[1].powerWatts).toBe(810);
  });
  it('joinNodeExporterResults maps instance to nodename', () => {
    const N = SERIES.nodeExporter;
    const r = {};
    r[N.chips] = [vec({ instance: 'i', chip: 'c' }, 1)];
    r[N.uname] = [vec({ instance: 'i', nodename: 'node-x' }, 1)];
    expect(joinNodeExporterResults(r).gpus[0].nodeName).toBe('node-x');
  });
});

describe('fetchSeries', () => {
  it('returns per-node power and HBM series', async () => {
    const src = createMetricsSource({ request: prom(), clock: { setTimeout, clearTimeout, now: () => 1000000 } });
    const s = await src.fetchSeries(600, 30);
    expect(s.power.n0).toEqual([[960, 100], [990, 200]]);
    expect(s.vram.n0[1][1]).toBe(200 * 1024 * 1024);
  });
  it('fetches only new steps after the first call', async () => {
    let now = 1000000;
    const request = prom();
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    await src.fetchSeries(600, 30);
    const ranges = () => request.mock.calls.map((c) => c[0]).filter((p) => p.indexOf('query_range') >= 0);
    expect(ranges()).toHaveLength(1); // power and HBM in one query
    now += 10000; // same 30 s step: served from cache, no request
    await src.fetchSeries(600, 30);
    expect(ranges()).toHaveLength(1);
    now += 50000; // two steps later: only the new window is requested
    await src.fetchSeries(600, 30);
    expect(ranges()).toHaveLength(2);
    const last = ranges()[1];
    const startT = Number(/start=(\d+)/.exec(last)[1]);
    const endT = Number(/end=(\d+)/.exec(last)[1]);
    expect(endT - startT).toBe(30);
  });
  it('drops points that fall out of the window and keeps merged history', async () => {
    let now = 1000000;
    const request = vi.fn((path) => {
      if (path.indexOf('query=1') >= 0) return Promise.resolve(ok([]));
      const start = Number(/start=(\d+)/.exec(path)[1]);
      const end = Number(/end=(\d+)/.exec(path)[1]);
      const values = [];
      for (let t = start; t <= end; t += 30) values.push([t, '1']);
      return Promise.resolve({
        status: 'success',
        data: { resultType: 'matrix', result: [{ metric: { __name__: 'gpu_power_usage', hostname: 'n0' }, values }] },
      });
    });
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => now } });
    const a = await src.fetchSeries(300, 30);
    expect(a.power.n0).toHaveLength(11);
    now += 90000;
    const b = await src.fetchSeries(300, 30);
    expect(b.power.n0).toHaveLength(11);
    expect(b.power.n0[10][0]).toBe(Math.floor(now / 1000 / 30) * 30);
  });
  it('passes start/end/step to query_range', async () => {
    const request = prom();
    const src = createMetricsSource({ request, clock: { setTimeout, clearTimeout, now: () => 1000000 } });
    await src.fetchSeries(600, 15);
    const rq = request.mock.calls.map((c) => c[0]).find((p) => p.indexOf('query_range') >= 0);
    expect(rq).toContain('&start=390&end=990&step=15');
  });
});

describe('summarizeMetrics', () => {
  it('sums power, caps and HBM and averages activity', () => {
    const s = summarizeMetrics(joinExporterResults(exporterData(['n0'])));
    expect(s.gpus).toBe(8);
    expect(s.powerWatts).toBe(700 * 8 + 28);
    expect(s.powerCapWatts).toBe(8 * 1400);
    expect(s.avgGfxActivityPct).toBe(50);
  });
  it('totals RAS counters only over GPUs that report them', () => {
    const E = SERIES.exporter;
    const r = exporterData(['n0']);
    r[E.eccCorrect] = [vec({ hostname: 'n0', gpu_id: '0' }, 4), vec({ hostname: 'n0', gpu_id: '1' }, 0)];
    r[E.eccUncorrect] = [vec({ hostname: 'n0', gpu_id: '0' }, 1), vec({ hostname: 'n0', gpu_id: '1' }, 0)];
    const j = joinExporterResults(r);
    expect([j.gpus[0].eccCorrectable, j.gpus[0].eccUncorrectable]).toEqual([4, 1]);
    expect(j.gpus[2].eccUncorrectable).toBeNull();
    const s = summarizeMetrics(j);
    expect([s.eccCorrectable, s.eccUncorrectable]).toEqual([4, 1]);
    expect(summarizeMetrics(joinExporterResults(exporterData(['n0']))).eccUncorrectable).toBeNull();
  });
  it('asks for the RAS counters in the refresh and merged queries', () => {
    const E = SERIES.exporter;
    [exporterQuery(false), mergedQuery(false)].forEach((q) => {
      expect(q).toContain(E.eccCorrect);
      expect(q).toContain(E.eccUncorrect);
    });
  });
});

describe('stringLabels: label values are strings or absent', () => {
  it('returns a clean row as is and drops labels of any other type', () => {
    const clean = { metric: { __name__: 'gpu_power_usage', hostname: 'n0', gpu_id: '0' }, value: [0, '1'] };
    expect(stringLabels(clean)).toBe(clean);
    const dirty = { metric: { __name__: 'gpu_power_usage', hostname: { a: 1 }, gpu_id: 0, card_model: ['x'], pod: null }, value: [0, '2'] };
    expect(stringLabels(dirty)).toEqual({ metric: { __name__: 'gpu_power_usage' }, value: [0, '2'] });
    expect(dirty.metric.hostname).toEqual({ a: 1 }); // the answer itself is not modified
    expect(stringLabels(null)).toBe(null);
    expect(stringLabels({ metric: 'x' })).toEqual({ metric: 'x' });
  });

  it('a node whose hostname label is not a string gets no telemetry, and the others keep theirs', async () => {
    const bad = JSON.parse(JSON.stringify(flatten(exporterData(['n0', 'n1']))));
    bad.forEach((r) => { if (r.metric.hostname === 'n1') r.metric.hostname = { name: 'n1' }; });
    const src = createMetricsSource({ request: (p) => Promise.resolve(/query=1$/.test(p) ? ok([{ metric: {}, value: [0, '1'] }]) : ok(bad)) });
    const m = await src.fetchGpuMetrics('gauges');
    const hosts = new Set(m.gpus.map((g) => g.nodeName));
    expect(hosts.has('n0')).toBe(true);
    expect(m.gpus.filter((g) => g.nodeName === 'n0')).toHaveLength(8);
    expect([...hosts].every((x) => typeof x === 'string')).toBe(true);
  });
});

describe('the one-node answer draws the Node detail section the cluster-wide answer draws', () => {
  /** n1's 8 GPUs on the full mesh, neighbour k of GPU g = GPU (g + 1 + k) % 8, each link a distinct throughput. */
  function meshData(withLinks) {
    const d = exporterData(['n0', 'n1']);
    d.__xgmi = [];
    d.gpu_xgmi_link_hops = [];
    ['n0', 'n1'].forEach((h) => {
      for (let g = 0; g < 8; g++) {
        for (let k = 0; k < 7; k++) {
          const peer = (g + 1 + k) % 8;
          d.__xgmi.push(vec({ __name__: 'xgmi_neighbor_' + k + '_tx_throughput', hostname: h, gpu_id: String(g), instance: h + ':5000' },
            (10 * g + k + 1) * 1e9));
          if (withLinks) {
            d.gpu_xgmi_link_hops.push(vec({ __name__: 'gpu_xgmi_link_hops', hostname: h, gpu_id: String(g), peer_gpu_id: String(peer),
              neighbor: String(k) }, 1));
          }
        }
      }
    });
    return d;
  }

  [true, false].forEach((withLinks) => {
    it((withLinks ? 'links pin the neighbours: throughput per link' : 'no link series: throughput per GPU') + ', the same HTML', async () => {
      const d = meshData(withLinks);
      const node = makeGpuNode('n1');
      const ctx = makeContext({ nodes: [node], pods: [makeGpuPod('train-0', { node: 'n1', gpus: 2 })] });
      const scoped = await createMetricsSource({ request: prom({ data: d }) }).fetchNodeMetrics('n1');
      const wide = nodeSlice(await createMetricsSource({ request: prom({ data: d }) }).fetchGpuMetrics(), 'n1');
      clearViewMemo();
      const a = renderSection(nodeDetailView(node, ctx, { now: NOW, metrics: scoped }));
      clearViewMemo();
      const b = renderSection(nodeDetailView(node, ctx, { now: NOW, metrics: wide }));
      expect(a).toBe(b);
      expect(a).toContain(withLinks ? 'data-throughput="measured"' : 'data-throughput="per-gpu"');
      expect(a).toContain(withLinks ? 'data-topology="measured"' : 'data-topology="assumed"');
      // GPU 2's neighbour 3 is GPU 6: 24 GB/s on that link when pinned; GPU 2's total is 21 + … + 27 = 168
      expect(a).toContain('\u03a3 168.0 GB/s');
      if (withLinks) expect(Object.keys(scoped.xgmi.n1)).toContain('2-6');
      if (withLinks) expect(scoped.xgmi.n1['2-6']).toBe(24);
    });
  });
});

