/**
 * Randomised property checks (seeded, so failures reproduce): the domain
 * model and the structural-sharing helpers against independent oracles
 * over a few hundred generated nodes / pods / snapshots each.
 */
import { getPodGpuDemand } from '../../src/api/amdPods.js';
import { buildClusterIndex } from '../../src/api/clusterIndex.js';
import { formatBytes, formatWatts } from '../../src/api/k8sCore.js';
import { clusterPowerStats, shareGpus, shareMap } from '../../src/api/telemetry.js';
import { buildXgmiMatrix, isFullMesh } from '../../src/api/topology.js';
import { makeGpuNode } from './fixtures.js';
import { int, mutate, pick, rng } from './fuzzlib.js';

/** Every page view-model module, merged (what the fuzz cases call by name). */
async function loadPages() {
  const mods = ['common', 'details', 'devicePlugins', 'metricsPage', 'nodes', 'overview', 'paging', 'pods'];
  const out = {};
  for (let i = 0; i < mods.length; i++) Object.assign(out, await import('../../src/view/pages/' + mods[i] + '.js'));
  return out;
}

const RES = ['amd.com/gpu', 'amd.com/cpx_nps4'];

function randContainer(r, name, sidecar) {
  const requests = {};
  const limits = {};
  RES.forEach((k) => {
    if (r() < 0.5) {
      const v = int(r, 0, 4);
      const mode = int(r, 0, 2); // requests only / limits only / both
      if (mode !== 1) requests[k] = String(v);
      if (mode !== 0) limits[k] = String(mode === 2 ? v : int(r, 0, 4));
    }
  });
  const c = { name, resources: { requests, limits } };
  if (sidecar) c.restartPolicy = 'Always';
  return c;
}

function randPod(r, i, nodes) {
  const containers = [];
  const initContainers = [];
  for (let j = 0, n = int(r, 1, 3); j < n; j++) containers.push(randContainer(r, 'c' + j, false));
  for (let j = 0, n = int(r, 0, 3); j < n; j++) initContainers.push(randContainer(r, 'i' + j, r() < 0.4));
  return {
    metadata: { name: 'p' + i, namespace: 'ns', uid: 'u' + i, creationTimestamp: '2026-10-01T00:00:00Z' },
    spec: { nodeName: r() < 0.9 ? pick(r, nodes) : undefined, containers, initContainers },
    status: { phase: pick(r, ['Running', 'Running', 'Pending', 'Succeeded', 'Failed']) },
  };
}

/** Kubernetes effective request, simulated as a timeline of container starts. */
function oracleDemand(pod, key) {
  const val = (c) => {
    const q = c.resources.requests[key];
    const l = c.resources.limits[key];
    // extended resources: a limit alone implies an equal request
    return q !== undefined ? parseInt(q, 10) : l !== undefined ? parseInt(l, 10) : 0;
  };
  let running = 0; // sidecars started so far
  let peak = 0;
  for (const c of pod.spec.initContainers) {
    if (c.restartPolicy === 'Always') running += val(c);
    else peak = Math.max(peak, running + val(c));
  }
  let steady = running;
  for (const c of pod.spec.containers) steady += val(c);
  return Math.max(peak, steady);
}

describe('properties', () => {
  it('effective GPU demand matches a timeline simulation of container starts', () => {
    const r = rng(42);
    for (let i = 0; i < 400; i++) {
      const p = randPod(r, i, ['n0']);
      const d = getPodGpuDemand(p);
      RES.forEach((k) => expect(d[k] || 0).toBe(oracleDemand(p, k)));
    }
  });

  it('cluster index: per-node sums equal totals, free never negative, terminal pods hold nothing', () => {
    const r = rng(7);
    for (let trial = 0; trial < 40; trial++) {
      const names = [];
      const nodes = [];
      for (let i = 0, n = int(r, 1, 6); i < n; i++) {
        const name = 'n' + i;
        names.push(name);
        nodes.push(makeGpuNode(name, { gpus: int(r, 0, 8) }));
      }
      const pods = [];
      for (let i = 0, n = int(r, 0, 30); i < n; i++) pods.push(randPod(r, i, names.concat(['elsewhere'])));
      const idx = buildClusterIndex(nodes, pods);
      let inUse = 0;
      let cap = 0;
      for (const n of names) {
        inUse += idx.nodeStats.get(n).inUse;
        cap += idx.nodeStats.get(n).capacity;
      }
      expect(idx.totals.inUse).toBe(inUse);
      expect(idx.totals.capacity).toBe(cap);
      expect(idx.totals.free).toBe(Math.max(0, idx.totals.allocatable - idx.totals.inUse));
      expect(idx.totals.free).toBeGreaterThanOrEqual(0);
      let expected = 0;
      for (const p of pods) {
        if (!p.spec.nodeName || names.indexOf(p.spec.nodeName) < 0) continue;
        if (p.status.phase === 'Succeeded' || p.status.phase === 'Failed') continue;
        expected += RES.reduce((s, k) => s + oracleDemand(p, k), 0);
      }
      expect(inUse).toBe(expected);
    }
  });

  it('formatBytes is within 0.5 % of the value and never loses the unit', () => {
    const r = rng(3);
    const unit = { B: 1, KiB: 1024, MiB: 1024 ** 2, GiB: 1024 ** 3, TiB: 1024 ** 4, PiB: 1024 ** 5 };
    for (let i = 0; i < 500; i++) {
      const v = Math.floor(Math.pow(2, r() * 52));
      const [num, u] = formatBytes(v).split(' ');
      expect(unit[u]).toBeDefined();
      const back = parseFloat(num) * unit[u];
      expect(Math.abs(back - v)).toBeLessThanOrEqual(Math.max(0.5, v * 0.005));
    }
  });

  it('structural sharing returns content-equal results and reuses every unchanged element', () => {
    const r = rng(11);
    const mk = () => {
      const gpus = [];
      for (let n = 0; n < 3; n++) {
        for (let g = 0; g < 4; g++) {
          gpus.push({ nodeName: 'n' + n, gpu: String(g), powerWatts: int(r, 0, 2) * 100, pod: r() < 0.5 ? 'p' : null });
        }
      }
      return gpus;
    };
    let prev = mk();
    for (let i = 0; i < 200; i++) {
      const next = mk();
      const out = shareGpus(prev, next);
      expect(out).toEqual(next);
      out.forEach((g, j) => {
        const p = prev.find((x) => x.nodeName === g.nodeName && x.gpu === g.gpu);
        if (JSON.stringify(p) === JSON.stringify(next[j])) expect(g).toBe(p);
      });
      const m1 = { a: { x: int(r, 0, 1) }, b: { y: int(r, 0, 1) } };
      const m2 = { a: { x: int(r, 0, 1) }, b: { y: int(r, 0, 1) } };
      const sm = shareMap(m1, m2);
      expect(sm).toEqual(m2);
      if (JSON.stringify(m1) === JSON.stringify(m2)) expect(sm).toBe(m1);
      prev = out;
    }
  });

  it('a symmetric measured topology gives a symmetric matrix; the default is a full mesh', () => {
    const r = rng(5);
    for (let n = 1; n <= 8; n++) {
      const probed = {};
      for (let i = 0; i < n; i++) {
        for (let j = i + 1; j < n; j++) {
          if (r() < 0.7) probed[i + '-' + j] = probed[j + '-' + i] = { type: 'XGMI', hops: 1 };
        }
      }
      const m = buildXgmiMatrix(n, null, probed);
      for (let i = 0; i < n; i++) for (let j = 0; j < n; j++) expect(m.cells[i][j].kind).toBe(m.cells[j][i].kind);
      expect(isFullMesh(buildXgmiMatrix(n))).toBe(n > 1);
    }
  });

  it('a matrix block\'s facts and summary, read from the link maps, are what its grid says', async () => {
    const { matrixBlock } = await import('../../src/view/pages/nodes.js');
    const { matrixSummary } = await import('../../src/view/ir.js');
    const r = rng(77);
    for (let round = 0; round < 200; round++) {
      const n = int(r, 0, 9);
      const probed = r() < 0.5 ? {} : null;
      const measured = r() < 0.7 ? {} : null;
      for (let i = 0; i < n; i++) {
        for (let j = 0; j < n; j++) {
          if (i === j) continue;
          if (probed && r() < 0.85) probed[i + '-' + j] = { type: r() < 0.8 ? 'XGMI' : 'PCIE', hops: r() < 0.9 ? 1 : 2 };
          if (measured && r() < 0.6) measured[i + '-' + j] = Math.round(r() * 100);
        }
      }
      const b = matrixBlock(n, measured, probed, false);
      const grid = buildXgmiMatrix(n, measured, probed && Object.keys(probed).length ? probed : undefined);
      expect(b.fullMesh).toBe(isFullMesh(grid));
      expect(b.linksPerGpu).toBe(grid.linksPerGpu);
      expect(b.ringBusGBs).toBe(grid.ringBusGBs);
      // the summary from the maps = the summary from the cells
      expect(matrixSummary(b)).toBe(matrixSummary({ matrix: grid }));
      expect(b.matrix.cells).toEqual(grid.cells);
    }
  });
});

describe('malformed cluster objects (what a real apiserver, an old CRD version or a half-written object can hand over)', () => {
  it('no page, detail section, column or index throws on them', async () => {
    const pages = await loadPages();
    const html = await import('../../src/view/html.js');
    const text = await import('../../src/view/text.js');
    const svg = await import('../../src/view/svg.js');
    const { createClusterStore } = await import('../../src/api/clusterStore.js');
    const { makeGpuPod, makePlainPod, makePluginPod, makeNode, makeDeviceConfig } = await import('./fixtures.js');
    const r = rng(4242);
    const ROUNDS = Number(process.env.FUZZ_ROUNDS || 120);
    const now = Date.parse('2026-10-16T00:00:00Z');
    for (let round = 0; round < ROUNDS; round++) {
      const nodes = [makeGpuNode('g0'), makeGpuNode('g1', { partition: 'CPX/NPS4' }), makeNode('c0')].map((n) => (r() < 0.5 ? mutate(r, n, 0) : n));
      const pods = [makeGpuPod('a', { node: 'g0', gpus: 2 }), makeGpuPod('b', { node: 'g1' }), makePlainPod('w', 'c0'), makePluginPod('dp')]
        .map((p) => (r() < 0.5 ? mutate(r, p, 0) : p));
      const dcs = [makeDeviceConfig()].map((d) => (r() < 0.5 ? mutate(r, d, 0) : d));
      const store = createClusterStore({
        request: (path) => Promise.resolve({ kind: 'List', items: path.indexOf('deviceconfigs') >= 0 ? dcs : [] }),
      });
      store.setNodes(nodes, null);
      store.setPods(pods, null);
      await store.refresh();
      const ctx = store.getSnapshot();
      const opts = { now };
      const vms = [pages.overviewView(ctx, opts), pages.devicePluginsView(ctx, opts), pages.nodesView(ctx, opts),
        pages.podsView(ctx, opts), pages.metricsView(ctx, { metrics: null, fetchError: null, fetching: false }, opts)];
      const sections = nodes.map((n) => pages.nodeDetailView(n, ctx, opts)).concat(pods.map((p) => pages.podDetailView(p, opts)));
      // The HTML (bench, snapshots), terminal (bin/amd-gpu-dash.js) and SVG (screenshots) renderers take them too.
      vms.forEach((vm) => {
        expect(typeof html.renderPage(vm)).toBe('string');
        expect(typeof text.renderText(vm, { color: false })).toBe('string');
        const picture = svg.renderPageSvg(vm);
        expect(picture).toMatch(/^<svg [^>]*height="\d+(\.\d)?"[\s\S]*<\/svg>\n$/);
        // no coordinate or size is NaN (a name may well be "NaN": text is the object's)
        expect(/="[^"]*NaN/.test(picture)).toBe(false);
      });
      sections.forEach((sec) => {
        if (!sec) return;
        expect(typeof html.renderSection(sec)).toBe('string');
        expect(text.textSection(sec, false).every((l) => typeof l === 'string')).toBe(true);
        expect(/="[^"]*NaN/.test(svg.renderSectionSvg(sec))).toBe(false);
      });
      const cols = pages.nodeColumns();
      nodes.forEach((n) => cols.forEach((c) => c.getter(n)));
      pages.clearViewMemo();
    }
  });
});

describe('malformed Prometheus answers', () => {
  it('joins and telemetry views never throw on wrong-shaped rows', async () => {
    const pages = await loadPages();
    const { joinExporterResults, joinNodeExporterResults, splitByName, summarizeMetrics, clusterPowerStats } = await import('../../src/api/telemetry.js');
    const { exporterData, flatten } = await import('./promFake.js');
    const { makeContext, makeGpuNode, makeGpuPod } = await import('./fixtures.js');
    const r = rng(77);
    const WRONG = [null, undefined, 0, '', 'NaN', '+Inf', '-1', [], {}, [1], { x: 1 }, 'abc'];
    const ctx = makeContext({ nodes: [makeGpuNode('n0'), makeGpuNode('n1')], pods: [makeGpuPod('train-0', { node: 'n0' })] });
    for (let round = 0; round < 200; round++) {
      const rows = flatten(exporterData(['n0', 'n1'])).map((row) => {
        if (r() > 0.15) return row;
        const k = pick(r, ['metric', 'value', 'metric.gpu_id', 'metric.hostname', 'value.1', 'metric.__name__']);
        const out = JSON.parse(JSON.stringify(row));
        const path = k.split('.');
        let o = out;
        for (let i = 0; i < path.length - 1; i++) o = o[path[i]];
        o[path[path.length - 1]] = pick(r, WRONG);
        return out;
      });
      if (r() < 0.1) rows.push(pick(r, WRONG));
      const split = splitByName(rows.filter((x) => x && typeof x === 'object'));
      const m = Object.assign({ source: 'amd-exporter', fetchedAt: new Date(0).toISOString(), prometheusPath: '/p' }, joinExporterResults(split));
      joinNodeExporterResults(split);
      summarizeMetrics(m);
      const power = { n0: [[0, pick(r, [1, NaN, null])], [30, 2]] };
      clusterPowerStats(power);
      pages.metricsView(ctx, { metrics: m, series: { power, vram: {} }, fetchError: null, fetching: false }, { now: 0 });
      pages.nodesView(ctx, { metrics: m, now: 0 });
      pages.podsView(ctx, { metrics: m, now: 0 });
      pages.nodeDetailView(ctx.gpuNodes[0], ctx, { metrics: m, series: { power: power.n0 } });
      pages.podDetailView(ctx.gpuPods[0], { metrics: m, series: { power: power.n0 } });
      pages.clearViewMemo();
    }
  });

  it('ranked and size-guarded answers with hostile rows never throw, in the client or the Metrics view', async () => {
    const pages = await loadPages();
    const { createMetricsSource } = await import('../../src/api/metrics.js');
    const { exporterData, flatten, ok } = await import('./promFake.js');
    const { makeContext, makeGpuNode } = await import('./fixtures.js');
    const r = rng(91);
    const WRONG = [null, undefined, 0, '', 'NaN', '+Inf', '-1', [], {}, [1], { x: 1 }, 'abc'];
    const ctx = makeContext({ nodes: [makeGpuNode('n0'), makeGpuNode('n1')] });
    for (let round = 0; round < 120; round++) {
      const rows = flatten(exporterData(['n0', 'n1'])).filter(() => r() < 0.7);
      for (let i = 0, n = Math.floor(r() * 6); i < n; i++) {
        const agg = pick(r, ['rank', 'ranked', 'gpu_nodes', 'gpu_pods', 'sum', 'count', 'nodes', pick(r, WRONG)]);
        const metric = { agg: agg };
        if (r() < 0.7) metric.hostname = pick(r, ['n0', 'n1', 'ghost', pick(r, WRONG)]);
        if (r() < 0.4) metric.pod = pick(r, ['train-0', 'ghost', pick(r, WRONG)]);
        if (r() < 0.4) metric.namespace = pick(r, ['ml', pick(r, WRONG)]);
        if (r() < 0.5) metric.__name__ = pick(r, ['gpu_power_usage', 'gpu_total_vram', pick(r, WRONG)]);
        rows.push({ metric: metric, value: [0, pick(r, ['12', '0', '9e99'].concat(WRONG))] });
      }
      if (r() < 0.1) rows.push(pick(r, WRONG));
      const request = (path) => Promise.resolve(/query=1$/.test(path) ? ok([{ metric: {}, value: [0, '1'] }]) : ok(rows));
      const src = createMetricsSource({ request: request });
      const ranked = await src.fetchGpuMetrics('gauges', { rank: { by: 'power', page: Math.floor(r() * 3), per: 8, filter: '' }, summary: true });
      const small = await src.fetchGpuMetrics('topology', { scope: r() < 0.5 ? [] : ['n0'], small: true });
      const owners = await src.fetchGpuOwners({ pods: [], small: true });
      const rankedOwners = await src.fetchGpuOwners({ rank: { by: 'power', page: Math.floor(r() * 3), per: 25, filter: '' } });
      if (rankedOwners) pages.podsView(ctx, { metrics: rankedOwners, now: 0, pager: { sort: 'power' } });
      for (const m of [ranked, small, owners]) {
        const st = { metrics: m, series: null, fetchError: null, fetching: false };
        pages.metricsView(ctx, st, { now: 0, pager: { sort: pick(r, ['power', 'name', 'in-use']) } });
        pages.nodesView(ctx, { metrics: m, now: 0 });
        pages.podsView(ctx, { metrics: m, now: 0 });
      }
      pages.clearViewMemo();
    }
  });
});

describe('clusterPowerStats', () => {
  // The per-step sum as a plain object keyed by step (integer keys iterate in
  // ascending order): the definition the faster implementation must match.
  function oracle(byNode) {
    const total = {};
    for (const n in byNode) {
      for (const [t, v] of byNode[n]) if (typeof v === 'number' && isFinite(v)) total[t] = (total[t] || 0) + v;
    }
    const ts = Object.keys(total);
    if (!ts.length) return null;
    let peak = -Infinity;
    let peakAt = 0;
    let sum = 0;
    for (const t of ts) {
      sum += total[t];
      if (total[t] > peak) {
        peak = total[t];
        peakAt = Number(t);
      }
    }
    return { peakWatts: peak, peakAt: peakAt, avgWatts: sum / ts.length, steps: ts.length };
  }

  it('equals the per-step sum over nodes, for one series and for several, with gaps and non-numbers', () => {
    const r = rng(2026);
    let compared = 0;
    for (let round = 0; round < 400; round++) {
      const byNode = {};
      const nodes = int(r, 1, 3);
      for (let n = 0; n < nodes; n++) {
        const pts = [];
        const start = 1760000000 + 15 * int(r, 0, 4);
        const len = int(r, 0, 40);
        for (let i = 0; i < len; i++) {
          if (r() < 0.2) continue; // a missing step
          pts.push([start + 15 * i, pick(r, [int(r, 0, 1400), int(r, 0, 1400) + 0.5, 700, 700, NaN, null, Infinity, '5'])]);
        }
        byNode['n' + n] = pts;
      }
      const got = clusterPowerStats(byNode);
      const want = oracle(byNode);
      if (want === null) expect(got).toBeNull();
      else {
        expect(got.peakWatts).toBe(want.peakWatts);
        expect(got.peakAt).toBe(want.peakAt);
        expect(got.steps).toBe(want.steps);
        expect(Math.abs(got.avgWatts - want.avgWatts)).toBeLessThan(1e-9 * Math.max(1, Math.abs(want.avgWatts)));
        compared++;
      }
    }
    expect(compared).toBeGreaterThan(300);
  });
});

describe('formatters', () => {
  it('formatWatts writes what toFixed(1) writes, and formatBytes trims as the regex /\\.?0+$/ does', () => {
    const r = rng(355);
    const xs = [0, -0, 1, -3, 0.05, 0.15, 2.5, 1023.95, 2 ** 53, 2 ** 53 + 2, -(2 ** 53), 1e21, 294896 * 1048576];
    for (let i = 0; i < 5000; i++) {
      xs.push(r() * Math.pow(2, r() * 70), Math.round(r() * Math.pow(2, r() * 70)), Math.round(r() * 30000) / 10, -r() * 100);
    }
    const units = ['B', 'KiB', 'MiB', 'GiB', 'TiB', 'PiB'];
    function bytesOracle(b) {
      let v = b;
      let u = 0;
      while (v >= 1024 && u < units.length - 1) {
        v /= 1024;
        u++;
      }
      const digits = v >= 100 || u === 0 ? 0 : v >= 10 ? 1 : 2;
      const t = v.toFixed(digits);
      return (digits > 0 ? t.replace(/\.?0+$/, '') : t) + ' ' + units[u];
    }
    for (const x of xs) {
      expect(formatWatts(x)).toBe(x.toFixed(1) + ' W');
      if (x >= 0) expect(formatBytes(x)).toBe(bytesOracle(x));
    }
  });
});
