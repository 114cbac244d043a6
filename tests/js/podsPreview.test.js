/**
 * The GPU Pods page before the pod list is in (ADR 013): the owner query's
 * preview branch (promql.js ownersQuery), its answer (ownerSnapshots.js) and
 * the partial page (pods.js podsPreview / podsView).
 */
import { createMetricsSource } from '../../src/api/metrics.js';
import { ownersQuery } from '../../src/api/promql.js';
import { SERIES, SMALL_CLUSTER_PODS } from '../../src/api/series.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { ownersScope, podsPreview, podsView } from '../../src/view/pages/pods.js';
import { PODS_PER_PAGE } from '../../src/view/pages/paging.js';
import { sectionTitles } from '../../src/view/ir.js';
import { renderPage } from '../../src/view/html.js';
import { ok, vec } from './promFake.js';

const E = SERIES.exporter;

function owner(ns, pod, node, gpu, w) {
  return vec({ __name__: E.power, namespace: ns, pod: pod, hostname: node, gpu_id: String(gpu) }, w);
}

/** A pending pod list: what the GPU Pods page sees on a cold open. */
const PENDING = { podsState: 'pending', podsLoading: true, nodesState: 'ready', nodesLoading: false, gpuPods: [], loading: true };

beforeEach(() => clearViewMemo());

describe('ownersScope before the pod list', () => {
  it('asks the small owner query with a preview of one page', () => {
    expect(ownersScope(PENDING, { page: 0, filter: '' })).toEqual({ enabled: true, pods: [], small: true, preview: PODS_PER_PAGE });
  });
  it('the preview branch is a power ranking guarded to clusters of more than one page of owners', () => {
    const q = ownersQuery([], true, 25);
    expect(q).toContain('topk(25, sum by (namespace, pod)');
    expect(q).toContain('> ' + SMALL_CLUSTER_PODS);
    expect(q).toContain('"agg", "rank"');
    // a page of pods asked: no preview
    expect(ownersQuery(['ml/a'], true, 25)).not.toContain('topk(');
    expect(ownersQuery([], true)).not.toContain('topk(');
  });
});

describe('the preview answer (ownerSnapshots.js)', () => {
  it('large cluster: the ranked pods, their watts and the owner count', async () => {
    const asked = [];
    const request = (path) => {
      asked.push(decodeURIComponent(path));
      if (path.indexOf('query=1') >= 0) return Promise.resolve(ok([]));
      return Promise.resolve(ok([
        owner('ml', 'big', 'n1', 0, 700), owner('ml', 'big', 'n1', 1, 700), owner('ml', 'mid', 'n2', 0, 500),
        vec({ namespace: 'ml', pod: 'big', agg: 'rank' }, 1400), vec({ namespace: 'ml', pod: 'mid', agg: 'rank' }, 500),
        vec({ agg: 'gpu_pods' }, 300),
      ]));
    };
    const m = await createMetricsSource({ request }).fetchGpuOwners({ pods: [], small: true, preview: 25 });
    expect(asked.some((p) => p.indexOf('topk(25,') >= 0)).toBe(true);
    expect(m.small).toEqual({ count: 300, limit: SMALL_CLUSTER_PODS, exceeded: true });
    expect(m.preview.order).toEqual(['ml/big', 'ml/mid']);
    expect(m.preview.count).toBe(300);
    expect(m.preview.watts['ml/big']).toBe(1400);
    expect(m.gpus.filter((g) => g.pod === 'big')).toHaveLength(2);
  });

  it('small cluster: every owner, no preview ranking', async () => {
    const request = () => Promise.resolve(ok([owner('ml', 'a', 'n1', 0, 300), vec({ agg: 'gpu_pods' }, 1)]));
    const m = await createMetricsSource({ request }).fetchGpuOwners({ pods: [], small: true, preview: 25 });
    expect(m.small.exceeded).toBe(false);
    expect(m.preview).toBeUndefined();
  });
});

describe('podsPreview / podsView with the pod list pending', () => {
  function metrics(gpus, preview) {
    return { gpus: gpus, xgmi: {}, links: {}, scope: 'owners', preview: preview };
  }
  function g(ns, pod, node, gpu, w) {
    return { namespace: ns, pod: pod, nodeName: node, gpu: String(gpu), powerWatts: w };
  }

  it('nothing to show without an owner answer: the loader', () => {
    expect(podsPreview(null)).toBeNull();
    expect(podsPreview(metrics([g('', '', 'n1', 0, 100)].filter((x) => x.pod)))).toBeNull();
    const vm = podsView(PENDING, { metrics: null });
    expect(renderPage(vm)).toContain('Loading GPU pod data...');
  });

  it('small cluster: every owner in namespace / name order, marked partial, with GPUs held', () => {
    const m = metrics([g('ml', 'b', 'n1', 0, 300), g('ml', 'a', 'n1', 1, 200), g('ml', 'a', 'n2', 0, 200), g('', null, 'n2', 1, 90)]);
    const vm = podsView(PENDING, { metrics: m });
    const html = renderPage(vm);
    expect(sectionTitles(vm)).toEqual(['Summary (partial)', 'GPU Pods (partial)']);
    expect(html).toContain('Partial — the pod list is loading');
    expect(html.indexOf('>a<')).toBeLessThan(html.indexOf('>b<'));
    expect(html).toContain('n1, n2');
    expect(html).toContain('2 GPUs held');
    expect(html).toContain('400.0 W');
    expect(html).not.toContain('Loading GPU pod data...');
  });

  it('the Phase cell says what the exporter knows (the pod holds GPUs), not Running', () => {
    // Devices are bound at admission: a pod in ContainerCreating (Pending) is attributed too.
    const vm = podsView(PENDING, { metrics: metrics([g('ml', 'starting', 'n1', 0, 0)]) });
    const t = vm.items[1].blocks[0];
    expect(t.rows[0][t.columns.indexOf('Phase')]).toBe('Holds GPUs');
    expect(renderPage(vm)).not.toContain('Running');
  });

  it('large cluster: the ranked pods in power order, out of every pod holding a GPU', () => {
    const m = metrics([g('ml', 'low', 'n1', 0, 100), g('ml', 'high', 'n2', 0, 700)],
      { per: 25, count: 4000, order: ['ml/high', 'ml/low'], watts: { 'ml/high': 700, 'ml/low': 100 } });
    const vm = podsView(PENDING, { metrics: m });
    const html = renderPage(vm);
    expect(sectionTitles(vm)).toEqual(['Summary (partial)', 'GPU Pods Drawing the Most Power (partial)']);
    expect(html).toContain('4000');
    expect(html.indexOf('>high<')).toBeLessThan(html.indexOf('>low<'));
  });

  it('the pod list in: the partial sections give way to the full page', () => {
    const m = metrics([g('ml', 'a', 'n1', 0, 200)]);
    const ready = { podsState: 'ready', podsLoading: false, nodesState: 'ready', nodesLoading: false, gpuPods: [], loading: false,
      index: { phases: { Running: 0, Pending: 0, Failed: 0 }, totals: { heldGpus: 0 } } };
    expect(sectionTitles(podsView(ready, { metrics: m }))).toEqual(['No GPU Pods Found']);
  });
});

describe('Overview before the pod list (overview.js overviewOwnersScope / overviewPodsPreview)', () => {
  const nodesOf = (n) => Array.from({ length: n }, (_, i) => ({ metadata: { name: 'n' + i } }));
  const base = { nodesState: 'ready', podsState: 'pending', podsLoading: true, nodesLoading: false };

  it('asks the exporter only on a cluster of more than one page of GPU nodes, and only while its pod list loads', async () => {
    const { overviewOwnersScope, ACTIVE_PODS_LIMIT } = await import('../../src/view/pages/overview.js');
    const { SMALL_CLUSTER_NODES: per } = await import('../../src/api/series.js');
    expect(overviewOwnersScope(Object.assign({}, base, { gpuNodes: nodesOf(per) })).enabled).toBe(false);
    expect(overviewOwnersScope(Object.assign({}, base, { gpuNodes: nodesOf(per + 1) })))
      .toEqual({ enabled: true, pods: [], small: true, preview: ACTIVE_PODS_LIMIT });
    expect(overviewOwnersScope(Object.assign({}, base, { gpuNodes: nodesOf(per + 1), podsState: 'ready', podsLoading: false })).enabled).toBe(false);
    expect(overviewOwnersScope(Object.assign({}, base, { gpuNodes: [], nodesState: 'pending' })).enabled).toBe(false);
    expect(overviewOwnersScope(null).enabled).toBe(false);
  });

  it('the ranked owners, at most ACTIVE_PODS_LIMIT, with their GPUs and power; nothing without owners', async () => {
    const { overviewPodsPreview, ACTIVE_PODS_LIMIT } = await import('../../src/view/pages/overview.js');
    const gpus = [];
    const order = [];
    for (let i = 0; i < 12; i++) {
      gpus.push({ namespace: 'ml', pod: 'p' + i, nodeName: 'n' + i, gpu: '0', powerWatts: 100 + i });
      order.push('ml/p' + (11 - i));
    }
    const s = overviewPodsPreview({ gpus: gpus, preview: { per: ACTIVE_PODS_LIMIT, count: 300, order: order, watts: {} } });
    expect(s.title).toBe('GPU Pods Drawing the Most Power (partial)');
    const t = s.blocks[1];
    expect(t.rows).toHaveLength(ACTIVE_PODS_LIMIT);
    expect(t.rows[0]).toEqual(['p11', 'ml', 'n11: GPU 0', '111.0 W']);
    expect(s.blocks[0].rows[1]).toEqual({ name: 'Pods Holding GPUs', value: '300' });
    expect(overviewPodsPreview({ gpus: [{ namespace: '', pod: null, nodeName: 'n0', gpu: '0' }] })).toBeNull();
    expect(overviewPodsPreview(null)).toBeNull();
  });
});
