/**
 * Native detail pages opened on a warm cluster (a plugin page loaded
 * before): Pod detail and Node detail each fetch their node's telemetry with
 * a hostname-scoped query on a fresh metrics client, next to the
 * cluster-wide snapshot the pod detail would otherwise need; Node detail on a
 * cold store; the reference's provider for the same open; and the GPU Pods
 * page with its attribution-only query. Driver command 'detail'.
 */
import { fetchNodePods } from '../src/api/clusterStore.js';
import { createMetricsSource } from '../src/api/metrics.js';
import { filterGpuRequestingPods } from '../src/api/amdPods.js';
import { nodeDetailView, podDetailView } from '../src/view/pages/details.js';
import { ownersScope, podsView } from '../src/view/pages/pods.js';
import { renderPage, renderSection } from '../src/view/html.js';
import { createReferenceSchedule } from './referenceSchedule.js';
import { hiResClock, makeRequest, ms } from './common.js';
import { PAGER } from './pageRender.js';
import { wiredNodeDetailOpen } from './wiredDetail.js';

/** Opens per wired mode: the 'after a page' mode downloads that page's lists first (untimed). */
const WIRED_OPENS = 3;

/**
 * `n` opens of each mode over the pods of `ctx` (a warm store's snapshot).
 * @returns {{detail: Object, detailSlow: Array}}
 */
export async function detailOpens(url, counter, ctx, n) {
  const out = {};
  const pods = ctx.gpuPods.filter(function (p) { return p.spec && p.spec.nodeName; });
  const MODES = ['podScoped', 'podDetail', 'podClusterWide', 'nodeScoped', 'nodeDetail', 'nodeDetailCold',
    'nodeDetailColdReference', 'podsPageOwners'];
  const modes = {};
  const bytes = {};
  const reqs = {};
  MODES.forEach(function (k) { modes[k] = []; bytes[k] = 0; reqs[k] = 0; });
  const slow = [];
  // Each mode's own request function and counter: a request still in flight
  // when its open ends (the reference's 2 s-capped requests on a 1,000-node
  // cluster) lands its bytes on the mode that sent it, not on whichever open
  // it completes during.
  const own = {};
  const reqOf = {};
  MODES.forEach(function (k) {
    own[k] = { n: 0, bytes: 0 };
    reqOf[k] = makeRequest(url, own[k]);
  });
  for (let i = 0; i < n && pods.length; i++) {
    const pod = pods[i % pods.length];
    const node = ctx.gpuNodes.filter(function (x) { return x.metadata.name === pod.spec.nodeName; })[0];
    const runs = [
      ['podScoped', function (src) { return src.fetchNodeMetrics(pod.spec.nodeName).then(function (m) { return podDetailView(pod, { metrics: m }); }); }],
      // As src/plugin.js wires the Pod detail page: the node's telemetry
      // and the pod's power history, in one wave.
      ['podDetail', function (src) {
        return Promise.all([
          src.fetchNodeMetrics(pod.spec.nodeName),
          src.fetchPodSeries(pod.metadata.namespace || '', pod.metadata.name, 1800, 30),
        ]).then(function (r) { return podDetailView(pod, { metrics: r[0], series: r[1] }); });
      }],
      ['podClusterWide', function (src) { return src.fetchGpuMetrics().then(function (m) { return podDetailView(pod, { metrics: m }); }); }],
      ['nodeScoped', function (src) {
        return src.fetchNodeMetrics(pod.spec.nodeName).then(function (m) { return node ? nodeDetailView(node, ctx, { metrics: m }) : null; });
      }],
      // As src/plugin.js wires the Node detail page: telemetry + power history in one wave.
      ['nodeDetail', function (src) {
        return Promise.all([src.fetchNodeMetrics(pod.spec.nodeName), src.fetchNodeSeries(pod.spec.nodeName, 1800, 30)])
          .then(function (r) { return node ? nodeDetailView(node, ctx, { metrics: r[0], series: r[1] }) : null; });
      }],
      // Node detail on a COLD store (no plugin page visited), as
      // src/plugin.js NodeDetailCold wires it: the node's pods by the list
      // request of its node-scoped list + watch (fieldSelector
      // spec.nodeName=…; the watch then keeps it live), its telemetry and
      // history, one wave.
      ['nodeDetailCold', function (src) {
        const nm = pod.spec.nodeName;
        return Promise.all([fetchNodePods(reqOf.nodeDetailCold, nm), src.fetchNodeMetrics(nm), src.fetchNodeSeries(nm, 1800, 30)])
          .then(function (r) {
            const cold = { loading: false, gpuPods: filterGpuRequestingPods(r[0]), podsState: 'ready', error: null };
            return node ? nodeDetailView(node, cold, { metrics: r[1], series: r[2] }) : null;
          });
      }],
      // The reference on the same open: a full provider (both
      // cluster-wide lists alongside CRD + 3 serial selector requests,
      // src/index.tsx:152-160), then its section from that context.
      ['nodeDetailColdReference', function () {
        const ref = createReferenceSchedule(reqOf.nodeDetailColdReference);
        return ref.coldOpenPage('nodes').then(function () { return node ? nodeDetailView(node, ref.snapshot()) : null; });
      }],
      // GPU Pods page: pod → GPU attribution of its first page of pods only.
      ['podsPageOwners', function (src) {
        const o = ownersScope(ctx, PAGER);
        return src.fetchGpuOwners(o.pods === undefined ? undefined : { pods: o.pods }).then(function (m) {
          renderPage(podsView(ctx, { metrics: m, pager: PAGER }));
          return null;
        });
      }],
    ];
    for (let r = 0; r < runs.length; r++) {
      const spans = [];
      // A fresh metrics client (cold cache) per open, over the page's
      // connection pool: a browser keeps its keep-alive sockets to the
      // Headlamp origin across in-app navigations.
      const src = createMetricsSource({
        request: reqOf[runs[r][0]], clock: hiResClock, onTrace: function (sp) { spans.push(sp); },
      });
      const t0 = process.hrtime();
      const start = hiResClock.now();
      const s = await runs[r][1](src);
      if (s) renderSection(s);
      const took = ms(process.hrtime(t0));
      modes[runs[r][0]].push(took);
      // Opens far above the injected RTT: where the time went (request spans vs client work).
      if (took > 80) {
        slow.push({ mode: runs[r][0], i: i, ms: took, spans: spans.map(function (sp) {
          return { name: sp.name, startMs: sp.start - start, durMs: sp.end - sp.start, ok: sp.ok };
        }) });
      }
    }
  }
  MODES.forEach(function (k) {
    bytes[k] = own[k].bytes;
    reqs[k] = own[k].n;
    counter.n += own[k].n;
    counter.bytes += own[k].bytes;
  });
  out.detail = {};
  out.detailSlow = slow;
  for (const k in modes) {
    out.detail[k] = { latencies: modes[k], bytesPerOpen: bytes[k] / Math.max(1, modes[k].length), requestsPerOpen: reqs[k] / Math.max(1, modes[k].length) };
  }
  // The Node detail section through the plugin's own wiring (bench/wiredDetail.js):
  // after GPU Nodes was visited and unmounted, and on a cold start. Its list
  // hooks are counted next to its requests and bytes.
  const wired = [['nodeDetailWired', 'nodes'], ['nodeDetailWiredCold', null]];
  for (let w = 0; w < wired.length; w++) {
    const runs = [];
    for (let i = 0; i < Math.min(n, WIRED_OPENS) && pods.length; i++) {
      const pod = pods[i % pods.length];
      const node = ctx.gpuNodes.filter(function (x) { return x.metadata.name === pod.spec.nodeName; })[0];
      if (node) runs.push(await wiredNodeDetailOpen(url, node, wired[w][1], wired[w][0] + '-' + i));
    }
    const k = runs.length || 1;
    const sum = function (f) { return runs.reduce(function (a, r) { return a + f(r); }, 0) / k; };
    out.detail[wired[w][0]] = {
      latencies: runs.map(function (r) { return r.ms; }),
      bytesPerOpen: sum(function (r) { return r.bytes; }),
      requestsPerOpen: sum(function (r) { return r.requests; }),
      listsPerOpen: sum(function (r) { return r.lists.length; }),
      clusterWideListsPerOpen: sum(function (r) { return r.clusterWideLists; }),
      deviceConfigRequestsPerOpen: sum(function (r) { return r.deviceConfigRequests; }),
      serverMs: runs.map(function (r) { return r.serverMs; }),
      listPaths: runs.length ? runs[runs.length - 1].lists : [],
      rendered: runs.every(function (r) { return r.section && !r.loading; }),
    };
  }
  return out;
}
