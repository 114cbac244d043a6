/**
 * The reference's pages and this plugin's, each page mounted on real React
 * 18.3.1 (production builds) from the same synthetic cluster (see
 * ./referenceRender.js). Reference: mount with its data (its per-render
 * aggregation included), re-render on a watch event (a new context value:
 * new arrays of the same objects), and the provider's per-event filtering of
 * the whole lists (IntelGpuDataContext.tsx:200-208) apart. This plugin: mount
 * including the view-model built from a cold memo, re-render on the same
 * watch event (a new snapshot of the same data), first page of each pager.
 * Driven by tools/render_compare.py (driver command 'refRender').
 */
import { createMetricsSource } from '../src/api/metrics.js';
import { clearViewMemo } from '../src/view/pages/common.js';
import { loadReferencePages, referenceContext, toGpuMetrics, toIntelNode, toIntelPod } from './referenceRender.js';
import { amdSchedule } from './schedules.js';
import { makeRequest, ms, stats } from './common.js';
import { PAGES, pageVm } from './pageRender.js';
import { mountCycle, realReact } from './reactMount.js';

/** The header each reference page shows once its data is in (its Loader gone). */
const REFERENCE_TITLES = {
  overview: 'Intel GPU — Overview', devicePlugins: 'Intel GPU — Device Plugins', nodes: 'Intel GPU — Nodes',
  pods: 'Intel GPU — Pods', metrics: 'Intel GPU — Metrics',
};

export async function compareRenders(url, c) {
  const R = await realReact(c.umdDir);
  const ref = loadReferencePages(c.referenceDir, R.React, R.CC);
  const reps = c.reps || 5;
  // (no 2 s request limit: the fake Prometheus evaluates 8,000 GPUs in Python on this host)
  const s = amdSchedule(makeRequest(url, { n: 0, bytes: 0 }), null, 600000);
  await s.coldOpen();
  const request = makeRequest(url, { n: 0, bytes: 0 });
  // Every GPU's gauges for the reference's one-card-per-chip Metrics page (the
  // fake Prometheus needs seconds for 8,000 GPUs: no 2 s request timeout here).
  const every = await createMetricsSource({ request: request, timeoutMs: 600000 }).fetchGpuMetrics('gauges');
  if (!every) throw new Error('compareRenders: no telemetry');
  const lists = await Promise.all([request('/api/v1/nodes'), request('/api/v1/pods')]);
  const snap = s.ctx();
  const t0 = process.hrtime();
  const refCtx = referenceContext(ref.k8s, {
    nodes: lists[0].items, pods: lists[1].items, deviceConfigs: snap.deviceConfigs, pluginPods: snap.pluginPods,
  });
  const deriveMs = ms(process.hrtime(t0));
  // the provider's useMemo filters, per watch event (the lists already in the reference's shapes)
  const intelNodes = lists[0].items.map(toIntelNode);
  const intelPods = lists[1].items.map(toIntelPod);
  const d0 = process.hrtime();
  ref.k8s.filterIntelGpuNodes(intelNodes);
  ref.k8s.filterGpuRequestingPods(intelPods);
  const filterMs = ms(process.hrtime(d0));
  const refMetrics = toGpuMetrics(every);
  const out = { pages: {}, referenceProviderFilterMs: filterMs, referenceContextBuildMs: deriveMs,
    gpuNodes: refCtx.gpuNodes.length, gpuPods: refCtx.gpuPods.length, chips: refMetrics.chips.length };
  for (let p = 0; p < PAGES.length; p++) {
    const page = PAGES[p];
    ref.setData(refCtx, refMetrics);
    const reference = await mountCycle(R, function () { return R.React.createElement(ref.pages[page]); },
      page === 'metrics' ? 'GPU Power Summary' : null, function () {
        ref.setData(Object.assign({}, refCtx, {
          gpuNodes: refCtx.gpuNodes.slice(), gpuPods: refCtx.gpuPods.slice(), pluginPods: refCtx.pluginPods.slice(),
          devicePlugins: refCtx.devicePlugins.slice(),
        }), refMetrics);
      }, reps, REFERENCE_TITLES[page]);
    const mstatePage = page === 'metrics' ? s.pageMstate() : s.mstate();
    let ctx = snap;
    const amd = await mountCycle(R, function () {
      return R.React.createElement(R.view.Page, { vm: pageVm(page, ctx, mstatePage, s.pageMetrics(page)) });
    }, null, function () { ctx = Object.assign({}, snap); }, 1);
    // mount from a cold view memo each rep (the first page render of a session)
    const colds = [];
    for (let i = 0; i < reps; i++) {
      clearViewMemo();
      ctx = snap;
      colds.push(await mountCycle(R, function () {
        return R.React.createElement(R.view.Page, { vm: pageVm(page, ctx, mstatePage, s.pageMetrics(page)) });
      }, null, function () { ctx = Object.assign({}, snap); }, 1));
    }
    out.pages[page] = {
      reference: reference,
      amd: { mountMs: stats(colds.map(function (x) { return x.mountMs; })).p50,
        rerenderMs: stats(colds.map(function (x) { return x.rerenderMs; })).p50, elements: amd.elements, reps: reps },
    };
  }
  return out;
}
