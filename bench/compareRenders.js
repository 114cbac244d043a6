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

/** The V8 flag the opt-in comparison's process must run with (no host Function constructor compiles code). */
export const NO_CODEGEN_FLAG = '--disallow-code-generation-from-strings';

/**
 * Refuses unless the caller opted in (`allowReferenceExec`) and this process
 * runs with NO_CODEGEN_FLAG: the reference's sources are untrusted public
 * content, run only in bench/tsx.js's sandbox under that flag (ADR 014).
 */
export function assertReferenceSandbox(c) {
  if (!c || c.allowReferenceExec !== true) {
    throw new Error('refRender runs the reference\'s sources: opt in with tools/render_compare.py --allow-reference-exec');
  }
  if (process.execArgv.indexOf(NO_CODEGEN_FLAG) < 0) {
    throw new Error('refRender needs a process started with ' + NO_CODEGEN_FLAG + ' (tools/render_compare.py does this)');
  }
}

/** p50 and interquartile range of a sample (ms). */
function spread(xs) {
  const st = stats(xs);
  const q = function (p) {
    const v = xs.slice().sort(function (a, b) { return a - b; });
    const idx = (v.length - 1) * p;
    const lo = Math.floor(idx);
    const hi = Math.ceil(idx);
    return v[lo] + (v[hi] - v[lo]) * (idx - lo);
  };
  return { p50: st.p50, q1: q(0.25), q3: q(0.75) };
}

function summary(x) {
  const m = spread(x.mount);
  const r = spread(x.rerender);
  return {
    elements: x.elements, reps: x.mount.length,
    mountMs: m.p50, mountQ1: m.q1, mountQ3: m.q3, rerenderMs: r.p50, rerenderQ1: r.q1, rerenderQ3: r.q3,
  };
}

export async function compareRenders(url, c) {
  assertReferenceSandbox(c);
  const R = await realReact(c.umdDir);
  const ref = loadReferencePages(c.referenceDir, R.React, R.CC);
  const reps = Math.max(15, c.reps || 15);
  const warm = c.warm === undefined ? 5 : c.warm;
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
    gpuNodes: refCtx.gpuNodes.length, gpuPods: refCtx.gpuPods.length, chips: refMetrics.chips.length, reps: reps, warm: warm };
  const refEvent = function () {
    ref.setData(Object.assign({}, refCtx, {
      gpuNodes: refCtx.gpuNodes.slice(), gpuPods: refCtx.gpuPods.slice(), pluginPods: refCtx.pluginPods.slice(),
      devicePlugins: refCtx.devicePlugins.slice(),
    }), refMetrics);
  };
  for (let p = 0; p < PAGES.length; p++) {
    const page = PAGES[p];
    const mstatePage = page === 'metrics' ? s.pageMstate() : s.mstate();
    let ctx = snap;
    function referenceOnce() {
      ref.setData(refCtx, refMetrics);
      return mountCycle(R, function () { return R.React.createElement(ref.pages[page]); },
        page === 'metrics' ? 'GPU Power Summary' : null, refEvent, 1, REFERENCE_TITLES[page]);
    }
    // Mount from a cold view memo each time (the first page render of a session).
    function amdOnce() {
      clearViewMemo();
      ctx = snap;
      return mountCycle(R, function () {
        return R.React.createElement(R.view.Page, { vm: pageVm(page, ctx, mstatePage, s.pageMetrics(page)) });
      }, null, function () { ctx = Object.assign({}, snap); }, 1);
    }
    // The same page with its view-model built before the timed mount: the
    // React side of the figure alone (diagnostic; `vmMs` is the build).
    function amdPrebuiltOnce() {
      clearViewMemo();
      const t0 = process.hrtime();
      const vm = pageVm(page, snap, mstatePage, s.pageMetrics(page));
      const vmMs = ms(process.hrtime(t0));
      return mountCycle(R, function () { return R.React.createElement(R.view.Page, { vm: vm }); }, null, null, 1)
        .then(function (r) { return Object.assign(r, { vmMs: vmMs }); });
    }
    // Untimed warm mounts of both (JIT, first-use caches), then `reps`
    // interleaved pairs, the order alternating, so drift and noise land on both.
    for (let i = 0; i < warm; i++) {
      await referenceOnce();
      await amdOnce();
    }
    const prebuilt = { mount: [], vm: [] };
    const samples = { reference: { mount: [], rerender: [], elements: 0 }, amd: { mount: [], rerender: [], elements: 0 } };
    for (let i = 0; i < reps; i++) {
      const order = i % 2 === 0 ? ['reference', 'amd'] : ['amd', 'reference'];
      for (let k = 0; k < 2; k++) {
        const r = await (order[k] === 'reference' ? referenceOnce() : amdOnce());
        samples[order[k]].mount.push(r.mounts[0]);
        samples[order[k]].rerender.push(r.rerenders[0]);
        samples[order[k]].elements = r.elements;
      }
      const pb = await amdPrebuiltOnce();
      prebuilt.mount.push(pb.mounts[0]);
      prebuilt.vm.push(pb.vmMs);
    }
    out.pages[page] = {
      reference: summary(samples.reference),
      amd: Object.assign(summary(samples.amd), { reactOnlyMs: spread(prebuilt.mount).p50, vmBuildMs: spread(prebuilt.vm).p50 }),
      // The samples themselves, so runs in several processes can be pooled (tools/render_compare.py --runs).
      samples: { reference: samples.reference, amd: samples.amd, prebuilt: prebuilt },
    };
  }
  return out;
}
