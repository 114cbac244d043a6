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
 *
 * The reference's pages run in bench/refWorker.cjs's realm, in the process
 * ./refIsolated.js starts without network or writes; this process only sends
 * it text and reads back its timings (ADR 014). Both realms mount the same
 * calibration tree, so the two environments' React speed is on record.
 */
import { createMetricsSource } from '../src/api/metrics.js';
import { clearViewMemo } from '../src/view/pages/common.js';
import { referenceData } from './referenceRender.js';
import { referenceWorker } from './refIsolated.js';
import { amdSchedule } from './schedules.js';
import { makeRequest, ms, stats } from './common.js';
import { PAGES, pageVm } from './pageRender.js';
import { mountCycle, realReact } from './reactMount.js';

/** Rows of the calibration table both realms mount (bench/refWorker.cjs `calibrate`). */
const CALIBRATION_ROWS = 100;

/** The calibration tree mounted in this realm, as the worker's realm does (ms per mount). */
function calibrateHere(R, reps) {
  const h = R.React.createElement;
  const times = [];
  let elements = 0;
  for (let i = 0; i < reps; i++) {
    const t0 = process.hrtime();
    const trs = [];
    for (let k = 0; k < CALIBRATION_ROWS; k++) trs.push(h('tr', { key: k }, h('td', null, 'node-' + k), h('td', null, String(k * 7))));
    const c = document.createElement('div');
    document.body.appendChild(c);
    const root = R.ReactDOM.createRoot(c);
    R.ReactDOM.flushSync(function () { root.render(h('table', null, h('tbody', null, trs))); });
    elements = c.querySelectorAll('*').length;
    R.ReactDOM.flushSync(function () { root.unmount(); });
    document.body.removeChild(c);
    times.push(ms(process.hrtime(t0)));
  }
  return { times: times, elements: elements };
}

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
 * content. This process runs none of them; it starts the worker that does,
 * without network or writes, in a realm of their own (./refIsolated.js,
 * ./refWorker.cjs; ADR 014).
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
  const ref = await referenceWorker(c.referenceDir, c.umdDir);
  try {
    return await measure(url, c, R, ref);
  } finally {
    await ref.close();
  }
}

async function measure(url, c, R, ref) {
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
  const refInfo = await ref.call('setData', {
    json: referenceData({ nodes: lists[0].items, pods: lists[1].items, deviceConfigs: snap.deviceConfigs, pluginPods: snap.pluginPods }, every),
  });
  // the provider's useMemo filters, per watch event (the lists already in the reference's shapes)
  const filterMs = await ref.call('filter');
  const calReps = Math.max(31, warm);
  const calRef = await ref.call('calibrate', { rows: CALIBRATION_ROWS, reps: calReps });
  const calHere = calibrateHere(R, calReps);
  const out = { pages: {}, referenceProviderFilterMs: filterMs, referenceContextBuildMs: refInfo.contextBuildMs,
    gpuNodes: refInfo.gpuNodes, gpuPods: refInfo.gpuPods, chips: refInfo.chips, reps: reps, warm: warm,
    calibration: { rows: CALIBRATION_ROWS, elements: calHere.elements, referenceRealmMs: spread(calRef.times.slice(5)).p50,
      driverRealmMs: spread(calHere.times.slice(5)).p50 } };
  const pages = Array.isArray(c.pages) && c.pages.length ? PAGES.filter(function (x) { return c.pages.indexOf(x) >= 0; }) : PAGES;
  for (let p = 0; p < pages.length; p++) {
    const page = pages[p];
    const mstatePage = page === 'metrics' ? s.pageMstate() : s.mstate();
    let ctx = snap;
    function referenceOnce() {
      return ref.call('cycle', { page: page, waitText: page === 'metrics' ? 'GPU Power Summary' : null, mustShow: REFERENCE_TITLES[page] })
        .then(function (r) { return { mounts: [r.mount], rerenders: [r.rerender], elements: r.elements }; });
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
