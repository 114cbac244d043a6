#!/usr/bin/env node
/**
 * Dashboard-refresh benchmark driver (runs the SHIPPED plugin data layer).
 *
 *   node bench/driver.js --url http://127.0.0.1:PORT --steps K --warmup W \
 *        [--cold N] [--out result.json] [--schedule amd|reference|both]
 *
 * Talks HTTP to the fake control plane (headlamp_intel_gpu_plugin_amd.sim)
 * through a keep-alive agent capped at 6 sockets — the per-origin HTTP/1.1
 * connection limit of the browser Headlamp runs in.
 *
 * For each schedule it measures, in wall-clock ms:
 *   refresh     warm page; Refresh clicked → every dashboard page's data
 *               (DeviceConfigs, operator pods, GPU telemetry; for the amd
 *               schedule also the power/HBM time series) committed and all
 *               five page view-models + node/pod detail sections + Nodes-table
 *               columns rebuilt and rendered to HTML;
 *   cold        route mount on an empty cache (node + pod lists included);
 *   switch      navigating to another plugin route after the first load
 *               (shared store: cached render + background revalidate; the
 *               reference mounts a fresh provider, i.e. a cold open).
 * and the rows each view renders.
 */

import http from 'http';
import fs from 'fs';
import path from 'path';
import { createClusterStore, fetchNodePods } from '../src/api/clusterStore.js';
import { createMetricsSource } from '../src/api/metrics.js';
import { filterGpuRequestingPods } from '../src/api/amdgpu.js';
import {
  overviewView, devicePluginsView, nodesView, podsView, metricsView,
  nodeDetailView, podDetailView, nodeColumns, nodePage, ownersScope, podPage, telemetryScope, clearViewMemo,
} from '../src/view/pages.js';
import { countRows, sections } from '../src/view/ir.js';
import { renderPage, renderSection } from '../src/view/html.js';
import { createReferenceSchedule } from './referenceSchedule.js';
import { PAGE_NEEDS } from '../src/plugin.js';
import { loadReferencePages, referenceContext, toGpuMetrics, toIntelNode, toIntelPod } from './referenceRender.js';
// The harness React (the Node-12 stand-in the spec suite renders the plugin
// with) and its CommonComponents: the pages are also mounted through the
// shipped renderer (src/view/react.js) to count elements and time a
// mount / re-render, next to the IR → HTML figure.
import * as HarnessReact from '../tests/js/stubs/react.js';
import * as HarnessCC from '../tests/js/stubs/CommonComponents.js';
import { createRenderer } from '../src/view/react.js';
import { PerformanceObserver, performance } from 'perf_hooks';

// Garbage-collection pauses (start, duration in ms, performance.now() clock),
// so a timed sample can say how much of it was the collector.
const gcPauses = [];
try {
  new PerformanceObserver(function (list) {
    list.getEntries().forEach(function (e) { gcPauses.push([e.startTime, e.duration]); });
    if (gcPauses.length > 4096) gcPauses.splice(0, gcPauses.length - 4096);
  }).observe({ entryTypes: ['gc'] });
} catch (e) {
  // no GC entries on this runtime
}

/** GC pause time (ms) that started inside [from, to] (performance.now() clock). */
function gcBetween(from, to) {
  let t = 0;
  for (let i = 0; i < gcPauses.length; i++) if (gcPauses[i][0] >= from && gcPauses[i][0] <= to) t += gcPauses[i][1];
  return t;
}

function parseArgs(argv) {
  const a = { url: null, steps: 20, warmup: 3, cold: 5, out: null, schedule: 'both' };
  for (let i = 0; i < argv.length; i++) {
    const k = argv[i];
    const v = argv[i + 1];
    if (k === '--url') a.url = v;
    else if (k === '--steps') a.steps = parseInt(v, 10);
    else if (k === '--warmup') a.warmup = parseInt(v, 10);
    else if (k === '--cold') a.cold = parseInt(v, 10);
    else if (k === '--out') a.out = v;
    else if (k === '--schedule') a.schedule = v;
    else continue;
    i++;
  }
  if (!a.url) throw new Error('--url is required');
  return a;
}

function makeRequest(base, counter) {
  const agent = new http.Agent({ keepAlive: true, maxSockets: 6 });
  const u = new URL(base);
  return function request(path) {
    counter.n++;
    return new Promise(function (resolve, reject) {
      const req = http.get({ hostname: u.hostname, port: u.port, path: path, agent: agent, headers: { Accept: 'application/json' } }, function (res) {
        const chunks = [];
        res.on('data', function (c) { chunks.push(c); });
        res.on('end', function () {
          const body = Buffer.concat(chunks);
          counter.bytes += body.length;
          let json = null;
          try {
            json = JSON.parse(body.toString('utf8'));
          } catch (e) {
            reject(new Error('bad JSON from ' + path));
            return;
          }
          if (res.statusCode >= 400) {
            const err = new Error((json && json.message) || 'HTTP ' + res.statusCode);
            err.status = res.statusCode;
            // Prometheus answers 4xx with a JSON body the caller may want.
            if (json && json.status === 'error') resolve(json);
            else reject(err);
            return;
          }
          resolve(json);
        });
      });
      req.on('error', reject);
    });
  };
}

function ms(hr) {
  return hr[0] * 1e3 + hr[1] / 1e6;
}

// Epoch milliseconds with sub-millisecond resolution (Date.now() anchored,
// hrtime deltas): request spans resolve to microseconds instead of 1 ms.
const EPOCH0 = Date.now();
const HR0 = process.hrtime();
const hiResClock = {
  setTimeout: function (fn, t) { return setTimeout(fn, t); },
  clearTimeout: function (h) { clearTimeout(h); },
  now: function () { return EPOCH0 + ms(process.hrtime(HR0)); },
};

function stats(xs) {
  const s = xs.slice().sort(function (a, b) { return a - b; });
  const q = function (p) {
    if (!s.length) return null;
    const idx = (s.length - 1) * p;
    const lo = Math.floor(idx);
    const hi = Math.ceil(idx);
    return s[lo] + (s[hi] - s[lo]) * (idx - lo);
  };
  const mean = s.reduce(function (a, b) { return a + b; }, 0) / (s.length || 1);
  return { n: s.length, p50: q(0.5), p95: q(0.95), min: s[0], max: s[s.length - 1], mean: mean };
}

/**
 * Build and render every dashboard view of schedule `s` as each page holds
 * its data (the first page of each pager, that page's own metrics), plus the
 * native detail sections of the nodes and pods those first pages show and
 * the Nodes-table columns of every node; returns the row counts.
 */
function renderAll(s) {
  const ctx = s.ctx();
  const pages = {};
  for (let p = 0; p < PAGES.length; p++) {
    const page = PAGES[p];
    pages[page] = pageVm(page, ctx, page === 'metrics' ? s.pageMstate() : s.mstate(), s.pageMetrics(page));
  }
  const rows = {};
  let htmlBytes = 0;
  for (const k in pages) {
    rows[k] = countRows(pages[k]);
    htmlBytes += renderPage(pages[k]).length;
  }
  let detailSections = 0;
  const nodeMetrics = s.pageMetrics('nodes');
  const shownNodes = nodePage(ctx.gpuNodes, PAGER).nodes;
  for (let i = 0; i < shownNodes.length; i++) {
    const sec = nodeDetailView(shownNodes[i], ctx, { metrics: nodeMetrics });
    if (sec) {
      detailSections++;
      htmlBytes += renderSection(sec).length;
    }
  }
  const shownPods = podPage(ctx.gpuPods, PAGER).nodes;
  for (let i = 0; i < shownPods.length; i++) {
    const sec = podDetailView(shownPods[i], { metrics: s.pageMetrics('pods') });
    if (sec) {
      detailSections++;
      htmlBytes += renderSection(sec).length;
    }
  }
  const cols = nodeColumns();
  let columnCells = 0;
  for (let i = 0; i < ctx.gpuNodes.length; i++) {
    for (let c = 0; c < cols.length; c++) {
      cols[c].getter(ctx.gpuNodes[i]);
      columnCells++;
    }
  }
  const m = s.pageMstate().metrics;
  return {
    gpuNodes: ctx.gpuNodes.length,
    gpuPods: ctx.gpuPods.length,
    // every GPU reporting (the Metrics page's cluster totals), not only the page's
    gpusMonitored: m ? (m.totals ? m.totals.gpus : m.gpus.length) : 0,
    nodeSummaryRows: rows.nodes.tableRows,
    podTableRows: rows.pods.tableRows,
    gpuCells: rows.nodes.gpuCells,
    metricsRows: rows.metrics.tableRows,
    detailSections: detailSections,
    columnCells: columnCells,
    htmlBytes: htmlBytes,
  };
}

/** The five routes, in sidebar order (src/routes.js). */
export const PAGES = ['overview', 'devicePlugins', 'nodes', 'pods', 'metrics'];

/** Build ONE page's view-model (the one whose Refresh was clicked), first page of the pager. */
function pageVm(page, ctx, mstate, pageMetrics) {
  if (page === 'overview') return overviewView(ctx);
  if (page === 'devicePlugins') return devicePluginsView(ctx, { pager: PAGER });
  if (page === 'nodes') return nodesView(ctx, { metrics: pageMetrics, pager: PAGER });
  if (page === 'pods') return podsView(ctx, { metrics: pageMetrics, pager: PAGER });
  return metricsView(ctx, mstate, { pager: PAGER });
}

/**
 * True when a page's view-model shows content rather than a loader: the
 * full-page loader is gone (title set); on Metrics, whose header and static
 * availability box render at once, a section of telemetry (or one saying
 * there is none / Prometheus is unreachable) is there too.
 */
function hasContent(page, vm) {
  if (!vm || vm.title === null) return false;
  if (page !== 'metrics') return true;
  return sections(vm).some(function (s) { return s.title !== 'Metric Availability'; });
}

/** Build and render ONE page; returns its row count. */
function renderOne(page, ctx, mstate, pageMetrics) {
  const vm = pageVm(page, ctx, mstate, pageMetrics);
  renderPage(vm);
  return countRows(vm).tableRows;
}

/** The pager state a page opens with (plugin.js usePager). */
const PAGER = { page: 0, filter: '' };

const harnessView = createRenderer(HarnessReact, HarnessCC);

/** Elements in an HTML string (opening tags). */
function htmlElements(html) {
  const m = html.match(/<[a-z]/g);
  return m ? m.length : 0;
}

/**
 * Mount `vm` as the page component renders it (harness React + shipped
 * renderer), then re-render with `vm2` (the page after a refresh).
 * @returns {{mountMs: number, rerenderMs: number, elements: number, htmlElements: number}}
 */
function reactMeasure(vm, vm2) {
  const h = HarnessReact.createElement;
  const t0 = process.hrtime();
  const r = HarnessReact.render(h(harnessView.Page, { vm: vm }));
  const mountMs = ms(process.hrtime(t0));
  const t1 = process.hrtime();
  r.rerender(h(harnessView.Page, { vm: vm2 }));
  const rerenderMs = ms(process.hrtime(t1));
  const elements = r.queryAll(function () { return true; }).length;
  r.unmount();
  return { mountMs: mountMs, rerenderMs: rerenderMs, elements: elements, htmlElements: htmlElements(renderPage(vm2)) };
}

/** Real React 18.3.1 production builds + the shipped renderer, loaded on first use (umdDir: see reactDomMeasure). */
let realDom = null;
async function realReact(umdDir) {
  if (!realDom) {
    const umd = await import('../tests/js/harness/umd-load.js');
    const cc = await import('../tests/js/harness/commonComponents.js');
    const loaded = umd.loadUmdReact(umdDir, 'production');
    const CC = cc.makeCommonComponents(loaded.React.createElement);
    realDom = { React: loaded.React, ReactDOM: loaded.ReactDOM, CC: CC, view: createRenderer(loaded.React, CC) };
  }
  return realDom;
}

/**
 * The same mount / re-render on REAL React: react@18.3.1 + react-dom@18.3.1
 * production UMD builds (what Headlamp serves users) committing with
 * ReactDOM.flushSync into the minimal DOM (tests/js/harness/minidom.js).
 * Median of `reps` mount + re-render + unmount cycles (the first warms the
 * JIT); elements = host elements in the container after the re-render.
 */
async function reactDomMeasure(umdDir, vm, vm2, reps) {
  const R = await realReact(umdDir);
  const h = R.React.createElement;
  const mounts = [];
  const rerenders = [];
  let elements = 0;
  for (let i = 0; i < reps; i++) {
    const c = document.createElement('div');
    document.body.appendChild(c);
    const root = R.ReactDOM.createRoot(c);
    const t0 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(h(R.view.Page, { vm: vm })); });
    mounts.push(ms(process.hrtime(t0)));
    const t1 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(h(R.view.Page, { vm: vm2 })); });
    rerenders.push(ms(process.hrtime(t1)));
    elements = c.querySelectorAll('*').length;
    R.ReactDOM.flushSync(function () { root.unmount(); });
    document.body.removeChild(c);
  }
  return { mountMs: stats(mounts).p50, rerenderMs: stats(rerenders).p50, elements: elements, reps: reps };
}

/**
 * Mount `make()` into a fresh root on real React (flushSync), wait until the
 * container shows `waitText` when given (a page whose data arrives through an
 * effect: the reference's MetricsPage fetches in useEffect), then call
 * `beforeRerender()` (a watch event: a new context value) and render again.
 * Median over `reps` cycles of the mount and re-render wall times.
 */
async function mountCycle(R, make, waitText, beforeRerender, reps, mustShow) {
  const mounts = [];
  const rerenders = [];
  let elements = 0;
  for (let i = 0; i < reps; i++) {
    const c = document.createElement('div');
    document.body.appendChild(c);
    const root = R.ReactDOM.createRoot(c);
    const t0 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(make()); });
    const errors = [];
    const consoleError = console.error;
    console.error = function () { errors.push(Array.prototype.join.call(arguments, ' ').slice(0, 500)); };
    try {
      const until = Date.now() + 60000;
      while (waitText && c.textContent.indexOf(waitText) < 0 && Date.now() < until && !errors.length) {
        await new Promise(function (r) { setImmediate(r); });
      }
    } finally {
      console.error = consoleError;
    }
    if (waitText && c.textContent.indexOf(waitText) < 0) {
      throw new Error('mountCycle: "' + waitText + '" never rendered' + (errors.length ? ': ' + errors.join(' | ') : ''));
    }
    mounts.push(ms(process.hrtime(t0)));
    if (mustShow && c.textContent.indexOf(mustShow) < 0) throw new Error('mountCycle: the page does not show "' + mustShow + '"');
    if (beforeRerender) beforeRerender();
    const t1 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(make()); });
    rerenders.push(ms(process.hrtime(t1)));
    elements = c.querySelectorAll('*').length;
    R.ReactDOM.flushSync(function () { root.unmount(); });
    document.body.removeChild(c);
  }
  return { mountMs: stats(mounts).p50, rerenderMs: stats(rerenders).p50, elements: elements, reps: reps };
}

/**
 * The reference's pages and this plugin's, each page mounted on real React
 * 18.3.1 (production builds) from the same synthetic cluster (see
 * ./referenceRender.js). Reference: mount with its data (its per-render
 * aggregation included), re-render on a watch event (a new context value:
 * new arrays of the same objects), and the provider's per-event filtering of
 * the whole lists (IntelGpuDataContext.tsx:200-208) apart. This plugin: mount
 * including the view-model built from a cold memo, re-render on the same
 * watch event (a new snapshot of the same data), first page of each pager.
 */
/** The header each reference page shows once its data is in (its Loader gone). */
const REFERENCE_TITLES = {
  overview: 'Intel GPU — Overview', devicePlugins: 'Intel GPU — Device Plugins', nodes: 'Intel GPU — Nodes',
  pods: 'Intel GPU — Pods', metrics: 'Intel GPU — Metrics',
};

async function compareRenders(c) {
  const R = await realReact(c.umdDir);
  const ref = loadReferencePages(c.referenceDir, R.React, R.CC);
  const reps = c.reps || 5;
  // (no 2 s request limit: the fake Prometheus evaluates 8,000 GPUs in Python on this host)
  const s = amdSchedule(makeRequest(a0.url, { n: 0, bytes: 0 }), null, 600000);
  await s.coldOpen();
  const request = makeRequest(a0.url, { n: 0, bytes: 0 });
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

const SNAPSHOT_CSS =
  'body{font-family:system-ui,sans-serif;margin:24px;color:#222;max-width:1200px}' +
  'h1{font-size:22px}h2{font-size:16px;border-bottom:1px solid #ddd;padding-bottom:4px;margin-top:28px}' +
  'table{border-collapse:collapse;font-size:13px;margin:8px 0}td,th{border:1px solid #e0e0e0;padding:3px 8px;text-align:left}' +
  'dl{display:grid;grid-template-columns:max-content auto;gap:2px 16px;font-size:13px}dt{font-weight:600}' +
  '[data-status=success]{color:#2e7d32}[data-status=warning]{color:#ef6c00}[data-status=error]{color:#c62828}' +
  'button{margin-left:12px}';

/** Write one static HTML file per view (plus a node and a pod detail section). */
function writeSnapshots(ctx, mstate, dir, now, history) {
  const hist = history || {};
  fs.mkdirSync(dir, { recursive: true });
  const opts = { metrics: mstate.metrics, now: now };
  const views = [
    ['01-overview', renderPage(overviewView(ctx, opts))],
    ['02-device-plugins', renderPage(devicePluginsView(ctx, opts))],
    ['03-gpu-nodes', renderPage(nodesView(ctx, opts))],
    ['04-gpu-pods', renderPage(podsView(ctx, opts))],
    ['05-metrics', renderPage(metricsView(ctx, Object.assign({}, mstate, { now: now })))],
  ];
  if (ctx.gpuNodes.length) {
    const s = nodeDetailView(ctx.gpuNodes[0], ctx, Object.assign({}, opts, { series: hist.node }));
    if (s) views.push(['06-node-detail', renderSection(s)]);
  }
  if (ctx.gpuPods.length) {
    const s = podDetailView(ctx.gpuPods[0], Object.assign({}, opts, { series: hist.pod }));
    if (s) views.push(['07-pod-detail', renderSection(s)]);
  }
  const files = [];
  for (let i = 0; i < views.length; i++) {
    const f = path.join(dir, views[i][0] + '.html');
    fs.writeFileSync(
      f,
      '<!doctype html><html><head><meta charset="utf-8"><title>amd-gpu — ' + views[i][0] + '</title><style>' +
        SNAPSHOT_CSS + '</style></head><body>\n' + views[i][1] + '\n</body></html>\n'
    );
    files.push(f);
  }
  return files;
}

// ---------------------------------------------------------------------------
// Schedules
// ---------------------------------------------------------------------------

function amdSchedule(request, clock, timeoutMs) {
  // Request spans from the data layer's tracing hook (clusterStore/metrics onTrace).
  const spans = [];
  function onTrace(span) {
    spans.push(span);
  }
  const clk = clock || hiResClock;
  const store = createClusterStore({ request: request, onTrace: onTrace, clock: clk, timeoutMs: timeoutMs });
  const metrics = createMetricsSource({ request: request, onTrace: onTrace, clock: clk, timeoutMs: timeoutMs });
  const mstate = { metrics: null, fetchError: null, fetching: false, series: null };
  // Per-page metrics state, as each page's own hook holds it (plugin.js):
  // GPU Nodes → owners + xGMI links of the nodes on its first page
  // ('topology', scoped), GPU Pods → pod→GPU attribution only, Metrics →
  // cluster totals + per-GPU gauges + series of the nodes on its first page
  // ('gauges', scoped). Cold open / route switch / the all-pages composite
  // fetch every live series in one query ('all').
  const pageMetrics = { nodes: null, pods: null };
  const metricsPage = { metrics: null, fetchError: null, fetching: false, series: null };
  function fetchMetrics(view) {
    return Promise.all([metrics.fetchGpuMetrics(view), metrics.fetchSeries(1800, 30)]).then(function (r) {
      mstate.metrics = r[0];
      mstate.series = r[1];
      mstate.fetchError = r[0] ? null : 'Could not reach Prometheus';
    });
  }
  /**
   * What the page's hook asks for now (pages.js telemetryScope): its query
   * key (null = disabled) and fetch options. While the node list loads, and
   * while every GPU node fits on one page, that is the size-guarded
   * small-cluster query under one key.
   */
  function scoped(summary) {
    const t = telemetryScope(store.getSnapshot(), PAGER);
    const key = !t.enabled ? null : t.scope === undefined ? 'all' : t.small ? 'small' : 'scope:' + t.scope.join(',');
    return t.scope === undefined ? { key: key, opts: undefined, scope: undefined, small: false }
      : { key: key, opts: { scope: t.scope, summary: summary, small: !!t.small }, scope: t.scope, small: !!t.small };
  }
  function ownersKey() {
    const o = ownersScope(store.getSnapshot(), PAGER);
    return !o.enabled ? null : o.pods === undefined ? 'all' : o.small ? 'small' : 'pods:' + o.pods.join(',');
  }
  /**
   * A page's metrics hook from mount to the lists: it fetches under the key
   * of its first render and again only if the lists change that key (a
   * larger cluster's first page), as useMetricsFetch does.
   */
  function pageOpen(page, onData) {
    const keyOf = page === 'pods' ? ownersKey : function () { return scoped(false).key; };
    const fetch0 = page === 'pods' ? fetchPodsPage : page === 'nodes' ? fetchNodesPage : fetchMetricsPage;
    const fetch = onData ? function () { return fetch0().then(onData); } : fetch0;
    const k0 = keyOf();
    const first = k0 === null ? Promise.resolve() : fetch();
    const second = listed(page === 'pods' ? 'podsState' : 'nodesState').then(function () {
      const k1 = keyOf();
      return k1 !== null && k1 !== k0 ? fetch() : first;
    });
    return Promise.all([first, second]);
  }
  function listed(which) {
    return new Promise(function (resolve) {
      function done() {
        const st = store.getSnapshot()[which];
        return st === 'ready' || st === 'error';
      }
      if (done()) return resolve();
      const off = store.subscribe(function () {
        if (done()) {
          off();
          resolve();
        }
      });
    });
  }
  function pageMetricsOf(page) {
    return page in pageMetrics && pageMetrics[page] ? pageMetrics[page] : mstate.metrics;
  }
  function fetchPodsPage() {
    const o = ownersScope(store.getSnapshot(), PAGER);
    return metrics.fetchGpuOwners(o.pods === undefined ? undefined : { pods: o.pods, small: !!o.small }).then(function (m) { pageMetrics.pods = m; });
  }
  function fetchNodesPage() {
    return metrics.fetchGpuMetrics('topology', scoped(false).opts).then(function (m) { pageMetrics.nodes = m; });
  }
  function fetchMetricsPage() {
    const sc = scoped(true);
    return Promise.all([metrics.fetchGpuMetrics('gauges', sc.opts), metrics.fetchSeries(1800, 30, sc.scope, sc.small)]).then(function (r) {
      metricsPage.metrics = r[0];
      metricsPage.series = r[1];
      metricsPage.fetchError = r[0] ? null : 'Could not reach Prometheus';
    });
  }
  return {
    /**
     * Every page's data at once, as each page fetches it: the lists, the
     * DeviceConfig and the pages' size-guarded telemetry in one wave; on a
     * cluster larger than one page, GPU Nodes / Metrics / GPU Pods telemetry
     * of their first pages once the node (pod) list is in.
     */
    coldOpen: function () {
      return Promise.all([store.loadLists(), store.refresh(), pageOpen('nodes'), pageOpen('metrics'), pageOpen('pods')]);
    },
    /** Composite refresh: every page's Refresh in one wave (5 requests, within the 6 browser sockets). */
    refresh: function () {
      return Promise.all([store.refresh(), fetchNodesPage(), fetchPodsPage(), fetchMetricsPage()]);
    },
    /** Every live series of every GPU (the terminal client's and the screenshots' snapshot). */
    fetchAll: function () {
      return fetchMetrics();
    },
    /** One page's Refresh button, as src/plugin.js wires it. */
    refreshPage: function (page) {
      // GPU Nodes / GPU Pods renew their telemetry only (plugin.js: the lists are watches).
      if (page === 'nodes') return fetchNodesPage();
      if (page === 'pods') return fetchPodsPage();
      if (page === 'metrics') return fetchMetricsPage();
      return store.refresh();
    },
    /**
     * One page opened on an empty cache, as src/plugin.js mounts it: the
     * provider's lists + DeviceConfig request and the page's size-guarded
     * telemetry in one wave — all of it on a cluster of one page; a larger
     * cluster's GPU Nodes / Metrics (GPU Pods) ask for their first page of
     * nodes (pods) once the node (pod) list is there (a second wave).
     *
     * `marks` (all optional) are called as the page fills in:
     *   first     the page's view-model first shows content (pages.js decides:
     *             its full-page loader gone; on Metrics, telemetry or a state
     *             saying there is none) — built and rendered on every store
     *             commit and telemetry answer, as the mounted page re-renders;
     *   content   the lists + DeviceConfig committed (the reference's content);
     *   complete  everything THIS page draws is in (Metrics: the node list and
     *             its telemetry, not the pod list; Device Plugins: the
     *             DeviceConfigs and the pod list; the others: both lists, the
     *             DeviceConfigs where shown, their telemetry).
     * Resolves when every request has finished (the next open starts drained).
     */
    coldOpenPage: function (page, marks) {
      const mk = marks || {};
      // What the page's route mounts (src/plugin.js PAGE_NEEDS).
      const needs = PAGE_NEEDS[page === 'devicePlugins' ? 'device-plugins' : page];
      let shown = !mk.first;
      function check() {
        if (shown) return;
        const vm = pageVm(page, store.getSnapshot(), page === 'metrics' ? metricsPage : mstate, pageMetricsOf(page));
        if (!hasContent(page, vm)) return;
        shown = true;
        renderPage(vm);
        mk.first();
      }
      const off = store.subscribe(check);
      const lists = store.loadLists({ nodes: needs.nodes, pods: needs.pods });
      const crd = needs.crd ? store.refresh() : Promise.resolve();
      // The page's metrics hook runs from the first render (pages.js
      // telemetryScope) and once more if the node list changes its key.
      const telemetry = page === 'nodes' || page === 'metrics' || page === 'pods' ? pageOpen(page, check) : Promise.resolve();
      const content = Promise.all([lists, crd]).then(function () { if (mk.content) mk.content(); });
      // Everything the page draws: what its route mounts, and its telemetry.
      const complete = Promise.all([lists, crd, telemetry]).then(function () { if (mk.complete) mk.complete(); });
      return Promise.all([lists, crd, telemetry, content, complete]).then(function () { off(); });
    },
    pageMetrics: pageMetricsOf,
    /** The Metrics page's own state (its hook), for rendering that page. */
    pageMstate: function () { return metricsPage; },
    /** Route switch: render from the shared store now, revalidate in the background. */
    switchRoute: function () {
      const bg = Promise.all([store.refresh(), fetchNodesPage(), fetchPodsPage(), fetchMetricsPage()]);
      return { rendered: Promise.resolve(), background: bg };
    },
    ctx: function () { return store.getSnapshot(); },
    mstate: function () { return mstate; },
    source: metrics,
    spans: spans,
  };
}

/** p50 latency per traced request kind, plus how many of each were issued. */
function traceSummary(spans) {
  const by = {};
  for (let i = 0; i < spans.length; i++) {
    const s = spans[i];
    const k = s.name.replace(/-\d+$/, '');
    if (!by[k]) by[k] = [];
    by[k].push(s.end - s.start);
  }
  const out = {};
  for (const k in by) out[k] = { n: by[k].length, p50_ms: stats(by[k]).p50 };
  return out;
}

function referenceSchedule(request) {
  const r = createReferenceSchedule(request);
  return {
    coldOpen: r.coldOpen,
    refresh: r.refresh,
    switchRoute: function () {
      const p = r.coldOpen();
      return { rendered: p, background: p };
    },
    refreshPage: r.refreshPage,
    coldOpenPage: r.coldOpenPage,
    pageMetrics: function () { return r.metrics(); },
    pageMstate: function () { return { metrics: r.metrics(), fetchError: r.metrics() ? null : 'unreachable', fetching: false }; },
    ctx: r.snapshot,
    mstate: function () { return { metrics: r.metrics(), fetchError: r.metrics() ? null : 'unreachable', fetching: false }; },
  };
}

async function measure(name, factory, base, a) {
  const counter = { n: 0, bytes: 0 };
  const request = makeRequest(base, counter);
  const out = { schedule: name };

  // Cold opens: fresh schedule each time.
  const cold = [];
  let coldRequests = 0;
  for (let i = 0; i < a.cold; i++) {
    const s = factory(makeRequest(base, counter));
    const before = counter.n;
    const t0 = process.hrtime();
    await s.coldOpen();
    renderAll(s);
    cold.push(ms(process.hrtime(t0)));
    coldRequests = counter.n - before;
  }
  out.cold = stats(cold);
  out.coldRequests = coldRequests;

  // Warm refreshes on one long-lived page.
  const s = factory(request);
  await s.coldOpen();
  for (let i = 0; i < a.warmup; i++) {
    await s.refresh();
    renderAll(s);
  }
  const lat = [];
  const reqBefore = counter.n;
  const bytesBefore = counter.bytes;
  let rows = null;
  for (let i = 0; i < a.steps; i++) {
    const t0 = process.hrtime();
    await s.refresh();
    rows = renderAll(s);
    lat.push(ms(process.hrtime(t0)));
  }
  out.refresh = stats(lat);
  out.refreshSamples = lat;
  out.requestsPerRefresh = (counter.n - reqBefore) / Math.max(1, a.steps);
  out.bytesPerRefresh = (counter.bytes - bytesBefore) / Math.max(1, a.steps);
  out.rows = rows;

  // Route switches (time to first render with data).
  const sw = [];
  for (let i = 0; i < Math.max(3, Math.min(a.cold, 10)); i++) {
    const t0 = process.hrtime();
    const r = s.switchRoute();
    await r.rendered;
    renderAll(s);
    sw.push(ms(process.hrtime(t0)));
    await r.background;
  }
  out.switch = stats(sw);
  return out;
}

/**
 * --serve: line-oriented JSON command loop on stdin/stdout so the Python
 * harness can bracket exactly the timed steps with its own barrier / clock.
 *   {"cmd":"cold","schedule":"amd","n":3}
 *   {"cmd":"steps","schedule":"amd","n":K}      → per-step latencies
 *   {"cmd":"switch","schedule":"amd","n":3}
 *   {"cmd":"quit"}
 */
/** The serve loop's arguments (compareRenders fetches from the same control plane). */
let a0 = null;

async function serve(a) {
  a0 = a;
  // The views format "Last Fetched" with Date#toLocaleTimeString. Its first
  // call in a process builds an Intl formatter: V8 loads the ICU data the
  // Node binary carries, paged in from disk on a fresh host. A browser
  // (Headlamp) has ICU resident; a fresh Node process does not, and on the
  // GPU box that cost landed in the first timed refresh (~1 s,
  // profiles/r3b_smoke.log). It is paid here, once, before any command, and
  // reported by 'hello'.
  const icu0 = process.hrtime();
  new Date(0).toLocaleTimeString();
  const startup = { icuMs: ms(process.hrtime(icu0)), node: process.version };
  const counter = { n: 0, bytes: 0 };
  const live = {};
  function get(name) {
    if (!live[name]) {
      const f = name === 'reference' ? referenceSchedule : amdSchedule;
      live[name] = { s: f(makeRequest(a.url, counter)), opened: false };
    }
    return live[name];
  }
  const rl = (await import('readline')).createInterface({ input: process.stdin });
  for await (const line of rl) {
    if (!line.trim()) continue;
    const c = JSON.parse(line);
    const out = { cmd: c.cmd };
    try {
      if (c.cmd === 'hello') {
        out.startup = startup;
        process.stdout.write(JSON.stringify(out) + '\n');
        continue;
      }
      if (c.cmd === 'quit') {
        process.stdout.write(JSON.stringify(out) + '\n');
        break;
      }
      const name = c.schedule || 'amd';
      const n = c.n || 1;
      if (c.cmd === 'cold') {
        const lat = [];
        const renderMs = [];
        let req = 0;
        // Cold caches, warm connections: a browser keeps its keep-alive
        // sockets to the Headlamp origin across in-app navigations.
        const pool = makeRequest(a.url, counter);
        for (let i = 0; i < n; i++) {
          const s = (name === 'reference' ? referenceSchedule : amdSchedule)(pool);
          const before = counter.n;
          const t0 = process.hrtime();
          await s.coldOpen();
          const t1 = process.hrtime();
          renderAll(s);
          lat.push(ms(process.hrtime(t0)));
          renderMs.push(ms(process.hrtime(t1)));
          req = counter.n - before;
          if (s.spans) out.trace = traceSummary(s.spans);
        }
        out.latencies = lat;
        out.renderMs = renderMs;
        out.requests = req;
      } else if (c.cmd === 'coldPages') {
        // Per-page cold open: a fresh schedule (empty caches, new client)
        // per open; time to that page's data committed + the page rendered.
        out.pages = {};
        const pool = makeRequest(a.url, counter); // warm connections, as for 'cold'
        for (let p = 0; p < PAGES.length; p++) {
          const page = PAGES[p];
          const lat = [];
          const renderMs = [];
          const gcMs = [];
          let req = 0;
          let trace = null;
          const content = [];
          const first = [];
          for (let i = 0; i < n; i++) {
            const s = (name === 'reference' ? referenceSchedule : amdSchedule)(pool);
            const before = counter.n;
            const p0 = performance.now();
            const t0 = process.hrtime();
            let tf = null;
            let tc = null;
            let done = null;
            const render = function () {
              const t1 = process.hrtime();
              renderOne(page, s.ctx(), page === 'metrics' ? s.pageMstate() : s.mstate(), s.pageMetrics(page));
              renderMs.push(ms(process.hrtime(t1)));
              done = ms(process.hrtime(t0));
            };
            await s.coldOpenPage(page, {
              first: function () { tf = ms(process.hrtime(t0)); },
              content: function () { tc = ms(process.hrtime(t0)); },
              complete: render,
            });
            // The reference's schedule has no marks: one full-page loader
            // until its whole open is in, then the page.
            if (done === null) render();
            lat.push(done);
            // Time to the reference-equivalent content (lists + DeviceConfig),
            // and to the first render with content (progressive pages).
            content.push(tc === null ? done : tc);
            first.push(tf === null ? done : tf);
            // observer entries are delivered asynchronously
            await new Promise(function (r) { setImmediate(r); });
            gcMs.push(gcBetween(p0, performance.now()));
            req = counter.n - before;
            if (s.spans) trace = traceSummary(s.spans);
          }
          out.pages[page] = { latencies: lat, contentMs: content, firstMs: first, renderMs: renderMs, gcMs: gcMs, requests: req, trace: trace };
        }
      } else if (c.cmd === 'steps') {
        const L = get(name);
        if (!L.opened) {
          await L.s.coldOpen();
          // The page rendered when it mounted: a Refresh click always comes
          // after a first render (untimed here, as in the browser).
          renderAll(L.s);
          L.opened = true;
        }
        const lat = [];
        const before = counter.n;
        const bytesBefore = counter.bytes;
        const spanStart = L.s.spans ? L.s.spans.length : 0;
        const render = [];
        let rows = null;
        const stepStarts = [];
        const renderCpu = [];
        for (let i = 0; i < n; i++) {
          stepStarts.push(hiResClock.now());
          const t0 = process.hrtime();
          await L.s.refresh();
          const t1 = process.hrtime();
          const c0 = process.cpuUsage();
          rows = renderAll(L.s);
          const cu = process.cpuUsage(c0);
          render.push(ms(process.hrtime(t1)));
          // CPU this process spent rendering: far below the wall time means
          // it was not running (descheduled / throttled), not slow code.
          renderCpu.push((cu.user + cu.system) / 1000);
          lat.push(ms(process.hrtime(t0)));
        }
        // Data committed → every view rebuilt and rendered, per step.
        out.renderMs = render;
        out.renderCpuMs = renderCpu;
        if (L.s.spans) out.trace = traceSummary(L.s.spans.slice(spanStart));
        // Every request of these steps, epoch ms (diagnostics: attribute one slow step).
        if (c.rawSpans && L.s.spans) {
          out.spans = L.s.spans.slice(spanStart).map(function (sp) {
            return { name: sp.name, start: sp.start, end: sp.end, ok: sp.ok };
          });
          out.stepStarts = stepStarts;
        }
        const snap = L.s.ctx();
        const ms_ = L.s.pageMstate ? L.s.pageMstate() : L.s.mstate();
        out.state = {
          error: snap.error, crdAvailable: snap.crdAvailable, deviceConfigs: snap.deviceConfigs.length,
          pluginPods: snap.pluginPods.length, metrics: !!ms_.metrics, stale: !!(ms_.metrics && ms_.metrics.stale),
        };
        out.latencies = lat;
        out.requestsPerStep = (counter.n - before) / n;
        out.bytesPerStep = (counter.bytes - bytesBefore) / n;
        out.rows = rows;
      } else if (c.cmd === 'pages') {
        // Per-page refresh: n rounds through the five routes; on each, the
        // page's own Refresh button is clicked and the time to its data
        // committed + that page rebuilt and rendered is recorded.
        const L = get(name);
        if (!L.opened) {
          await L.s.coldOpen();
          renderAll(L.s); // mounted pages rendered once (untimed)
          L.opened = true;
        }
        const lat = {};
        const reqs = {};
        const rows = {};
        const rend = {};
        for (let p = 0; p < PAGES.length; p++) {
          lat[PAGES[p]] = [];
          rend[PAGES[p]] = [];
          reqs[PAGES[p]] = 0;
        }
        for (let i = 0; i < n; i++) {
          for (let p = 0; p < PAGES.length; p++) {
            const page = PAGES[p];
            const before = counter.n;
            const t0 = process.hrtime();
            await L.s.refreshPage(page);
            const t1 = process.hrtime();
            rows[page] = renderOne(page, L.s.ctx(), page === 'metrics' ? L.s.pageMstate() : L.s.mstate(), L.s.pageMetrics(page));
            lat[page].push(ms(process.hrtime(t0)));
            rend[page].push(ms(process.hrtime(t1)));
            reqs[page] += counter.n - before;
          }
        }
        out.pages = {};
        for (let p = 0; p < PAGES.length; p++) {
          out.pages[PAGES[p]] = {
            latencies: lat[PAGES[p]], renderMs: rend[PAGES[p]], requestsPerClick: reqs[PAGES[p]] / n, tableRows: rows[PAGES[p]],
          };
        }
        if (c.react) {
          // Untimed: each page mounted in the harness React, refreshed, re-rendered.
          out.react = {};
          for (let p = 0; p < PAGES.length; p++) {
            const page = PAGES[p];
            const ms0 = function () { return page === 'metrics' ? L.s.pageMstate() : L.s.mstate(); };
            const vm = pageVm(page, L.s.ctx(), ms0(), L.s.pageMetrics(page));
            await L.s.refreshPage(page);
            const vm2 = pageVm(page, L.s.ctx(), ms0(), L.s.pageMetrics(page));
            out.react[page] = reactMeasure(vm, vm2);
            if (c.reactUmdDir) {
              out.reactDom = out.reactDom || {};
              out.reactDom[page] = await reactDomMeasure(c.reactUmdDir, vm, vm2, c.reactReps || 9);
            }
          }
        }
      } else if (c.cmd === 'snapshot') {
        // Static HTML of every view (docs/screenshots): same IR → HTML path as
        // the benchmark. With `now` the data layer runs on that fixed clock
        // (fetch times, range windows), so the files are reproducible.
        let snap;
        let history = null;
        if (c.now) {
          const fixed = { setTimeout: setTimeout, clearTimeout: clearTimeout, now: function () { return c.now; } };
          snap = amdSchedule(makeRequest(a.url, counter), fixed);
          await snap.coldOpen();
          await snap.fetchAll();
          // The detail pages' power history, as src/plugin.js fetches it.
          const c0 = snap.ctx();
          const n0 = c0.gpuNodes[0];
          const p0 = c0.gpuPods[0];
          history = {
            node: n0 ? await snap.source.fetchNodeSeries(n0.metadata.name, 1800, 30) : null,
            pod: p0 ? await snap.source.fetchPodSeries(p0.metadata.namespace || '', p0.metadata.name, 1800, 30) : null,
          };
        } else {
          const L = get(name);
          if (!L.opened) {
            await L.s.coldOpen();
            L.opened = true;
          }
          if (L.s.fetchAll) await L.s.fetchAll();
          snap = L.s;
        }
        out.files = writeSnapshots(snap.ctx(), snap.mstate(), c.dir, c.now, history);
      } else if (c.cmd === 'detail') {
        // Native detail pages opened on a warm cluster (a plugin page loaded
        // before): Pod detail and Node detail each fetch their node's
        // telemetry with a hostname-scoped query on a fresh metrics client,
        // next to the cluster-wide snapshot the pod detail would otherwise
        // need; and the GPU Pods page with its attribution-only query.
        const L = get('amd');
        if (!L.opened) {
          await L.s.coldOpen();
          L.opened = true;
        }
        const ctx = L.s.ctx();
        const pods = ctx.gpuPods.filter(function (p) { return p.spec && p.spec.nodeName; });
        const MODES = ['podScoped', 'podDetail', 'podClusterWide', 'nodeScoped', 'nodeDetail', 'nodeDetailCold',
          'nodeDetailColdReference', 'podsPageOwners'];
        const modes = {};
        const bytes = {};
        const reqs = {};
        MODES.forEach(function (k) { modes[k] = []; bytes[k] = 0; reqs[k] = 0; });
        const slow = [];
        const detailRequest = makeRequest(a.url, counter);
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
            // src/plugin.js NodeDetailCold wires it: the node's pods by one
            // field-selected request, its telemetry and history, one wave.
            ['nodeDetailCold', function (src) {
              const nm = pod.spec.nodeName;
              return Promise.all([fetchNodePods(detailRequest, nm), src.fetchNodeMetrics(nm), src.fetchNodeSeries(nm, 1800, 30)])
                .then(function (r) {
                  const cold = { loading: false, gpuPods: filterGpuRequestingPods(r[0]), podsState: 'ready', error: null };
                  return node ? nodeDetailView(node, cold, { metrics: r[1], series: r[2] }) : null;
                });
            }],
            // The reference on the same open: a full provider (both
            // cluster-wide lists alongside CRD + 3 serial selector requests,
            // src/index.tsx:152-160), then its section from that context.
            ['nodeDetailColdReference', function () {
              const ref = createReferenceSchedule(detailRequest);
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
              request: detailRequest, clock: hiResClock, onTrace: function (sp) { spans.push(sp); },
            });
            const b0 = counter.bytes;
            const n0 = counter.n;
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
            bytes[runs[r][0]] += counter.bytes - b0;
            reqs[runs[r][0]] += counter.n - n0;
          }
        }
        out.detail = {};
        out.detailSlow = slow;
        for (const k in modes) {
          out.detail[k] = { latencies: modes[k], bytesPerOpen: bytes[k] / Math.max(1, modes[k].length), requestsPerOpen: reqs[k] / Math.max(1, modes[k].length) };
        }
      } else if (c.cmd === 'refRender') {
        // The reference's own pages next to this plugin's, on real React (bench/referenceRender.js).
        out.render = await compareRenders(c);
      } else if (c.cmd === 'switch') {
        const L = get(name);
        if (!L.opened) {
          await L.s.coldOpen();
          L.opened = true;
        }
        const lat = [];
        for (let i = 0; i < n; i++) {
          const t0 = process.hrtime();
          const r = L.s.switchRoute();
          await r.rendered;
          renderAll(L.s);
          lat.push(ms(process.hrtime(t0)));
          await r.background;
        }
        out.latencies = lat;
      } else {
        throw new Error('unknown cmd ' + c.cmd);
      }
    } catch (e) {
      out.error = String(e && e.stack ? e.stack : e);
    }
    process.stdout.write(JSON.stringify(out) + '\n');
  }
}

async function main() {
  const argv = process.argv.slice(2);
  const a = parseArgs(argv);
  if (argv.indexOf('--serve') >= 0) return serve(a);
  const res = { url: a.url, steps: a.steps, warmup: a.warmup, node: process.version, results: {} };
  if (a.schedule === 'reference' || a.schedule === 'both') res.results.reference = await measure('reference', referenceSchedule, a.url, a);
  if (a.schedule === 'amd' || a.schedule === 'both') res.results.amd = await measure('amd', amdSchedule, a.url, a);
  const txt = JSON.stringify(res);
  if (a.out) fs.writeFileSync(a.out, txt);
  else process.stdout.write(txt + '\n');
}

main().then(
  function () { process.exit(0); },
  function (e) {
    process.stderr.write(String(e && e.stack ? e.stack : e) + '\n');
    process.exit(1);
  }
);
