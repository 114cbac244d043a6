/**
 * The benchmark's page builds: each route's view-model as its page builds it
 * (first page of each pager), rendered to HTML (IR → HTML, src/view/html.js)
 * or mounted in the harness React through the shipped renderer
 * (src/view/react.js); and the static HTML snapshots of every view.
 */
import fs from 'fs';
import path from 'path';
import { nodeColumns, nodeDetailView, podDetailView } from '../src/view/pages/details.js';
import { devicePluginsView } from '../src/view/pages/devicePlugins.js';
import { metricsView } from '../src/view/pages/metricsPage.js';
import { nodesView } from '../src/view/pages/nodes.js';
import { overviewView } from '../src/view/pages/overview.js';
import { nodePage, podPage } from '../src/view/pages/paging.js';
import { podsView } from '../src/view/pages/pods.js';
import { countRows, sections } from '../src/view/ir.js';
import { renderPage, renderSection } from '../src/view/html.js';
import { renderPageSvg, renderSectionSvg } from '../src/view/svg.js';
// The harness React (the Node-12 stand-in the spec suite renders the plugin
// with) and its CommonComponents: the pages are also mounted through the
// shipped renderer to count elements and time a mount / re-render, next to
// the IR → HTML figure.
import * as HarnessReact from '../tests/js/stubs/react.js';
import * as HarnessCC from '../tests/js/stubs/CommonComponents.js';
import { createRenderer } from '../src/view/react.js';
import { ms } from './common.js';

/** The pager state a page opens with (plugin.js usePager). */
export const PAGER = { page: 0, filter: '' };

/**
 * Build and render every dashboard view of schedule `s` as each page holds
 * its data (the first page of each pager, that page's own metrics), plus the
 * native detail sections of the nodes and pods those first pages show and
 * the Nodes-table columns of every node; returns the row counts.
 */
export function renderAll(s) {
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
export function pageVm(page, ctx, mstate, pageMetrics) {
  if (page === 'overview') return overviewView(ctx, { metrics: pageMetrics });
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
export function hasContent(page, vm) {
  if (!vm || vm.title === null) return false;
  if (page !== 'metrics') return true;
  return sections(vm).some(function (s) { return s.title !== 'Metric Availability'; });
}

/** Build and render ONE page; returns its row count. */
export function renderOne(page, ctx, mstate, pageMetrics) {
  const vm = pageVm(page, ctx, mstate, pageMetrics);
  renderPage(vm);
  return countRows(vm).tableRows;
}

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
export function reactMeasure(vm, vm2) {
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

const SNAPSHOT_CSS =
  'body{font-family:system-ui,sans-serif;margin:24px;color:#222;max-width:1200px}' +
  'h1{font-size:22px}h2{font-size:16px;border-bottom:1px solid #ddd;padding-bottom:4px;margin-top:28px}' +
  'table{border-collapse:collapse;font-size:13px;margin:8px 0}td,th{border:1px solid #e0e0e0;padding:3px 8px;text-align:left}' +
  'dl{display:grid;grid-template-columns:max-content auto;gap:2px 16px;font-size:13px}dt{font-weight:600}' +
  '[data-status=success]{color:#2e7d32}[data-status=warning]{color:#ef6c00}[data-status=error]{color:#c62828}' +
  'button{margin-left:12px}';

/** Write one static HTML file per view (plus a node and a pod detail section). */
export function writeSnapshots(ctx, mstate, dir, now, history) {
  const hist = history || {};
  fs.mkdirSync(dir, { recursive: true });
  const opts = { metrics: mstate.metrics, now: now };
  // [file name, page view-model] or [file name, section, true]
  const views = [
    ['01-overview', overviewView(ctx, opts)],
    ['02-device-plugins', devicePluginsView(ctx, opts)],
    ['03-gpu-nodes', nodesView(ctx, opts)],
    ['04-gpu-pods', podsView(ctx, opts)],
    ['05-metrics', metricsView(ctx, Object.assign({}, mstate, { now: now }))],
  ];
  if (ctx.gpuNodes.length) {
    const s = nodeDetailView(ctx.gpuNodes[0], ctx, Object.assign({}, opts, { series: hist.node }));
    if (s) views.push(['06-node-detail', s, true]);
  }
  if (ctx.gpuPods.length) {
    const s = podDetailView(ctx.gpuPods[0], Object.assign({}, opts, { series: hist.pod }));
    if (s) views.push(['07-pod-detail', s, true]);
  }
  const files = [];
  for (let i = 0; i < views.length; i++) {
    const v = views[i];
    const f = path.join(dir, v[0] + '.html');
    fs.writeFileSync(
      f,
      '<!doctype html><html><head><meta charset="utf-8"><title>amd-gpu — ' + v[0] + '</title><style>' +
        SNAPSHOT_CSS + '</style></head><body>\n' + (v[2] ? renderSection(v[1]) : renderPage(v[1])) + '\n</body></html>\n'
    );
    files.push(f);
    // The same view-model as a picture (ArtifactHub and README cannot show HTML).
    const g = path.join(dir, v[0] + '.svg');
    fs.writeFileSync(g, v[2] ? renderSectionSvg(v[1]) : renderPageSvg(v[1]));
    files.push(g);
  }
  return files;
}
