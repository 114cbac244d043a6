/**
 * View IR → static semantic HTML.
 *
 * Uses the same element mapping the reference's component tests use to mock
 * Headlamp CommonComponents (src/components/OverviewPage.test.tsx:8-61):
 * SectionBox → <section><h2>, SectionHeader → <h1>, NameValueTable → <dl>,
 * SimpleTable → <table>, StatusLabel → <span data-status>, Loader →
 * data-testid="loader", PercentageBar → data-testid="percentage-bar".
 *
 * Used by the Node-side tests and by the benchmark to measure "rows
 * rendered" on real output; the shipped plugin renders the IR with React
 * (src/view/react.js, bound in src/headlamp.ts).
 */

import { matrixCaption, matrixSummary, pagerIdle, pagerText } from './ir.js';

const NEEDS_ESC = /[&<>"]/;

function esc(s) {
  // Most values (names, numbers, units) need no escaping: one test, no copies.
  if (typeof s === 'number' || !NEEDS_ESC.test(s)) return String(s);
  return String(s)
    .replace(/&/g, '&amp;')
    .replace(/</g, '&lt;')
    .replace(/>/g, '&gt;')
    .replace(/"/g, '&quot;');
}

export function renderValue(v) {
  if (v === null || v === undefined) return '';
  if (typeof v === 'string' || typeof v === 'number') return esc(v);
  switch (v.t) {
    case 'status':
      return '<span data-status="' + esc(v.status) + '">' + esc(v.text) + '</span>';
    case 'bar':
      return (
        '<div class="bar"' + (v.pct === null ? '' : ' data-pct="' + v.pct + '"') + ' data-color="' + esc(v.color) + '">' +
        '<span>' + esc(v.text) + '</span></div>'
      );
    case 'lines':
      return v.lines
        .map(function (l) {
          return '<div>' + (l.label ? '<strong>' + esc(l.label) + '</strong>: ' : '') + esc(l.text) + '</div>';
        })
        .join('');
    default:
      return '';
  }
}

/** Whether a grid's diagonal carries per-GPU xGMI totals (a hand-made block has no throughputPerGpu). */
function selfMeasured(m) {
  for (let i = 0; i < m.size; i++) if (m.cells[i][i].measuredGBs !== null && m.cells[i][i].measuredGBs !== undefined) return true;
  return false;
}

function renderBlock(b) {
  switch (b.t) {
    case 'kv':
      return (
        '<dl>' +
        b.rows.map(function (r) { return '<div><dt>' + esc(r.name) + '</dt><dd>' + renderValue(r.value) + '</dd></div>'; }).join('') +
        '</dl>'
      );
    case 'table':
      return (
        '<table><thead><tr>' +
        b.columns.map(function (c) { return '<th>' + esc(c) + '</th>'; }).join('') +
        '</tr></thead><tbody>' +
        b.rows
          .map(function (r) { return '<tr>' + r.map(function (c) { return '<td>' + renderValue(c) + '</td>'; }).join('') + '</tr>'; })
          .join('') +
        '</tbody></table>'
      );
    case 'pctbar':
      return (
        '<div><div>' + esc(b.label) + '</div><div data-testid="percentage-bar" data-total="' + b.total + '">' +
        b.data.map(function (d) { return '<i data-name="' + esc(d.name) + '" data-value="' + d.value + '"></i>'; }).join('') +
        '</div></div>'
      );
    case 'slots':
      return (
        '<ol data-testid="gpu-slots" data-exact="' + (b.exact ? 'true' : 'false') + '">' +
        b.slots
          .map(function (s) {
            return '<li data-gpu="' + s.index + '"' + (s.pod ? ' data-pod="' + esc(s.pod) + '"' : '') + '>' +
              'GPU ' + (s.partition === null || s.partition === undefined ? s.index : s.board + '·' + s.partition) + ': ' + (s.pod ? esc(s.pod) + (s.inferred ? ' (inferred)' : '') : 'free') + '</li>';
          })
          .join('') +
        '</ol>'
      );
    case 'matrix': {
      const m = b.matrix;
      const attrs = 'data-testid="xgmi-matrix" data-full-mesh="' + (b.fullMesh ? 'true' : 'false') + '" data-topology="' +
        (b.measuredTopology ? 'measured' : 'assumed') + '" data-throughput="' + (b.measuredThroughput ? 'measured' : (b.throughputPerGpu !== undefined ? b.throughputPerGpu : selfMeasured(m)) ? 'per-gpu' : 'none') + '"';
      // A closed matrix (GPU Nodes cards) is its summary, as the React renderer draws it.
      if (b.open === false) return '<details ' + attrs + '><summary>' + esc(matrixCaption(b) + matrixSummary(b)) + '</summary></details>';
      let h = '<table ' + attrs + '><caption>' + esc(matrixCaption(b) + matrixSummary(b)) + '</caption><thead><tr><th></th>';
      for (let j = 0; j < m.size; j++) h += '<th>GPU ' + j + '</th>';
      h += '</tr></thead><tbody>';
      for (let i = 0; i < m.size; i++) {
        h += '<tr><th>GPU ' + i + '</th>';
        for (let j = 0; j < m.size; j++) {
          const c = m.cells[i][j];
          h += '<td data-kind="' + c.kind + '">' + (c.kind === 'self' ? (c.measuredGBs !== null ? '\u03a3 ' + c.measuredGBs.toFixed(1) + ' GB/s' : '—') : c.kind === 'xgmi'
            ? (c.measuredGBs !== null ? c.measuredGBs.toFixed(1) + '/' : '') + c.peakGBs + ' GB/s'
            : c.kind) + '</td>';
        }
        h += '</tr>';
      }
      return h + '</tbody></table>';
    }
    case 'series': {
      const nodes = Object.keys(b.power || {});
      return '<div data-testid="series" data-nodes="' + nodes.length + '">' +
        nodes.map(function (n) {
          const avg = b.avgPower && b.avgPower[n] !== undefined ? ' data-avg-w="' + b.avgPower[n].toFixed(1) + '"' : '';
          return '<div data-node="' + esc(n) + '" data-points="' + b.power[n].length + '"' + avg + '></div>';
        }).join('') +
        '</div>';
    }
    default:
      return '';
  }
}

const sectionCache = typeof WeakMap === 'function' ? new WeakMap() : null;

/**
 * Section → HTML, cached by section identity: the analog of `React.memo` on
 * View.tsx's Section. View-models return the same section object when its
 * inputs are unchanged, so an unchanged section is not re-rendered.
 */
export function renderSection(s) {
  if (!s) return '';
  if (sectionCache) {
    const hit = sectionCache.get(s);
    if (hit !== undefined) return hit;
  }
  const h = '<section><h2>' + esc(s.title) + '</h2>' + s.blocks.map(renderBlock).join('') + '</section>';
  if (sectionCache) sectionCache.set(s, h);
  return h;
}

/** Pager → <nav>: the range shown, the name filter and previous / next buttons. */
export function renderPager(p) {
  const head = '<nav data-testid="pager" data-page="' + p.page + '" data-pages="' + p.pages + '" data-total="' + p.total + '"';
  // Nothing to control (one page, no filter, default order): the count alone, as the React renderer draws it.
  if (pagerIdle(p)) return head + ' data-idle="true"><span>' + esc(pagerText(p)) + '</span></nav>';
  return head + '>' +
    '<input aria-label="Filter ' + esc(p.label || p.noun) + ' by name" value="' + esc(p.filter) + '">' +
    (p.sorts
      ? '<select aria-label="Sort ' + esc(p.label || p.noun) + '">' + p.sorts.map(function (o) {
        return '<option value="' + esc(o.value) + '"' + (o.value === p.sort ? ' selected' : '') + '>' + esc(o.label) + '</option>';
      }).join('') + '</select>'
      : '') +
    '<span>' + esc(pagerText(p)) + '</span>' +
    '<button aria-label="Previous page"' + (p.page > 0 ? '' : ' disabled') + '>‹</button>' +
    '<button aria-label="Next page"' + (p.page + 1 < p.pages ? '' : ' disabled') + '>›</button></nav>';
}

export function renderPage(vm) {
  let h = '';
  if (vm.title) {
    h += '<header><h1>' + esc(vm.title) + '</h1>';
    if (vm.refresh) {
      h += '<button aria-label="' + esc(vm.refresh.ariaLabel) + '"' + (vm.refresh.disabled ? ' disabled' : '') + '>' +
        esc(vm.refresh.label) + '</button>';
    }
    h += '</header>';
  }
  for (let i = 0; i < vm.items.length; i++) {
    const it = vm.items[i];
    if (it.t === 'loader') h += '<div data-testid="loader">' + esc(it.title) + '</div>';
    else if (it.t === 'pager') h += renderPager(it);
    else h += renderSection(it);
  }
  return h;
}

/** Visible text of rendered HTML (tags stripped, entities decoded). */
export function textContent(html) {
  return html
    .replace(/<[^>]*>/g, ' ')
    .replace(/&lt;/g, '<')
    .replace(/&gt;/g, '>')
    .replace(/&quot;/g, '"')
    .replace(/&amp;/g, '&')
    .replace(/\s+/g, ' ')
    .trim();
}
