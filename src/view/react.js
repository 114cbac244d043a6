/**
 * IR → React elements: the plugin's whole presentation layer, written
 * against an INJECTED React (createElement / memo / Fragment) and an
 * injected map of Headlamp CommonComponents, so it runs unchanged under the
 * real React inside Headlamp and under the Node-12 test harness's stand-in
 * (tests/js/stubs/react.js). No JSX: the file needs no transpiler.
 *
 * IR nodes → React (src/view/ir.js; typed in ir.d.ts):
 *   page     → SectionHeader + refresh <button aria-label> + items
 *   loader   → Loader
 *   section  → SectionBox (memoised: unchanged section IR is not re-rendered)
 *   kv       → NameValueTable
 *   table    → SimpleTable (one getter per column reading row[i])
 *   pctbar   → PercentageBar
 *   status   → StatusLabel
 *   bar      → one element: the bar is its background, the text its content
 *              (reference NodesPage.tsx:35-63, MetricsPage.tsx:50-89)
 *   slots    → per-GPU allocation strip, one element (MI355X, new)
 *   matrix   → xGMI neighbour matrix: a summary line with the grid one click
 *              away when built closed (MI355X, new)
 *   series   → inline SVG sparklines of per-node power / HBM (new)
 *   pager    → name filter + "Showing 1–16 of N" + previous / next (page
 *              item); a count line and one button while it has nothing to do
 * Cells and blocks are built inline (valueNode / blockNode), not as a
 * component each; the matrix and the pager, which keep state, are components.
 *
 * Only CommonComponents and plain elements are used, like the reference
 * (reference CLAUDE.md conventions). The plain elements take their styles
 * from one stylesheet (PLUGIN_CSS, added once per document) rather than an
 * inline style object each, except a bar's or strip's background.
 */

import { BAR_COLORS, formatWatts } from '../api/k8sCore.js';
import { matrixCaption, matrixCellText, matrixLine, pagerIdle, pagerText, slotOwner, slotsText } from './ir.js';

/** CommonComponents the renderer needs (reference src/components/OverviewPage.tsx:8-16). */
export const REQUIRED_COMPONENTS = [
  'Loader',
  'NameValueTable',
  'PercentageBar',
  'SectionBox',
  'SectionHeader',
  'SimpleTable',
  'StatusLabel',
];

/**
 * The renderer's own styles, as classes of one stylesheet added to the
 * document once (ensureStyles) instead of a style object on every element:
 * a page mounts a few hundred elements, and react-dom sets an inline style
 * property by property on each. Colours follow Headlamp's MUI theme through
 * its CSS variables, as the inline styles did.
 */
export const PLUGIN_CSS = [
  '.amdgpu-btn{padding:6px 16px;background-color:transparent;color:var(--mui-palette-primary-main,#ed1c24);' +
    'border:1px solid var(--mui-palette-primary-main,#ed1c24);border-radius:4px;cursor:pointer;font-size:13px;font-weight:500}',
  '.amdgpu-btn:disabled{cursor:not-allowed;opacity:.6}',
  '.amdgpu-head{display:flex;justify-content:space-between;align-items:center;margin-bottom:20px}',
  '.amdgpu-num{font-size:12px;font-variant-numeric:tabular-nums}',
  '.amdgpu-bar{display:inline-block;padding-left:108px;line-height:16px;background-size:100px 8px;' +
    'background-repeat:no-repeat;background-position:left center;font-size:12px;font-variant-numeric:tabular-nums}',
  '.amdgpu-line{margin-bottom:2px;font-size:13px}',
  '.amdgpu-muted{font-size:13px;margin-bottom:6px;color:var(--mui-palette-text-secondary)}',
  '.amdgpu-slots{margin-top:12px;padding-top:18px;font-size:12px;background-size:100% 12px;background-repeat:no-repeat;' +
    'background-position:left top}',
  '.amdgpu-mx{margin-top:12px;overflow-x:auto}',
  '.amdgpu-mx-closed{display:block;margin-top:12px;padding:0;border:0;background:none;font:inherit;font-size:13px;text-align:left;' +
    'cursor:pointer;color:var(--mui-palette-text-secondary)}',
  '.amdgpu-mx table{border-collapse:collapse;font-size:11px}',
  '.amdgpu-mx th{padding:2px 6px}',
  '.amdgpu-mx tbody th{text-align:right}',
  '.amdgpu-mx td{padding:2px 6px;text-align:center;border:1px solid var(--mui-palette-divider,#e0e0e0)}',
  '.amdgpu-pct{margin-bottom:16px}',
  '.amdgpu-pct-label{margin-bottom:8px;font-size:14px;color:var(--mui-palette-text-secondary)}',
  '.amdgpu-pager{display:flex;align-items:center;gap:8px;flex-wrap:wrap;margin:0 0 16px}',
  '.amdgpu-pager input{padding:4px 6px;font-size:13px;min-width:180px}',
  '.amdgpu-pager select{padding:4px 6px;font-size:13px}',
  '.amdgpu-pager span{font-size:13px;color:var(--mui-palette-text-secondary)}',
  '.amdgpu-count{margin:0 0 16px;font-size:13px;color:var(--mui-palette-text-secondary)}',
].join('\n');

const styledDocuments = typeof WeakSet === 'function' ? new WeakSet() : null;

/**
 * Add PLUGIN_CSS to `doc` (default: the global document) once; nothing
 * without a DOM (the harness React, server-side HTML). Returns true when the
 * document holds the stylesheet.
 */
export function ensureStyles(doc) {
  const d = doc || (typeof document !== 'undefined' ? document : null);
  if (!d || !d.head || typeof d.createElement !== 'function' || !styledDocuments) return false;
  if (styledDocuments.has(d)) return true;
  const el = d.createElement('style');
  el.setAttribute('data-amdgpu-styles', '');
  el.textContent = PLUGIN_CSS;
  d.head.appendChild(el);
  styledDocuments.add(d);
  return true;
}

/** Class of the refresh / pager / matrix buttons (PLUGIN_CSS: `:disabled` dims it). */
export const BUTTON_CLASS = 'amdgpu-btn';

/** SVG path of a sparkline over `points` ([t, v] pairs) in a w×h box; null below 2 points. */
export function sparklinePath(points, w, h) {
  if (!points || points.length < 2) return null;
  const t0 = points[0][0];
  const t1 = points[points.length - 1][0];
  let lo = Infinity;
  let hi = -Infinity;
  for (let i = 0; i < points.length; i++) {
    if (points[i][1] < lo) lo = points[i][1];
    if (points[i][1] > hi) hi = points[i][1];
  }
  const span = hi - lo || 1;
  const dt = t1 - t0 || 1;
  let d = '';
  for (let i = 0; i < points.length; i++) {
    const x = ((points[i][0] - t0) / dt) * w;
    const y = h - ((points[i][1] - lo) / span) * h;
    d += (i ? ' L' : 'M') + x.toFixed(1) + ',' + y.toFixed(1);
  }
  return d;
}

/** Inline style of a one-element bar (InlineBar, class amdgpu-bar): `pct` of its 100 × 8 px track in `color`. */
export function barStyle(pct, color) {
  const p = Math.max(0, Math.min(100, pct));
  return { backgroundImage: 'linear-gradient(to right, ' + color + ' ' + p + '%, ' + BAR_COLORS.track + ' ' + p + '%)' };
}

/** Background of a slot strip: one hard-edged segment per slot, held (dimmed when inferred) or free. */
export function slotsGradient(slots) {
  const pos = gradientStops(slots.length);
  let out = 'linear-gradient(to right';
  for (let i = 0; i < slots.length; i++) {
    const s = slots[i];
    const c = s.pod ? (s.inferred ? BAR_COLORS.okInferred : BAR_COLORS.ok) : BAR_COLORS.track;
    out += ', ' + c + pos[i][0] + ', ' + c + pos[i][1] + pos[i][2];
  }
  return out + ')';
}

const stopCache = {};

/** Per slot of an `n`-slot strip: its start, its end less a 1 px gap, and the gap ("transparent …"). */
function gradientStops(n) {
  if (stopCache[n]) return stopCache[n];
  const out = [];
  for (let i = 0; i < n; i++) {
    const a = (100 * i / n).toFixed(3);
    const z = (100 * (i + 1) / n).toFixed(3);
    out.push([' ' + a + '%', ' calc(' + z + '% - 1px)', ', transparent calc(' + z + '% - 1px), transparent ' + z + '%']);
  }
  stopCache[n] = out;
  return out;
}

/** Background of one xGMI matrix cell: measured utilisation shades it, otherwise link kind. */
export function matrixCellColor(c) {
  if (c.kind === 'self') return 'transparent';
  const util = c.measuredGBs !== null && c.peakGBs > 0 ? c.measuredGBs / c.peakGBs : null;
  if (util !== null) return 'rgba(237, 28, 36, ' + (0.15 + 0.85 * Math.min(1, util)).toFixed(3) + ')';
  return c.kind === 'xgmi' ? 'rgba(237, 28, 36, 0.08)' : BAR_COLORS.track;
}

export { matrixCaption };

/**
 * @param {{createElement: Function, memo: Function, Fragment: any}} React
 * @param {Record<string, Function>} CC  Headlamp CommonComponents
 */
export function createRenderer(React, CC) {
  if (!React || typeof React.createElement !== 'function') throw new Error('createRenderer: React is required');
  for (let i = 0; i < REQUIRED_COMPONENTS.length; i++) {
    if (!CC || !CC[REQUIRED_COMPONENTS[i]]) throw new Error('createRenderer: CommonComponents.' + REQUIRED_COMPONENTS[i] + ' is missing');
  }
  const h = React.createElement;
  const Fragment = React.Fragment;
  ensureStyles();

  /**
   * A 100 × 8 px bar and its text as ONE element: the bar is the element's
   * background (a two-stop gradient: fill up to `pct`, track after), drawn in
   * its left padding. A page holds two bars per GPU node row; four DOM nodes
   * each (track, fill, text, wrapper) were a tenth of GPU Nodes' elements.
   */
  function InlineBar(props) {
    return barNode(props.pct, props.color, props.text);
  }

  function barNode(pct, color, text) {
    if (pct === null) return h('span', { className: 'amdgpu-num' }, text);
    return h('span', { className: 'amdgpu-bar', 'data-pct': pct, 'data-color': color, style: barStyle(pct, color) }, text);
  }

  /**
   * One table / name-value cell as React nodes, built inline: a plain string
   * stays a string, and no component instance wraps a cell (a page holds a
   * few hundred cells; a component per cell cost more than the elements).
   */
  function valueNode(v) {
    if (v === null || v === undefined) return null;
    if (typeof v === 'string' || typeof v === 'number') return String(v);
    switch (v.t) {
      case 'status':
        return h(CC.StatusLabel, { status: v.status }, v.text);
      case 'bar':
        return barNode(v.pct, v.color, v.text);
      case 'lines':
        return h(
          Fragment,
          null,
          v.lines.map(function (l, i) {
            return h(
              'div',
              { key: i, className: 'amdgpu-line' },
              l.label ? h('strong', null, l.label) : null,
              l.label ? ': ' : null,
              l.text
            );
          })
        );
      default:
        return null;
    }
  }

  /** One table / name-value cell (valueNode as a component: the Nodes-table columns, tests). */
  function Value(props) {
    return valueNode(props.v);
  }

  /**
   * The per-GPU allocation strip as ONE element: one coloured segment per GPU
   * (or partition) in its background, the owners as text under it ("GPU 0–3
   * ml/train-a · GPU 4–7 free"), each slot's owner in `data-slots`.
   */
  function Slots(props) {
    return slotsNode(props.b);
  }

  function slotsNode(b, key) {
    const caption = 'Per-GPU allocation' + (b.exact ? '' : ' (inferred from pod order — exporter pod labels unavailable)');
    return h(
      'div',
      {
        key: key,
        'data-slots': b.slots.map(slotOwner).join(','),
        title: caption,
        className: 'amdgpu-slots',
        style: { backgroundImage: slotsGradient(b.slots) },
      },
      slotsText(b.slots) + (b.exact ? '' : ' (inferred)')
    );
  }

  /**
   * The xGMI matrix: its caption and summary line, and the 8 × 8 grid when
   * open. A block built closed (a GPU Nodes card) opens on click; the state
   * stays with the mounted section.
   */
  function Matrix(props) {
    const b = props.b;
    const st = React.useState(b.open !== false);
    const open = st[0];
    const setOpen = st[1];
    const flip = function () { setOpen(!open); };
    if (!open) {
      // Closed (a GPU Nodes card): the summary line is itself the toggle — one element.
      return h('button', {
        'data-matrix': 'closed', 'aria-expanded': 'false', className: 'amdgpu-mx-closed', onClick: flip,
      }, matrixLine(b) + ' · Show xGMI matrix');
    }
    const toggle = h('button', { 'aria-expanded': 'true', className: BUTTON_CLASS, onClick: flip }, 'Hide xGMI matrix');
    const m = b.matrix;
    return h(
      'div',
      { 'data-matrix': 'open', className: 'amdgpu-mx' },
      h('div', { className: 'amdgpu-muted' }, matrixLine(b) + ' ', toggle),
      h(
        'table',
        null,
        h('thead', null, h('tr', null, h('th', null), m.cells.map(function (_, j) { return h('th', { key: j }, 'GPU ' + j); }))),
        h(
          'tbody',
          null,
          m.cells.map(function (rowCells, i) {
            return h(
              'tr',
              { key: i },
              h('th', null, 'GPU ' + i),
              rowCells.map(function (c, j) {
                const txt = matrixCellText(c, '•');
                return h(
                  'td',
                  {
                    key: j,
                    title: c.kind === 'xgmi' ? c.hops + ' hop · ' + c.peakGBs + ' GB/s peak'
                      : c.kind === 'self' && c.measuredGBs !== null ? 'GPU ' + i + ' xGMI throughput, all links (GB/s)' : c.kind,
                    style: { backgroundColor: matrixCellColor(c) },
                  },
                  txt
                );
              })
            );
          })
        )
      )
    );
  }

  function Sparkline(props) {
    const w = 240;
    const hh = 36;
    const d = sparklinePath(props.points, w, hh);
    if (d === null) return h('span', null, '—');
    return h(
      'svg',
      { width: w, height: hh, viewBox: '0 0 ' + w + ' ' + hh, role: 'img', 'aria-label': props.label || 'time series' },
      h('path', { d: d, fill: 'none', stroke: props.color, strokeWidth: 1.5 })
    );
  }

  function Series(props) {
    const b = props.b;
    const nodes = Object.keys(b.power || {});
    const hbm = Object.keys(b.vram || {}).length > 0;
    return h(CC.SimpleTable, {
      columns: [
        { label: b.label || 'Node', getter: function (n) { return n; } },
        {
          label: 'Avg Power',
          getter: function (n) { return b.avgPower && b.avgPower[n] !== undefined ? formatWatts(b.avgPower[n]) : '—'; },
        },
        {
          label: 'Power (W)',
          getter: function (n) { return h(Sparkline, { points: b.power[n] || [], color: BAR_COLORS.ok, label: n + ' power' }); },
        },
      ].concat(hbm ? [{
        label: 'HBM in use',
        getter: function (n) { return h(Sparkline, { points: b.vram[n] || [], color: '#6a1b9a', label: n + ' HBM' }); },
      }] : []),
      data: nodes,
    });
  }

  /** Column descriptors of a `table` block: getter i reads cell i of the row array. */
  function tableColumns(b) {
    return b.columns.map(function (label, i) {
      return { label: label, getter: function (r) { return valueNode(r[i]); } };
    });
  }

  function Block(props) {
    return blockNode(props.b);
  }

  /**
   * One IR block as React nodes, built inline (no component of its own; the
   * matrix, which keeps open / closed state, is the one that has one).
   */
  function blockNode(b, key) {
    switch (b.t) {
      case 'kv':
        return h(CC.NameValueTable, {
          key: key,
          rows: b.rows.map(function (r) { return { name: r.name, value: valueNode(r.value) }; }),
        });
      case 'table':
        return h(CC.SimpleTable, { key: key, columns: tableColumns(b), data: b.rows });
      case 'pctbar':
        return h(
          'div',
          { key: key, className: 'amdgpu-pct' },
          h('div', { className: 'amdgpu-pct-label' }, b.label),
          h(CC.PercentageBar, { data: b.data, total: b.total })
        );
      case 'slots':
        return slotsNode(b, key);
      case 'matrix':
        return h(Matrix, { key: key, b: b });
      case 'series':
        return h(Series, { key: key, b: b });
      default:
        return null;
    }
  }

  function SectionImpl(props) {
    const s = props.s;
    if (!s) return null;
    return h(
      CC.SectionBox,
      { title: s.title },
      s.blocks.map(function (b, i) { return blockNode(b, i); })
    );
  }
  // View-models return the same section object while its inputs are
  // unchanged (pages.js memo + the store's structural sharing), so a memoised
  // Section skips re-rendering the unchanged parts of a page on refresh.
  const Section = React.memo(SectionImpl);

  /**
   * Pager of a long list (GPU nodes): name filter, the range shown and
   * previous / next, and the order when the list offers several (p.sorts).
   * The page component owns the state (props.onPage / onFilter / onSort);
   * without handlers the controls are inert.
   */
  function Pager(props) {
    const p = props.p;
    const shown = React.useState(false);
    // Nothing to control (ir.js pagerIdle): the count line and one button
    // that brings up the filter box and the order menu.
    if (pagerIdle(p) && !shown[0]) {
      return h('div', { 'data-pager': p.label || p.noun, 'data-idle': 'true', className: 'amdgpu-count' }, pagerText(p) + ' ',
        h('button', {
          'aria-label': 'Filter or sort ' + (p.label || p.noun), className: BUTTON_CLASS,
          onClick: function () { shown[1](true); },
        }, p.sorts ? 'Filter / sort' : 'Filter'));
    }
    const prev = p.page > 0;
    const next = p.page + 1 < p.pages;
    return h(
      'div',
      { 'data-pager': p.label || p.noun, className: 'amdgpu-pager' },
      h('input', {
        'aria-label': 'Filter ' + (p.label || p.noun) + ' by name',
        placeholder: 'Filter by name',
        value: p.filter,
        onChange: function (e) { if (props.onFilter) props.onFilter(e.target.value); },
      }),
      p.sorts
        ? h(
          'select',
          {
            'aria-label': 'Sort ' + (p.label || p.noun),
            value: p.sort,
            onChange: function (e) { if (props.onSort) props.onSort(e.target.value); },
          },
          p.sorts.map(function (o) { return h('option', { key: o.value, value: o.value }, o.label); })
        )
        : null,
      h('span', null, pagerText(p)),
      h('button', {
        'aria-label': 'Previous page', disabled: !prev, className: BUTTON_CLASS,
        onClick: function () { if (prev && props.onPage) props.onPage(p.page - 1); },
      }, '‹ Prev'),
      h('button', {
        'aria-label': 'Next page', disabled: !next, className: BUTTON_CLASS,
        onClick: function () { if (next && props.onPage) props.onPage(p.page + 1); },
      }, 'Next ›')
    );
  }

  function Page(props) {
    const vm = props.vm;
    const onRefresh = props.onRefresh;
    const header = vm.title
      ? h(
        'div',
        { className: 'amdgpu-head' },
        h(CC.SectionHeader, { title: vm.title }),
        vm.refresh
          ? h(
            'button',
            {
              onClick: function () { if (onRefresh) onRefresh(); },
              disabled: vm.refresh.disabled,
              'aria-label': vm.refresh.ariaLabel,
              className: BUTTON_CLASS,
            },
            vm.refresh.label
          )
          : null
      )
      : null;
    return h(
      Fragment,
      null,
      header,
      vm.items.map(function (it, i) {
        if (it.t === 'loader') return h(CC.Loader, { key: 'loader-' + i, title: it.title });
        if (it.t === 'pager') return h(Pager, { key: 'pager', p: it, onPage: props.onPage, onFilter: props.onFilter, onSort: props.onSort });
        return h(Section, { key: it.key || i, s: it });
      })
    );
  }

  return {
    Value: Value,
    valueNode: valueNode,
    InlineBar: InlineBar,
    Slots: Slots,
    Matrix: Matrix,
    Sparkline: Sparkline,
    Series: Series,
    Block: Block,
    Section: Section,
    SectionImpl: SectionImpl,
    Pager: Pager,
    Page: Page,
  };
}
