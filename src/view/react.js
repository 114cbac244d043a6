/**
 * IR → React elements: the plugin's whole presentation layer, written
 * against an INJECTED React (createElement / memo / Fragment) and an
 * injected map of Headlamp CommonComponents, so it runs unchanged under the
 * real React inside Headlamp and under the Node-12 test harness's stand-in
 * (tests/js/stubs/react.js). No JSX: the file needs no transpiler.
 *
 * One IR node → one component (src/view/ir.js; typed in ir.d.ts):
 *   page     → SectionHeader + refresh <button aria-label> + items
 *   loader   → Loader
 *   section  → SectionBox (memoised: unchanged section IR is not re-rendered)
 *   kv       → NameValueTable
 *   table    → SimpleTable (one getter per column reading row[i])
 *   pctbar   → PercentageBar
 *   status   → StatusLabel
 *   bar      → inline allocation / power bar (reference NodesPage.tsx:35-63,
 *              MetricsPage.tsx:50-89)
 *   slots    → per-GPU allocation strip (MI355X, new)
 *   matrix   → xGMI neighbour matrix (MI355X, new)
 *   series   → inline SVG sparklines of per-node power / HBM (new)
 *   pager    → name filter + "Showing 1–16 of N" + previous / next (page item)
 *
 * Only CommonComponents plus inline-styled elements are used, like the
 * reference (reference CLAUDE.md conventions; src/components/NodesPage.tsx:35-63
 * for the inline bar idiom).
 */

import { BAR_COLORS, formatWatts } from '../api/k8sCore.js';
import { matrixCaption, pagerText } from './ir.js';

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

const MUTED = { fontSize: '13px', marginBottom: '6px', color: 'var(--mui-palette-text-secondary)' };

/** Style of the page refresh button (disabled while a refresh is in flight). */
export function buttonStyle(disabled) {
  return {
    padding: '6px 16px',
    backgroundColor: 'transparent',
    color: 'var(--mui-palette-primary-main, #ed1c24)',
    border: '1px solid var(--mui-palette-primary-main, #ed1c24)',
    borderRadius: '4px',
    cursor: disabled ? 'not-allowed' : 'pointer',
    fontSize: '13px',
    fontWeight: 500,
    opacity: disabled ? 0.6 : 1,
  };
}

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

  function InlineBar(props) {
    const track = props.pct === null
      ? null
      : h(
        'div',
        { style: { width: '100px', height: '8px', backgroundColor: BAR_COLORS.track, borderRadius: '4px', overflow: 'hidden', flexShrink: 0 } },
        h('div', {
          'data-pct': props.pct,
          style: { width: props.pct + '%', height: '100%', backgroundColor: props.color, borderRadius: '4px', transition: 'width 0.4s ease' },
        })
      );
    return h(
      'div',
      { style: { display: 'flex', alignItems: 'center', gap: '8px' } },
      track,
      h('span', { style: { fontSize: '12px', fontVariantNumeric: 'tabular-nums' } }, props.text)
    );
  }

  /** One table / name-value cell. */
  function Value(props) {
    const v = props.v;
    if (v === null || v === undefined) return null;
    if (typeof v === 'string' || typeof v === 'number') return String(v);
    switch (v.t) {
      case 'status':
        return h(CC.StatusLabel, { status: v.status }, v.text);
      case 'bar':
        return h(InlineBar, { pct: v.pct, color: v.color, text: v.text });
      case 'lines':
        return h(
          Fragment,
          null,
          v.lines.map(function (l, i) {
            return h(
              'div',
              { key: i, style: { marginBottom: '2px', fontSize: '13px' } },
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

  function Slots(props) {
    const b = props.b;
    const cols = Math.min(8, b.partitionsPerGpu > 1 ? b.partitionsPerGpu : 8);
    return h(
      'div',
      { style: { marginTop: '12px' } },
      h('div', { style: MUTED }, 'Per-GPU allocation' + (b.exact ? '' : ' (inferred from pod order — exporter pod labels unavailable)')),
      h(
        'div',
        { style: { display: 'grid', gridTemplateColumns: 'repeat(' + cols + ', minmax(0, 1fr))', gap: '4px' } },
        b.slots.map(function (s) {
          const label = s.partition === null || s.partition === undefined ? 'GPU ' + s.index : 'GPU ' + s.board + '·' + s.partition;
          return h(
            'div',
            {
              key: s.index,
              'data-slot': s.index,
              title: s.pod ? (s.namespace ? s.namespace + '/' : '') + s.pod : 'free',
              style: {
                padding: '6px 4px', borderRadius: '4px', fontSize: '11px', textAlign: 'center', overflow: 'hidden',
                textOverflow: 'ellipsis', whiteSpace: 'nowrap', color: s.pod ? '#fff' : 'inherit',
                backgroundColor: s.pod ? BAR_COLORS.ok : BAR_COLORS.track, opacity: s.inferred ? 0.8 : 1,
              },
            },
            label,
            h('br', null),
            s.pod || 'free'
          );
        })
      )
    );
  }

  function Matrix(props) {
    const b = props.b;
    const m = b.matrix;
    const cell = { padding: '2px 6px' };
    return h(
      'div',
      { style: { marginTop: '12px', overflowX: 'auto' } },
      h('div', { style: MUTED }, matrixCaption(b)),
      h(
        'table',
        { style: { borderCollapse: 'collapse', fontSize: '11px' } },
        h('thead', null, h('tr', null, h('th', null), m.cells.map(function (_, j) { return h('th', { key: j, style: cell }, 'GPU ' + j); }))),
        h(
          'tbody',
          null,
          m.cells.map(function (rowCells, i) {
            return h(
              'tr',
              { key: i },
              h('th', { style: { padding: '2px 6px', textAlign: 'right' } }, 'GPU ' + i),
              rowCells.map(function (c, j) {
                const txt = c.kind === 'self' ? '—' : c.measuredGBs !== null ? c.measuredGBs.toFixed(0) : c.kind === 'xgmi' ? '•' : c.kind;
                return h(
                  'td',
                  {
                    key: j,
                    title: c.kind === 'xgmi' ? c.hops + ' hop · ' + c.peakGBs + ' GB/s peak' : c.kind,
                    style: {
                      padding: '2px 6px', textAlign: 'center', border: '1px solid var(--mui-palette-divider, #e0e0e0)',
                      backgroundColor: matrixCellColor(c),
                    },
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
      return { label: label, getter: function (r) { return h(Value, { v: r[i] }); } };
    });
  }

  function Block(props) {
    const b = props.b;
    switch (b.t) {
      case 'kv':
        return h(CC.NameValueTable, {
          rows: b.rows.map(function (r) { return { name: r.name, value: h(Value, { v: r.value }) }; }),
        });
      case 'table':
        return h(CC.SimpleTable, { columns: tableColumns(b), data: b.rows });
      case 'pctbar':
        return h(
          'div',
          { style: { marginBottom: '16px' } },
          h('div', { style: { marginBottom: '8px', fontSize: '14px', color: 'var(--mui-palette-text-secondary)' } }, b.label),
          h(CC.PercentageBar, { data: b.data, total: b.total })
        );
      case 'slots':
        return h(Slots, { b: b });
      case 'matrix':
        return h(Matrix, { b: b });
      case 'series':
        return h(Series, { b: b });
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
      s.blocks.map(function (b, i) { return h(Block, { key: i, b: b }); })
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
    const prev = p.page > 0;
    const next = p.page + 1 < p.pages;
    return h(
      'div',
      { 'data-pager': p.label || p.noun, style: { display: 'flex', alignItems: 'center', gap: '8px', flexWrap: 'wrap', margin: '0 0 16px' } },
      h('input', {
        'aria-label': 'Filter ' + (p.label || p.noun) + ' by name',
        placeholder: 'Filter by name',
        value: p.filter,
        style: { padding: '4px 6px', fontSize: '13px', minWidth: '180px' },
        onChange: function (e) { if (props.onFilter) props.onFilter(e.target.value); },
      }),
      p.sorts
        ? h(
          'select',
          {
            'aria-label': 'Sort ' + (p.label || p.noun),
            value: p.sort,
            style: { padding: '4px 6px', fontSize: '13px' },
            onChange: function (e) { if (props.onSort) props.onSort(e.target.value); },
          },
          p.sorts.map(function (o) { return h('option', { key: o.value, value: o.value }, o.label); })
        )
        : null,
      h('span', { style: { fontSize: '13px', color: 'var(--mui-palette-text-secondary)' } }, pagerText(p)),
      h('button', {
        'aria-label': 'Previous page', disabled: !prev, style: buttonStyle(!prev),
        onClick: function () { if (prev && props.onPage) props.onPage(p.page - 1); },
      }, '‹ Prev'),
      h('button', {
        'aria-label': 'Next page', disabled: !next, style: buttonStyle(!next),
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
        { style: { display: 'flex', justifyContent: 'space-between', alignItems: 'center', marginBottom: '20px' } },
        h(CC.SectionHeader, { title: vm.title }),
        vm.refresh
          ? h(
            'button',
            {
              onClick: function () { if (onRefresh) onRefresh(); },
              disabled: vm.refresh.disabled,
              'aria-label': vm.refresh.ariaLabel,
              style: buttonStyle(vm.refresh.disabled),
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
