/**
 * View IR → plain text for terminals (bin/amd-gpu-dash.js).
 *
 * The third renderer of the same IR (after View.tsx and html.js): sections
 * become underlined titles, name/value tables aligned "name  value" lines,
 * tables fixed-width columns, bars "[#####.....] 6/8 (75%)", statuses a
 * marker (✓ ! ✗) before the text, the per-GPU strip one line per board and
 * the xGMI matrix a small grid, power history a sparkline. Optional ANSI
 * colour for statuses.
 */

import { matrixCaption, pagerText } from './ir.js';

/** " · sorted by <label>" for a pager ranked other than by name. */
function sortText(p) {
  if (!p.sorts || !p.sort || p.sort === p.sorts[0].value) return '';
  for (let i = 0; i < p.sorts.length; i++) if (p.sorts[i].value === p.sort) return ' · sorted: ' + p.sorts[i].label;
  return '';
}

const MARK = { success: '✓', warning: '!', error: '✗' };
const ANSI = { success: '\u001b[32m', warning: '\u001b[33m', error: '\u001b[31m', reset: '\u001b[0m' };

/** Pad to `w` printable characters (ANSI colour escapes take no columns). */
function pad(s, w) {
  s = String(s);
  const n = [...s.replace(/\u001b\[[0-9;]*m/g, '')].length;
  return n >= w ? s : s + ' '.repeat(w - n);
}

function barText(p, width) {
  if (p === null || p === undefined) return '';
  const k = Math.max(0, Math.min(width, Math.round((p / 100) * width)));
  return '[' + '#'.repeat(k) + '.'.repeat(width - k) + '] ';
}

const SPARK = '▁▂▃▄▅▆▇█';

/**
 * Values as a sparkline of at most `width` characters: consecutive samples
 * are averaged into buckets, each bucket drawn by its height between the
 * window's min and max (a flat series is drawn mid-height). Non-numbers skip.
 */
export function sparkline(values, width) {
  const v = (values || []).filter(function (x) { return typeof x === 'number' && isFinite(x); });
  if (!v.length) return '';
  const w = Math.max(1, Math.min(width || 32, v.length));
  const buckets = [];
  for (let i = 0; i < w; i++) {
    const a = Math.floor((i * v.length) / w);
    const b = Math.max(a + 1, Math.floor(((i + 1) * v.length) / w));
    let sum = 0;
    for (let k = a; k < b; k++) sum += v[k];
    buckets.push(sum / (b - a));
  }
  const lo = Math.min.apply(null, buckets);
  const hi = Math.max.apply(null, buckets);
  return buckets.map(function (x) {
    const k = hi > lo ? Math.round(((x - lo) / (hi - lo)) * (SPARK.length - 1)) : 3;
    return SPARK[k];
  }).join('');
}

/** One IR cell/value as a single line of text. */
export function textValue(v, color) {
  if (v === null || v === undefined) return '';
  if (typeof v === 'string' || typeof v === 'number') return String(v);
  switch (v.t) {
    case 'status': {
      const s = (MARK[v.status] || '·') + ' ' + v.text;
      return color && ANSI[v.status] ? ANSI[v.status] + s + ANSI.reset : s;
    }
    case 'bar':
      return barText(v.pct, 10) + v.text;
    case 'lines':
      return v.lines.map(function (l) { return (l.label ? l.label + ': ' : '') + l.text; }).join('; ');
    default:
      return '';
  }
}

function blockLines(b, color) {
  const out = [];
  switch (b.t) {
    case 'kv': {
      let w = 0;
      b.rows.forEach(function (r) { w = Math.max(w, [...r.name].length); });
      b.rows.forEach(function (r) { out.push('  ' + pad(r.name, w) + '  ' + textValue(r.value, color)); });
      break;
    }
    case 'table': {
      const cells = b.rows.map(function (r) { return r.map(function (c) { return textValue(c, color); }); });
      const widths = b.columns.map(function (c, i) {
        let w = [...c].length;
        cells.forEach(function (r) { w = Math.max(w, [...String(r[i]).replace(/\u001b\[[0-9;]*m/g, '')].length); });
        return Math.min(w, 48);
      });
      out.push('  ' + b.columns.map(function (c, i) { return pad(c, widths[i]); }).join('  '));
      out.push('  ' + widths.map(function (w) { return '-'.repeat(w); }).join('  '));
      cells.forEach(function (r) { out.push('  ' + r.map(function (c, i) { return pad(c, widths[i]); }).join('  ')); });
      break;
    }
    case 'pctbar': {
      const parts = b.data.map(function (d) { return d.name + ' ' + d.value; }).join(', ');
      out.push('  ' + b.label + ': ' + parts + (b.total ? ' (of ' + b.total + ')' : ''));
      break;
    }
    case 'slots': {
      const per = b.partitionsPerGpu > 1 ? b.partitionsPerGpu : 8;
      out.push('  Per-GPU allocation' + (b.exact ? '' : ' (inferred)') + ':');
      for (let i = 0; i < b.slots.length; i += per) {
        out.push('    ' + b.slots.slice(i, i + per).map(function (s) {
          const id = s.partition === null || s.partition === undefined ? String(s.index) : s.board + '.' + s.partition;
          return id + ':' + (s.pod || '-');
        }).join('  '));
      }
      break;
    }
    case 'matrix': {
      const m = b.matrix;
      out.push('  ' + matrixCaption(b));
      m.cells.forEach(function (row, i) {
        out.push('    ' + pad('GPU ' + i, 6) + row.map(function (c) {
          const v = c.kind === 'self' ? (c.measuredGBs !== null ? 'S' + Math.round(c.measuredGBs) : '-') : c.measuredGBs !== null ? String(Math.round(c.measuredGBs))
            : c.kind === 'xgmi' ? 'x' : '.';
          return ' '.repeat(Math.max(1, 4 - v.length)) + v; // right-aligned, 4 columns per cell
        }).join(''));
      });
      break;
    }
    case 'series': {
      Object.keys(b.power || {}).forEach(function (n) {
        const pts = b.power[n];
        const last = pts.length ? pts[pts.length - 1][1] : null;
        const avg = b.avgPower && b.avgPower[n] !== undefined ? ', avg ' + b.avgPower[n].toFixed(0) + ' W' : '';
        const spark = sparkline(pts.map(function (p) { return p[1]; }), 32);
        out.push('  ' + n + ': ' + pts.length + ' power samples' + (last === null ? '' : ', last ' + last.toFixed(0) + ' W') + avg +
          (spark ? '  ' + spark : ''));
      });
      break;
    }
    default:
      break;
  }
  return out;
}

/** A section as text lines (title underlined). */
export function textSection(s, color) {
  if (!s) return [];
  const out = [s.title, '='.repeat([...s.title].length)];
  s.blocks.forEach(function (b) { out.push.apply(out, blockLines(b, color)); });
  return out;
}

/** A page view-model as one string. */
export function renderText(vm, opts) {
  const color = !!(opts && opts.color);
  const out = [];
  if (vm.title) out.push('# ' + vm.title, '');
  vm.items.forEach(function (it) {
    if (it.t === 'loader') out.push('… ' + it.title, '');
    else if (it.t === 'pager') out.push('[' + pagerText(it) + sortText(it) + ']', '');
    else out.push.apply(out, textSection(it, color).concat(['']));
  });
  return out.join('\n');
}
