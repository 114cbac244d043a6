/**
 * View IR → one static SVG picture (docs/screenshots/*.svg, the ArtifactHub
 * package's `screenshots:`).
 *
 * The fourth renderer of the IR, after react.js, html.js and text.js. The
 * reference publishes hand-drawn SVG mock-ups (artifacthub-pkg.yml:93-99,
 * docs/screenshots/0{1,2,3}-*.svg); these are the plugin's real view-models
 * drawn as text and boxes, so they change when a page does.
 *
 * No browser and no font metrics: text is set in a monospace face, and every
 * width (columns, wrapping, the position of a bar after its label) is counted
 * in characters of a fixed advance (CHAR_W). The output depends on the IR
 * alone, so a re-render on any host gives the same bytes.
 */

import { BAR_COLORS } from '../api/k8sCore.js';
import { matrixCaption, matrixCellText, matrixSummary, pagerText, slotsText } from './ir.js';
import { matrixCellColor, sparklinePath } from './react.js';

export const SVG_WIDTH = 1200;
const PAD = 24;
const INDENT = 16;
const CHAR_W = 7.8; // 13 px monospace advance (0.6 em)
const LINE = 20;
const MAX_COL = 44; // characters a table column may take before its cells are cut

const STATUS_COLORS = { success: '#2e7d32', warning: '#ed6c02', error: '#d32f2f' };

const STYLE =
  'text{font-family:"DejaVu Sans Mono",Menlo,Consolas,monospace;font-size:13px;fill:#212121}' +
  '.h{font-size:20px;font-weight:700}.s{font-size:15px;font-weight:700}.th{font-weight:700}' +
  '.m{fill:#616161}.btn{fill:#ed1c24;font-weight:700}';

/** XML text: & < > " escaped. */
export function xml(s) {
  return String(s).replace(/&/g, '&amp;').replace(/</g, '&lt;').replace(/>/g, '&gt;').replace(/"/g, '&quot;');
}

/** Printable characters of `s` (code points). */
function width(s) {
  return [...String(s)].length;
}

/** `s` cut to `n` characters, "…" marking the cut. */
function clip(s, n) {
  const c = [...String(s)];
  return c.length <= n ? String(s) : c.slice(0, Math.max(0, n - 1)).join('') + '…';
}

/** `s` broken into lines of at most `n` characters, at spaces where it can. */
export function wrap(s, n) {
  n = Math.max(1, Math.floor(n));
  const words = String(s).split(' ');
  const out = [];
  let line = '';
  for (let i = 0; i < words.length; i++) {
    let w = words[i];
    while (width(w) > n) {
      // a word longer than the line: hard breaks
      if (line) {
        out.push(line);
        line = '';
      }
      const c = [...w];
      out.push(c.slice(0, n).join(''));
      w = c.slice(n).join('');
    }
    if (!line) line = w;
    else if (width(line) + 1 + width(w) <= n) line += ' ' + w;
    else {
      out.push(line);
      line = w;
    }
  }
  if (line || !out.length) out.push(line);
  return out;
}

function text(x, y, s, cls) {
  return '<text x="' + num(x) + '" y="' + num(y) + '"' + (cls ? ' class="' + cls + '"' : '') + '>' + xml(s) + '</text>';
}

function rect(x, y, w, h, fill, extra) {
  return '<rect x="' + num(x) + '" y="' + num(y) + '" width="' + num(w) + '" height="' + num(h) + '" fill="' + fill + '"' +
    (extra || '') + '/>';
}

/** Coordinates with at most one decimal (stable text, smaller files). */
function num(v) {
  return String(Math.round(v * 10) / 10);
}

/** A cell's text as the other renderers print it (bars and statuses draw their marks beside it). */
function cellText(v) {
  if (v === null || v === undefined) return '';
  if (typeof v === 'string' || typeof v === 'number') return String(v);
  if (v.t === 'status' || v.t === 'bar') return v.text;
  if (v.t === 'lines') return v.lines.map(function (l) { return (l.label ? l.label + ': ' : '') + l.text; }).join('; ');
  return '';
}

const BAR_W = 60;
const BAR_GAP = 8;

/** Characters a cell needs on one line (a bar's track counts as its width in characters). */
function cellWidth(v) {
  if (v && v.t === 'bar' && v.pct !== null) return width(v.text) + Math.ceil((BAR_W + BAR_GAP) / CHAR_W);
  if (v && v.t === 'status') return width(v.text) + 2;
  if (v && v.t === 'lines') {
    let w = 0;
    for (let i = 0; i < v.lines.length; i++) w = Math.max(w, width((v.lines[i].label ? v.lines[i].label + ': ' : '') + v.lines[i].text));
    return w;
  }
  return width(cellText(v));
}

/** Lines a cell takes in a column of `cols` characters. */
function cellLines(v, cols) {
  if (v && v.t === 'lines') return v.lines.map(function (l) { return clip((l.label ? l.label + ': ' : '') + l.text, cols); });
  return [clip(cellText(v), cols)];
}

/**
 * Draw cell `v` with its first baseline at (x, y) in a column of `cols`
 * characters: a status is a coloured dot before its text, a bar a 60 × 8 px
 * track and fill before its text, a `lines` cell one line per entry.
 */
function drawCell(out, v, x, y, cols) {
  if (v && v.t === 'status') {
    out.push('<circle cx="' + num(x + 4) + '" cy="' + num(y - 4) + '" r="4" fill="' + (STATUS_COLORS[v.status] || '#9e9e9e') + '"/>');
    out.push(text(x + 2 * CHAR_W, y, clip(v.text, cols - 2)));
    return 1;
  }
  if (v && v.t === 'bar' && v.pct !== null) {
    const p = Math.max(0, Math.min(100, v.pct));
    out.push(rect(x, y - 9, BAR_W, 8, BAR_COLORS.track, ' rx="2"'));
    if (p > 0) out.push(rect(x, y - 9, (BAR_W * p) / 100, 8, v.color, ' rx="2"'));
    out.push(text(x + BAR_W + BAR_GAP, y, clip(v.text, cols - Math.ceil((BAR_W + BAR_GAP) / CHAR_W))));
    return 1;
  }
  const ls = cellLines(v, cols);
  for (let i = 0; i < ls.length; i++) out.push(text(x, y + i * LINE, ls[i]));
  return ls.length;
}

/**
 * Column widths (characters) of a table in `avail` characters: each column as
 * wide as its widest cell up to MAX_COL; when the sum is too wide the widest
 * columns give up characters first.
 */
export function columnWidths(columns, rows, avail) {
  const w = columns.map(function (c, i) {
    let m = width(c);
    for (let r = 0; r < rows.length; r++) m = Math.max(m, cellWidth(rows[r][i]));
    return Math.min(m, MAX_COL);
  });
  const gap = 2;
  let total = w.reduce(function (a, b) { return a + b + gap; }, 0);
  while (total > avail) {
    let k = 0;
    for (let i = 1; i < w.length; i++) if (w[i] > w[k]) k = i;
    if (w[k] <= 8) break;
    w[k]--;
    total--;
  }
  return w;
}

/** Draw block `b` at (x, y) in `cols` characters; returns the height used. */
function drawBlock(out, b, x, y, cols) {
  switch (b.t) {
    case 'kv': {
      let nameW = 0;
      b.rows.forEach(function (r) { nameW = Math.max(nameW, width(r.name)); });
      nameW = Math.min(nameW, 30);
      let h = 0;
      b.rows.forEach(function (r) {
        out.push(text(x, y + h + 14, clip(r.name, nameW), 'm'));
        const valueCols = cols - nameW - 2;
        const vx = x + (nameW + 2) * CHAR_W;
        let lines;
        if (typeof r.value === 'string' || typeof r.value === 'number') {
          const ws = wrap(String(r.value), valueCols);
          ws.forEach(function (l, i) { out.push(text(vx, y + h + 14 + i * LINE, l)); });
          lines = ws.length;
        } else {
          lines = drawCell(out, r.value, vx, y + h + 14, valueCols);
        }
        h += lines * LINE + 4;
      });
      return h + 4;
    }
    case 'table': {
      const ws = columnWidths(b.columns, b.rows, cols);
      const xs = [];
      let cx = x;
      for (let i = 0; i < ws.length; i++) {
        xs.push(cx);
        cx += (ws[i] + 2) * CHAR_W;
      }
      const right = Math.min(x + cols * CHAR_W, cx);
      out.push(rect(x - 6, y, right - x + 6, LINE + 6, '#f5f5f5'));
      b.columns.forEach(function (c, i) { out.push(text(xs[i], y + 17, clip(c, ws[i]), 'th')); });
      let h = LINE + 6;
      b.rows.forEach(function (r) {
        let lines = 1;
        r.forEach(function (c, i) { lines = Math.max(lines, drawCell(out, c, xs[i], y + h + 17, ws[i])); });
        h += lines * LINE + 6;
        out.push(rect(x - 6, y + h, right - x + 6, 1, '#e0e0e0'));
      });
      return h + 8;
    }
    case 'pctbar': {
      out.push(text(x, y + 14, b.label, 'm'));
      const W = Math.min(480, cols * CHAR_W);
      const total = b.total > 0 ? b.total : b.data.reduce(function (a, d) { return a + d.value; }, 0);
      let bx = x;
      out.push(rect(x, y + 24, W, 14, BAR_COLORS.track, ' rx="3"'));
      b.data.forEach(function (d) {
        const w = total > 0 ? (W * d.value) / total : 0;
        if (w > 0) out.push(rect(bx, y + 24, w, 14, d.fill));
        bx += w;
      });
      let lx = x;
      b.data.forEach(function (d) {
        out.push(rect(lx, y + 50, 10, 10, d.fill));
        const label = d.name + ' ' + d.value;
        out.push(text(lx + 16, y + 59, label));
        lx += 16 + (width(label) + 3) * CHAR_W;
      });
      return 72;
    }
    case 'slots': {
      const n = b.slots.length;
      const W = Math.min(cols * CHAR_W, 720);
      const sw = n ? W / n : W;
      b.slots.forEach(function (s, i) {
        const fill = s.pod ? (s.inferred ? BAR_COLORS.okInferred : BAR_COLORS.ok) : BAR_COLORS.track;
        out.push(rect(x + i * sw, y + 4, Math.max(1, sw - 2), 14, fill, ' rx="2"'));
      });
      const ls = wrap(slotsText(b.slots) + (b.exact ? '' : ' (inferred)'), cols);
      ls.forEach(function (l, i) { out.push(text(x, y + 36 + i * LINE, l, 'm')); });
      return 28 + ls.length * LINE;
    }
    case 'matrix': {
      const caption = matrixCaption(b) + matrixSummary(b);
      if (b.open === false) {
        const ls = wrap(caption, cols - 20);
        ls.forEach(function (l, i) { out.push(text(x, y + 14 + i * LINE, l, 'm')); });
        const bx = x + (width(ls[ls.length - 1]) + 2) * CHAR_W;
        const label = 'Show xGMI matrix';
        out.push(rect(bx - 6, y + (ls.length - 1) * LINE, (width(label) + 1.5) * CHAR_W, 19, 'none',
          ' stroke="#ed1c24" rx="3"'));
        out.push(text(bx, y + 14 + (ls.length - 1) * LINE, label, 'btn'));
        return ls.length * LINE + 6;
      }
      const ls = wrap(caption, cols);
      ls.forEach(function (l, i) { out.push(text(x, y + 14 + i * LINE, l, 'm')); });
      let h = ls.length * LINE + 6;
      const m = b.matrix;
      const cw = 56;
      for (let j = 0; j < m.size; j++) out.push(text(x + 64 + j * cw, y + h + 14, 'GPU ' + j, 'th'));
      h += LINE;
      m.cells.forEach(function (row, i) {
        out.push(text(x, y + h + 15, 'GPU ' + i, 'th'));
        row.forEach(function (c, j) {
          const fill = matrixCellColor(c);
          out.push(rect(x + 60 + j * cw, y + h, cw - 2, LINE, fill === 'transparent' ? 'none' : fill, ' stroke="#e0e0e0"'));
          const t = matrixCellText(c, '•');
          out.push(text(x + 60 + j * cw + (cw - 2 - width(t) * CHAR_W) / 2, y + h + 15, t));
        });
        h += LINE + 2;
      });
      return h + 6;
    }
    case 'series': {
      let h = 0;
      const nodes = Object.keys(b.power || {});
      const nameW = Math.min(28, nodes.reduce(function (a, n) { return Math.max(a, width(n)); }, width(b.label || 'Node')));
      out.push(text(x, y + 14, b.label || 'Node', 'th'));
      out.push(text(x + (nameW + 2) * CHAR_W, y + 14, 'Avg Power', 'th'));
      out.push(text(x + (nameW + 14) * CHAR_W, y + 14, 'Power (W)', 'th'));
      h += LINE + 6;
      nodes.forEach(function (n) {
        out.push(text(x, y + h + 20, clip(n, nameW)));
        const avg = b.avgPower && b.avgPower[n] !== undefined ? b.avgPower[n].toFixed(0) + ' W' : '—';
        out.push(text(x + (nameW + 2) * CHAR_W, y + h + 20, avg));
        const d = sparklinePath(b.power[n] || [], 240, 28);
        const sx = x + (nameW + 14) * CHAR_W;
        if (d) {
          out.push('<path transform="translate(' + num(sx) + ',' + num(y + h + 2) + ')" d="' + d + '" fill="none" stroke="' +
            BAR_COLORS.ok + '" stroke-width="1.5"/>');
        } else out.push(text(sx, y + h + 20, '—'));
        h += 36;
      });
      return h + 4;
    }
    default:
      return 0;
  }
}

/** Draw section `s` as a bordered card at y; returns its height. */
function drawSection(out, s, y) {
  const body = [];
  const x = PAD + INDENT;
  const cols = Math.floor((SVG_WIDTH - 2 * PAD - 2 * INDENT) / CHAR_W);
  let h = 40;
  s.blocks.forEach(function (b) {
    h += drawBlock(body, b, x, y + h, cols) + 8;
  });
  out.push(rect(PAD, y, SVG_WIDTH - 2 * PAD, h, '#ffffff', ' stroke="#e0e0e0" rx="6"'));
  out.push(text(x, y + 26, s.title, 's'));
  out.push.apply(out, body);
  return h;
}

function svgDocument(out, height, title) {
  return '<svg xmlns="http://www.w3.org/2000/svg" width="' + SVG_WIDTH + '" height="' + num(height) + '" viewBox="0 0 ' +
    SVG_WIDTH + ' ' + num(height) + '" role="img" aria-label="' + xml(title) + '">\n<style>' + STYLE + '</style>\n' +
    rect(0, 0, SVG_WIDTH, height, '#fafafa') + '\n' + out.join('\n') + '\n</svg>\n';
}

/** A page view-model (pages/*.js) as an SVG document. */
export function renderPageSvg(vm) {
  const out = [];
  let y = PAD;
  if (vm.title) {
    out.push(text(PAD, y + 22, vm.title, 'h'));
    if (vm.refresh) {
      const w = (width(vm.refresh.label) + 4) * CHAR_W;
      out.push(rect(SVG_WIDTH - PAD - w, y + 2, w, 28, 'none', ' stroke="#ed1c24" rx="4"'));
      out.push(text(SVG_WIDTH - PAD - w + 2 * CHAR_W, y + 21, vm.refresh.label, 'btn'));
    }
    y += 48;
  }
  vm.items.forEach(function (it) {
    if (it.t === 'loader') {
      out.push('<circle cx="' + (PAD + 8) + '" cy="' + num(y + 10) + '" r="7" fill="none" stroke="#ed1c24" stroke-width="2" ' +
        'stroke-dasharray="30 14"/>');
      out.push(text(PAD + 24, y + 15, it.title, 'm'));
      y += 32;
    } else if (it.t === 'pager') {
      out.push(text(PAD, y + 14, pagerText(it), 'm'));
      y += 28;
    } else {
      y += drawSection(out, it, y) + 16;
    }
  });
  return svgDocument(out, y + PAD - 16, vm.title || 'loading');
}

/** One section (a Node / Pod detail section) as an SVG document. */
export function renderSectionSvg(s) {
  const out = [];
  const h = drawSection(out, s, PAD);
  return svgDocument(out, h + 2 * PAD, s.title);
}
