/**
 * src/view/svg.js — the IR drawn as a static SVG (docs/screenshots/*.svg,
 * ArtifactHub's `screenshots:`): text layout in a fixed-advance face, every
 * block type, escaping, and output that depends on the IR alone.
 */
import { bar, kv, lines, loader, page, pager, pctbar, row, section, status, table } from '../../src/view/ir.js';
import { columnWidths, renderPageSvg, renderSectionSvg, SVG_WIDTH, wrap, xml } from '../../src/view/svg.js';
import { matrixBlock } from '../../src/view/pages/nodes.js';

function texts(svg) {
  const out = [];
  const re = /<text[^>]*>([^<]*)<\/text>/g;
  let m;
  while ((m = re.exec(svg))) out.push(m[1]);
  return out;
}

function count(svg, tag) {
  return (svg.match(new RegExp('<' + tag + '[ >]', 'g')) || []).length;
}

describe('text layout', () => {
  it('wrap breaks at spaces within the width, and hard-breaks a longer word', () => {
    expect(wrap('a bb ccc dddd', 6)).toEqual(['a bb', 'ccc', 'dddd']);
    expect(wrap('abcdefghij', 4)).toEqual(['abcd', 'efgh', 'ij']);
    expect(wrap('', 10)).toEqual(['']);
    expect(wrap('ab', 0)).toEqual(['a', 'b']); // a width below one character still makes progress
    // counted in code points, not UTF-16 units
    expect(wrap('°C °C °C', 5)).toEqual(['°C °C', '°C']);
  });

  it('xml escapes markup characters', () => {
    expect(xml('a < b & "c" > d')).toBe('a &lt; b &amp; &quot;c&quot; &gt; d');
  });

  it('columnWidths: each column as wide as its widest cell, the widest giving way when the table is too wide', () => {
    expect(columnWidths(['A', 'Name'], [['x', 'long-name'], ['yy', 'n']], 200)).toEqual([2, 9]);
    const w = columnWidths(['A', 'B'], [['a'.repeat(40), 'b'.repeat(40)]], 50);
    expect(w[0] + w[1] + 4).toBeLessThanOrEqual(50);
    // a bar cell counts its drawn track as characters
    const bw = columnWidths(['Power'], [[bar(1, 2, 50, '#000', '1/2')]], 100);
    expect(bw[0]).toBeGreaterThan(3);
  });
});

describe('renderPageSvg', () => {
  const vm = page('AMD GPU — Test', { label: 'Refresh', ariaLabel: 'Refresh test', disabled: false }, [
    pager({ page: 0, pages: 1, from: 0, to: 2, total: 2, matched: 2, filter: '', perPage: 8 }, 'GPU nodes'),
    section('Summary <x>', [
      kv([row('Status', status('success', 'Ready')), row('Note', 'word '.repeat(60).trim()), row('Multi', lines([{ label: 'a', text: '1' }, { label: 'b', text: '2' }]))]),
      table(['Node', 'Allocation'], [['n1', bar(6, 8, 75, '#f57c00', '6/8 (75%)')], ['n2', status('error', 'Not Ready')]]),
      pctbar('Readiness', [{ name: 'Ready', value: 3, fill: '#ed1c24' }, { name: 'Not Ready', value: 1, fill: '#9e9e9e' }], 4),
      { t: 'slots', slots: [0, 1, 2, 3].map((i) => ({ index: i, board: i, partition: null, pod: i < 2 ? 'p' : null, namespace: 'ml', inferred: false })), exact: true, partitionsPerGpu: 1 },
    ]),
    loader('Loading more...'),
  ]);

  it('is a well-formed document sized to what it draws', () => {
    const svg = renderPageSvg(vm);
    expect(svg.startsWith('<svg xmlns="http://www.w3.org/2000/svg" width="' + SVG_WIDTH + '"')).toBe(true);
    expect(svg.trim().endsWith('</svg>')).toBe(true);
    const h = Number(/height="([\d.]+)"/.exec(svg)[1]);
    const ys = [];
    const re = /<(?:rect|text)[^>]* y="([\d.]+)"(?:[^>]* height="([\d.]+)")?/g;
    let m;
    while ((m = re.exec(svg))) ys.push(Number(m[1]) + (m[2] ? Number(m[2]) : 0));
    expect(Math.max.apply(null, ys)).toBeLessThanOrEqual(h);
  });

  it('draws every item: title, refresh, pager text, section, rows, cells, loader', () => {
    const svg = renderPageSvg(vm);
    const t = texts(svg);
    expect(t[0]).toBe('AMD GPU — Test');
    expect(t).toContain('Refresh');
    expect(t).toContain('Showing 1–2 of 2 GPU nodes');
    expect(t).toContain('Summary &lt;x&gt;');
    expect(t).toContain('Ready');
    expect(t).toContain('a: 1');
    expect(t).toContain('b: 2');
    expect(t).toContain('6/8 (75%)');
    expect(t).toContain('Ready 3');
    expect(t.some((x) => x.startsWith('GPU 0–1 ml/p · GPU 2–3 free'))).toBe(true);
    expect(t).toContain('Loading more...');
    // the long note wrapped onto several lines
    expect(t.filter((x) => x.startsWith('word')).length).toBeGreaterThan(1);
    // statuses are dots (2 here), the bar a track and a fill, the strip one box per slot
    expect(count(svg, 'circle')).toBe(2 + 1); // + the loader's spinner
    expect(svg).toContain('fill="#f57c00"');
  });

  it('depends on the IR alone: the same view-model gives the same bytes', () => {
    expect(renderPageSvg(vm)).toBe(renderPageSvg(vm));
  });
});

describe('renderSectionSvg: the xGMI matrix', () => {
  const measured = {};
  for (let i = 0; i < 8; i++) for (let j = 0; j < 8; j++) if (i !== j) measured[i + '-' + j] = i === 2 && j === 3 ? 117 : 0;

  it('closed: the caption and summary with the toggle drawn as a button', () => {
    const svg = renderSectionSvg(section('n1', [matrixBlock(8, measured, null, false)]));
    const t = texts(svg);
    expect(t.join(' ')).toContain('xGMI topology');
    expect(t).toContain('Show xGMI matrix');
    expect(t).not.toContain('GPU 7');
  });

  it('open: the 8 × 8 grid with its headers and measured cells', () => {
    const svg = renderSectionSvg(section('n1', [matrixBlock(8, measured, null, true)]));
    const t = texts(svg);
    expect(t.filter((x) => x === 'GPU 7')).toHaveLength(2); // column and row header
    expect(t).toContain('117');
    // the diagonal: each GPU's xGMI total (GPU 2 sends 117 GB/s, the others nothing)
    expect(t.filter((x) => /^\u03a3/.test(x))).toEqual(['\u03a30', '\u03a30', '\u03a3117', '\u03a30', '\u03a30', '\u03a30', '\u03a30', '\u03a30']);
  });

  it('no measurements: an em dash on the diagonal', () => {
    const t = texts(renderSectionSvg(section('n1', [matrixBlock(8, null, null, true)])));
    expect(t.filter((x) => x === '\u2014')).toHaveLength(8);
  });
});
