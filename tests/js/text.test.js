/**
 * Terminal renderer (src/view/text.js) — the third renderer of the view IR.
 */
import { renderText, sparkline, textSection, textValue } from '../../src/view/text.js';
import { podDetailView } from '../../src/view/pages/details.js';
import { nodesView } from '../../src/view/pages/nodes.js';
import { bar, kv, lines, row, section, status, table } from '../../src/view/ir.js';
import { NOW, makeContext, makeGpuNode, makeGpuPod } from './fixtures.js';

describe('text renderer', () => {
  it('renders statuses with a marker and optional ANSI colour', () => {
    expect(textValue(status('success', 'Ready'))).toBe('✓ Ready');
    expect(textValue(status('error', 'Failed'), true)).toBe('\u001b[31m✗ Failed\u001b[0m');
  });
  it('renders bars as a 10-cell gauge plus their text', () => {
    expect(textValue(bar(6, 8, 75, '#f57c00', '6/8 (75%)'))).toBe('[########..] 6/8 (75%)');
    expect(textValue(bar(1, 0, null, '#000', '1 W'))).toBe('1 W');
  });
  it('aligns name/value rows and table columns (ANSI escapes take no width)', () => {
    const s = section('T', [kv([row('a', '1'), row('longer', '2')]), table(['Col', 'X'], [[status('warning', 'w'), 'yy']])]);
    const out = textSection(s, true);
    expect(out[0]).toBe('T');
    expect(out[2]).toBe('  a       1');
    expect(out[3]).toBe('  longer  2');
    expect(out[4]).toBe('  Col  X ');
    expect(out[6].replace(/\u001b\[[0-9;]*m/g, '')).toBe('  ! w  yy');
  });
  it('renders multi-line cells on one line', () => {
    expect(textValue(lines([{ label: 'a', text: '1' }, { label: '', text: '2' }]))).toBe('a: 1; 2');
  });
  it('renders a whole page: title, sections, GPU strip and xGMI grid', () => {
    const vm = nodesView(makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('p', { node: 'g0', gpus: 2 })] }), { now: NOW });
    const t = renderText(vm);
    expect(t.indexOf('# AMD GPU — Nodes')).toBe(0);
    expect(t).toContain('GPU Node Summary');
    expect(t).toContain('0:p  1:p  2:-');
    expect(t).toContain('xGMI topology (assumed MI355X full mesh) — full mesh, 7 links/GPU');
    expect(t).toContain('    GPU 0    -   x   x');
  });
  it('renders detail sections', () => {
    expect(textSection(podDetailView(makeGpuPod('q')))[0]).toBe('AMD GPU Resources');
  });
  it('draws power history as a sparkline scaled to the window', () => {
    expect(sparkline([0, 1, 2, 3, 4, 5, 6, 7], 8)).toBe('▁▂▃▄▅▆▇█');
    expect(sparkline([5, 5, 5], 8)).toBe('▄▄▄'); // flat: mid-height, one cell per sample
    expect(sparkline([], 8)).toBe('');
    expect(sparkline([1, null, 'x', 3], 8)).toBe('▁█'); // non-numbers skipped
    const long = [];
    for (let i = 0; i < 120; i++) long.push(i < 60 ? 100 : 1400);
    const s = sparkline(long, 32);
    expect([...s]).toHaveLength(32);
    expect(s[0]).toBe('▁');
    expect(s[s.length - 1]).toBe('█');
    const lines = textSection(section('h', [{ t: 'series', power: { n0: [[0, 600], [30, 1200], [60, 900]] }, avgPower: { n0: 900 } }]));
    expect(lines[2]).toBe('  n0: 3 power samples, last 900 W, avg 900 W  ▁█▅');
  });
});
