/**
 * Runner-agnostic specs of the IR → CommonComponents renderer
 * (src/view/react.js): what a user sees and can do — titles, loader, the
 * Refresh button, every block type, the pager — asserted on rendered text,
 * tags, attributes and aria-labels through the 'amd-test-harness' API. They
 * run on the harness React offline and on real React 18 + react-dom in
 * networked CI (see plugin.shared.test.js); the specs on the props each
 * CommonComponent is handed, and on memo skips, stay in tests/js/react.test.js.
 * The CommonComponents are the markup stand-ins the reference's component
 * tests mock them with (reference src/components/OverviewPage.test.tsx:8-61).
 */
import { React, render, tier } from 'amd-test-harness';
import * as CC from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { createRenderer, sparklinePath } from '../../../src/view/react.js';
import { bar, kv, lines, loader, page, pager, pctbar, row, section, status, table } from '../../../src/view/ir.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { matrixBlock, slotsBlock } from '../../../src/view/pages/nodes.js';
import { overviewView } from '../../../src/view/pages/overview.js';
import { nodePage } from '../../../src/view/pages/paging.js';
import { makeContext, makeGpuNode, makeGpuPod } from '../fixtures.js';

const h = React.createElement;
const v = () => createRenderer(React, CC);

describe('shared: Page (' + tier + ')', () => {
  it('renders the title as the page header', () => {
    const r = render(h(v().Page, { vm: page('AMD GPU — Overview', null, []) }));
    expect(r.byTag('h1').map((n) => r.textOf(n))).toEqual(['AMD GPU — Overview']);
    r.unmount();
  });

  it('renders no header while the page is only a loader', () => {
    const r = render(h(v().Page, { vm: page(null, null, [loader('Loading AMD GPU data...')]) }));
    expect(r.byTag('h1')).toHaveLength(0);
    expect(r.byAttr('data-testid').map((n) => r.attr(n, 'data-testid'))).toEqual(['loader']);
    expect(r.text()).toBe('Loading AMD GPU data...');
    r.unmount();
  });

  it('the Refresh button carries its aria-label and calls onRefresh on each click', () => {
    const onRefresh = vi.fn();
    const vm = page('T', { label: 'Refresh', ariaLabel: 'Refresh AMD GPU data', disabled: false }, []);
    const r = render(h(v().Page, { vm, onRefresh }));
    const btn = r.byLabel('Refresh AMD GPU data');
    expect(r.isDisabled(btn)).toBe(false);
    r.click(btn);
    r.click(btn);
    expect(onRefresh).toHaveBeenCalledTimes(2);
    r.unmount();
  });

  it('a disabled Refresh button does not fire and carries the button class (its :disabled style)', () => {
    const onRefresh = vi.fn();
    const vm = page('T', { label: 'Refreshing...', ariaLabel: 'Refresh metrics', disabled: true }, []);
    const r = render(h(v().Page, { vm, onRefresh }));
    const btn = r.byLabel('Refresh metrics');
    expect(r.isDisabled(btn)).toBe(true);
    expect(r.attr(btn, 'class')).toBe('amdgpu-btn');
    r.click(btn);
    expect(onRefresh).not.toHaveBeenCalled();
    r.unmount();
  });

  it('loader and section items render in order', () => {
    const r = render(h(v().Page, { vm: page('T', null, [section('A', []), loader('wait'), section('B', [])]) }));
    expect(r.byTag('h2').map((n) => r.textOf(n))).toEqual(['A', 'B']);
    expect(r.text()).toBe('TAwaitB');
    r.unmount();
  });
});

describe('shared: blocks (' + tier + ')', () => {
  it('kv → name / value rows; a status value carries its status', () => {
    const s = section('Cluster', [kv([row('GPU Nodes', '2'), row('State', status('success', 'Ready'))])]);
    const r = render(h(v().Section, { s }));
    expect(r.byTag('dt').map((n) => r.textOf(n))).toEqual(['GPU Nodes', 'State']);
    expect(r.byTag('dd').map((n) => r.textOf(n))).toEqual(['2', 'Ready']);
    expect(r.byAttr('data-status').map((n) => r.attr(n, 'data-status'))).toEqual(['success']);
    r.unmount();
  });

  it('table → a header row and one row per data row', () => {
    const rows = [['n0', '8'], ['n1', status('warning', '4')]];
    const r = render(h(v().Section, { s: section('Nodes', [table(['Node', 'GPUs'], rows)]) }));
    expect(r.byTag('th').map((n) => r.textOf(n))).toEqual(['Node', 'GPUs']);
    expect(r.byTag('tr')).toHaveLength(3);
    expect(r.byTag('td').map((n) => r.textOf(n))).toEqual(['n0', '8', 'n1', '4']);
    r.unmount();
  });

  it('pctbar → the percentage bar with its total, under its label', () => {
    const data = [{ name: 'Allocated', value: 3, fill: '#f00' }, { name: 'Free', value: 5, fill: '#ccc' }];
    const r = render(h(v().Section, { s: section('Alloc', [pctbar('GPU allocation', data, 8)]) }));
    const bars = r.byAttr('data-total');
    expect(bars.map((n) => r.attr(n, 'data-total'))).toEqual(['8']);
    expect(r.text()).toContain('GPU allocation');
    expect(r.text()).toContain('Allocated: 3');
    r.unmount();
  });

  it('bar cell → one element carrying its percentage and colour, and its text', () => {
    const r = render(h(v().Value, { v: bar(3, 8, 38, '#4caf50', '3/8 (38%)') }));
    const fill = r.byAttr('data-pct');
    expect(fill).toHaveLength(1);
    expect(r.attr(fill[0], 'data-pct')).toBe('38');
    expect(r.attr(fill[0], 'data-color')).toBe('#4caf50');
    expect(r.text()).toBe('3/8 (38%)');
    r.unmount();
  });

  it('bar cell without a percentage draws only the text', () => {
    const r = render(h(v().Value, { v: bar(3, null, null, '#000', '3 GPUs') }));
    expect(r.byAttr('data-pct')).toHaveLength(0);
    expect(r.text()).toBe('3 GPUs');
    r.unmount();
  });

  it('lines cell → one line each, labels in bold', () => {
    const r = render(h(v().Value, { v: lines([{ label: 'trainer', text: '2 GPUs' }, { label: '', text: 'plain' }]) }));
    expect(r.byTag('strong').map((n) => r.textOf(n))).toEqual(['trainer']);
    expect(r.text()).toBe('trainer: 2 GPUsplain');
    r.unmount();
  });

  it('null, strings and numbers render as text; unknown cells and blocks as nothing', () => {
    const V = v();
    const texts = [null, 7, 'x', { t: 'nope' }].map((x) => {
      const r = render(h(V.Value, { v: x }));
      const t = r.text();
      r.unmount();
      return t;
    });
    expect(texts).toEqual(['', '7', 'x', '']);
    const r = render(h(V.Section, { s: section('S', [{ t: 'mystery' }]) }));
    expect(r.text()).toBe('S');
    r.unmount();
  });

  it('slots → one strip: each slot\'s owner, the owners in runs as text, inferred allocation said so', () => {
    const b = slotsBlock(makeGpuNode('mi355x-0'), [makeGpuPod('train-a', { gpus: 2 }), makeGpuPod('train-b', { gpus: 1 })], null);
    const r = render(h(v().Block, { b }));
    const strip = r.byAttr('data-slots');
    expect(strip).toHaveLength(1);
    expect(r.attr(strip[0], 'data-slots').split(',').filter((o) => o === 'free')).toHaveLength(5);
    expect(r.attr(strip[0], 'data-slots').split(',')[0]).toBe('ml/train-a');
    expect(r.attr(strip[0], 'title')).toContain('inferred from pod order');
    expect(r.text()).toBe('GPU 0–1 ml/train-a · GPU 2 ml/train-b · GPU 3–7 free (inferred)');
    r.unmount();
  });

  it('matrix → an 8 × 8 table with dashed self cells and the assumed-topology caption', () => {
    const r = render(h(v().Block, { b: matrixBlock(8, null, null) }));
    expect(r.byTag('tbody')[0] && r.byTag('tr').length).toBeGreaterThanOrEqual(8);
    expect(r.byTag('td').filter((n) => r.textOf(n) === '—')).toHaveLength(8);
    expect(r.text()).toContain('assumed MI355X full mesh');
    r.unmount();
  });

  it('a matrix built closed (a GPU Nodes card) is its summary line; the toggle opens the grid and closes it', () => {
    const measured = {};
    for (let i = 0; i < 8; i++) for (let j = 0; j < 8; j++) if (i !== j) measured[i + '-' + j] = 40;
    const r = render(h(v().Block, { b: matrixBlock(8, measured, null, false) }));
    expect(r.byTag('td')).toHaveLength(0);
    expect(r.text()).toContain('measured: max 40, mean 40 GB/s over 56 links');
    const toggle = () => r.byTag('button')[0];
    // closed: the summary line is the toggle (one element)
    expect(r.byTag('button')).toHaveLength(1);
    expect(r.attr(toggle(), 'aria-expanded')).toBe('false');
    expect(r.textOf(toggle())).toMatch(/^xGMI topology \(.* · Show xGMI matrix$/);
    r.click(toggle());
    expect(r.byTag('td')).toHaveLength(64);
    expect(r.byTag('td').filter((n) => r.textOf(n) === '40')).toHaveLength(56);
    expect(r.attr(toggle(), 'aria-expanded')).toBe('true');
    expect(r.textOf(toggle())).toBe('Hide xGMI matrix');
    r.click(toggle());
    expect(r.byTag('td')).toHaveLength(0);
    expect(r.textOf(toggle())).toMatch(/ · Show xGMI matrix$/);
    r.unmount();
  });

  it('series → per-node sparklines labelled for screen readers', () => {
    const pts = [[0, 100], [30, 300], [60, 200]];
    const b = { t: 'series', power: { n0: pts, n1: [] }, vram: { n0: pts }, avgPower: { n0: 200 } };
    const r = render(h(v().Block, { b }));
    expect(r.byTag('th').map((n) => r.textOf(n))).toEqual(['Node', 'Avg Power', 'Power (W)', 'HBM in use']);
    const svgs = r.byTag('svg');
    expect(svgs).toHaveLength(2);
    expect(r.attr(svgs[0], 'aria-label')).toBe('n0 power');
    expect(r.attr(r.byTag('path')[0], 'd')).toBe(sparklinePath(pts, 240, 36));
    expect(r.text()).toContain('200.0 W');
    r.unmount();
  });
});

describe('shared: pager (' + tier + ')', () => {
  const nodes = Array.from({ length: 20 }, (_, i) => makeGpuNode('mi355x-' + String(i).padStart(3, '0')));

  it('Previous / Next ask for the neighbouring page; the ends are disabled', () => {
    const onPage = vi.fn();
    const first = render(h(v().Page, { vm: page('T', null, [pager(nodePage(nodes, { page: 0 }), 'GPU nodes')]), onPage }));
    expect(first.text()).toContain('Showing 1–8 of 20 GPU nodes · page 1 of 3');
    expect(first.isDisabled(first.byLabel('Previous page'))).toBe(true);
    first.click(first.byLabel('Next page'));
    expect(onPage).toHaveBeenCalledWith(1);
    first.unmount();
    const last = render(h(v().Page, { vm: page('T', null, [pager(nodePage(nodes, { page: 2 }), 'GPU nodes')]), onPage }));
    expect(last.isDisabled(last.byLabel('Next page'))).toBe(true);
    last.click(last.byLabel('Previous page'));
    expect(onPage).toHaveBeenLastCalledWith(1);
    last.unmount();
  });

  it('typing in the filter hands the text to onFilter', () => {
    const onFilter = vi.fn();
    const r = render(h(v().Page, { vm: page('T', null, [pager(nodePage(nodes, {}), 'GPU nodes')]), onFilter }));
    r.change(r.byLabel('Filter GPU nodes by name'), '01');
    expect(onFilter).toHaveBeenCalledWith('01');
    r.unmount();
  });
});

describe('shared: a real view-model end to end (' + tier + ')', () => {
  it('Overview of a 2-node MI355X cluster renders every section with its Refresh button', () => {
    clearViewMemo();
    const nodes = [makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1')];
    const pods = [makeGpuPod('train-a', { gpus: 4 }), makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' })];
    const vm = overviewView(makeContext({ nodes, pods }));
    const r = render(h(v().Page, { vm, onRefresh: () => {} }));
    expect(r.byTag('h2').map((n) => r.textOf(n))).toEqual(vm.items.filter((it) => it.t === 'section').map((it) => it.title));
    expect(r.byAttr('data-total').length).toBeGreaterThan(0);
    expect(r.text()).toContain('mi355x-1');
    expect(r.byLabel(vm.refresh.ariaLabel)).toBeTruthy();
    r.unmount();
  });
});
