/**
 * IR → CommonComponents renderer (src/view/react.js), executed under the
 * harness React (tests/js/stubs/react.js) with CommonComponents stand-ins
 * that render the markup the reference's component tests mock them with
 * (reference src/components/OverviewPage.test.tsx:8-61). Every spec checks
 * what the renderer HANDS each CommonComponent (props), not only the text;
 * what a user sees of the same blocks is also pinned runner-agnostically in
 * tests/js/shared/renderer.shared.test.js (both React tiers).
 */
import React, { render } from './stubs/react.js';
import * as CC from './stubs/CommonComponents.js';
import { BUTTON_CLASS, createRenderer, ensureStyles, PLUGIN_CSS, REQUIRED_COMPONENTS, matrixCaption, matrixCellColor, sparklinePath } from '../../src/view/react.js';
import { bar, kv, lines, loader, page, pctbar, row, section, status, table } from '../../src/view/ir.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { matrixBlock, slotsBlock } from '../../src/view/pages/nodes.js';
import { overviewView } from '../../src/view/pages/overview.js';
import { makeContext, makeGpuNode, makeGpuPod } from './fixtures.js';

const h = React.createElement;

function setup() {
  return createRenderer(React, CC);
}

function only(handle, type) {
  const all = handle.instances(type);
  expect(all).toHaveLength(1);
  return all[0].props;
}

describe('createRenderer', () => {
  it('requires React.createElement', () => {
    expect(() => createRenderer({}, CC)).toThrow('React is required');
  });
  it('names every missing CommonComponent', () => {
    REQUIRED_COMPONENTS.forEach((name) => {
      const partial = Object.assign({}, CC);
      delete partial[name];
      expect(() => createRenderer(React, partial)).toThrow('CommonComponents.' + name + ' is missing');
    });
  });
});

describe('Page', () => {
  it('renders the title through SectionHeader', () => {
    const v = setup();
    const r = render(h(v.Page, { vm: page('AMD GPU — Overview', null, []) }));
    expect(only(r, CC.SectionHeader).title).toBe('AMD GPU — Overview');
    expect(r.byTag('h1')).toHaveLength(1);
  });

  it('renders no header while the page is only a loader', () => {
    const v = setup();
    const r = render(h(v.Page, { vm: page(null, null, [loader('Loading AMD GPU data...')]) }));
    expect(r.instances(CC.SectionHeader)).toHaveLength(0);
    expect(only(r, CC.Loader).title).toBe('Loading AMD GPU data...');
    expect(r.getByTestId('loader')).toBeTruthy();
  });

  it('refresh button carries the aria-label and calls onRefresh on click', () => {
    const v = setup();
    const onRefresh = vi.fn();
    const vm = page('T', { label: 'Refresh', ariaLabel: 'Refresh AMD GPU data', disabled: false }, []);
    const r = render(h(v.Page, { vm, onRefresh }));
    const btn = r.getByLabelText('Refresh AMD GPU data');
    expect(btn.tag).toBe('button');
    expect(btn.props.disabled).toBe(false);
    r.click(btn);
    r.click(btn);
    expect(onRefresh).toHaveBeenCalledTimes(2);
  });

  it('disabled refresh button does not fire; its class dims it and shows the not-allowed cursor', () => {
    const v = setup();
    const onRefresh = vi.fn();
    const vm = page('T', { label: 'Refreshing...', ariaLabel: 'Refresh metrics', disabled: true }, []);
    const r = render(h(v.Page, { vm, onRefresh }));
    const btn = r.getByLabelText('Refresh metrics');
    expect(btn.props.disabled).toBe(true);
    expect(btn.props.className).toBe(BUTTON_CLASS);
    expect(PLUGIN_CSS).toContain('.' + BUTTON_CLASS + ':disabled{cursor:not-allowed;opacity:.6}');
    r.click(btn);
    expect(onRefresh).not.toHaveBeenCalled();
  });

  it('the stylesheet is added to a document once; nothing without a DOM', () => {
    const appended = [];
    const doc = {
      head: { appendChild: (el) => appended.push(el) },
      createElement: (tag) => ({ tag, attrs: {}, setAttribute(k, v) { this.attrs[k] = v; }, textContent: '' }),
    };
    expect(ensureStyles(doc)).toBe(true);
    expect(ensureStyles(doc)).toBe(true);
    expect(appended).toHaveLength(1);
    expect(appended[0].tag).toBe('style');
    expect(appended[0].textContent).toBe(PLUGIN_CSS);
    expect(ensureStyles({})).toBe(false);
  });

  it('maps loader and section items in order', () => {
    const v = setup();
    const vm = page('T', null, [section('A', []), loader('wait'), section('B', [])]);
    const r = render(h(v.Page, { vm }));
    expect(r.instances(CC.SectionBox).map((i) => i.props.title)).toEqual(['A', 'B']);
    expect(r.text()).toBe('TAwaitB');
  });
});

describe('blocks', () => {
  it('kv → NameValueTable rows (name + rendered value)', () => {
    const v = setup();
    const s = section('Cluster', [kv([row('GPU Nodes', '2'), row('State', status('success', 'Ready'))])]);
    const r = render(h(v.Section, { s }));
    expect(only(r, CC.SectionBox).title).toBe('Cluster');
    const rows = only(r, CC.NameValueTable).rows;
    expect(rows.map((x) => x.name)).toEqual(['GPU Nodes', 'State']);
    expect(r.byTag('dt').map((n) => n.children[0])).toEqual(['GPU Nodes', 'State']);
    expect(only(r, CC.StatusLabel).status).toBe('success');
    expect(r.getByText('Ready').props['data-status']).toBe('success');
  });

  it('table → SimpleTable with one column per label and getters reading cell i', () => {
    const v = setup();
    const rows = [['n0', '8'], ['n1', status('warning', '4')]];
    const r = render(h(v.Section, { s: section('Nodes', [table(['Node', 'GPUs'], rows)]) }));
    const p = only(r, CC.SimpleTable);
    expect(p.columns.map((c) => c.label)).toEqual(['Node', 'GPUs']);
    expect(p.data).toBe(rows);
    // cells are built inline: a string stays a string, a status cell is the StatusLabel itself
    expect(p.columns[0].getter(rows[0])).toBe('n0');
    expect(p.columns[1].getter(rows[1]).type).toBe(CC.StatusLabel);
    expect(p.columns[1].getter(rows[1]).props.status).toBe('warning');
    expect(r.byTag('tr')).toHaveLength(3);
    expect(r.byTag('th').map((n) => n.children[0])).toEqual(['Node', 'GPUs']);
  });

  it('pctbar → PercentageBar with data and total, under its label', () => {
    const v = setup();
    const data = [{ name: 'Allocated', value: 3, fill: '#f00' }, { name: 'Free', value: 5, fill: '#ccc' }];
    const r = render(h(v.Section, { s: section('Alloc', [pctbar('GPU allocation', data, 8)]) }));
    const p = only(r, CC.PercentageBar);
    expect(p.data).toBe(data);
    expect(p.total).toBe(8);
    expect(r.getByText('GPU allocation')).toBeTruthy();
    expect(r.getByTestId('percentage-bar').props['data-total']).toBe(8);
  });

  it('bar cell → ONE element: its fill as a gradient background up to the percentage, and its text', () => {
    const v = setup();
    const r = render(h(v.Value, { v: bar(3, 8, 38, '#4caf50', '3/8 (38%)') }));
    const fill = r.queryAll((n) => n.props['data-pct'] !== undefined);
    expect(fill).toHaveLength(1);
    expect(fill[0].props.style.backgroundImage).toBe('linear-gradient(to right, #4caf50 38%, #e0e0e0 38%)');
    expect(fill[0].props['data-color']).toBe('#4caf50');
    expect(r.text()).toBe('3/8 (38%)');
    expect(r.queryAll((n) => typeof n.tag === 'string')).toHaveLength(1);
  });

  it('bar cell without a percentage draws only the text', () => {
    const v = setup();
    const r = render(h(v.Value, { v: bar(3, null, null, '#000', '3 GPUs') }));
    expect(r.queryAll((n) => n.props['data-pct'] !== undefined)).toHaveLength(0);
    expect(r.text()).toBe('3 GPUs');
  });

  it('lines cell → one div per line with a bold label', () => {
    const v = setup();
    const r = render(h(v.Value, { v: lines([{ label: 'trainer', text: '2 GPUs' }, { label: '', text: 'plain' }]) }));
    expect(r.byTag('strong').map((n) => n.children[0])).toEqual(['trainer']);
    expect(r.text()).toBe('trainer: 2 GPUsplain');
  });

  it('null, strings and numbers render as plain text; unknown cells as nothing', () => {
    const v = setup();
    expect(render(h(v.Value, { v: null })).text()).toBe('');
    expect(render(h(v.Value, { v: 7 })).text()).toBe('7');
    expect(render(h(v.Value, { v: 'x' })).text()).toBe('x');
    expect(render(h(v.Value, { v: { t: 'nope' } })).text()).toBe('');
  });

  it('unknown block types render nothing', () => {
    const v = setup();
    const r = render(h(v.Section, { s: section('S', [{ t: 'mystery' }]) }));
    expect(r.text()).toBe('S');
  });

  it('slots → ONE element: a segment per GPU in its background, owners in runs as its text', () => {
    const v = setup();
    const node = makeGpuNode('mi355x-0');
    const pods = [makeGpuPod('train-a', { gpus: 2 }), makeGpuPod('train-b', { gpus: 1 })];
    const b = slotsBlock(node, pods, null);
    const r = render(h(v.Block, { b }));
    const strip = r.queryAll((n) => n.props['data-slots'] !== undefined);
    expect(strip).toHaveLength(1);
    expect(strip[0].props['data-slots'].split(',')).toEqual(['ml/train-a', 'ml/train-a', 'ml/train-b', 'free', 'free', 'free', 'free', 'free']);
    expect(r.text()).toBe('GPU 0–1 ml/train-a · GPU 2 ml/train-b · GPU 3–7 free (inferred)');
    expect(strip[0].props.title).toContain('inferred from pod order');
    expect(strip[0].props.style.backgroundImage.split('#e0e0e0').length - 1).toBe(10); // 5 free segments, 2 stops each
    expect(r.queryAll((n) => typeof n.tag === 'string')).toHaveLength(1);
  });

  it('a matrix built closed shows its summary and opens on click', () => {
    const v = setup();
    const r = render(h(v.Block, { b: matrixBlock(8, { '0-1': 40, '1-0': 60 }, null, false) }));
    expect(r.queryAll((n) => n.tag === 'td')).toHaveLength(0);
    expect(r.text()).toContain('measured: max 60, mean 50 GB/s over 2 links');
    const btn = r.queryAll((n) => n.tag === 'button')[0];
    expect(btn.props['aria-expanded']).toBe('false');
    r.click(btn);
    expect(r.queryAll((n) => n.tag === 'td')).toHaveLength(64);
    r.click(r.queryAll((n) => n.tag === 'button')[0]);
    expect(r.queryAll((n) => n.tag === 'td')).toHaveLength(0);
  });

  it('matrix → 8×8 table, self cells dashed, caption says the topology is assumed', () => {
    const v = setup();
    const b = matrixBlock(8, null, null);
    const r = render(h(v.Block, { b }));
    expect(r.byTag('tbody')[0].children).toHaveLength(8);
    const selfCells = r.byTag('td').filter((n) => n.children[0] === '—');
    expect(selfCells).toHaveLength(8);
    expect(r.text()).toContain('assumed MI355X full mesh');
    expect(matrixCaption(b)).toContain('assumed');
    expect(matrixCellColor({ kind: 'self' })).toBe('transparent');
  });

  it('series → SimpleTable of per-node sparklines', () => {
    const v = setup();
    const pts = [[0, 100], [30, 300], [60, 200]];
    const b = { t: 'series', power: { n0: pts, n1: [] }, vram: { n0: pts }, avgPower: { n0: 200 } };
    const r = render(h(v.Block, { b }));
    const p = only(r, CC.SimpleTable);
    expect(p.columns.map((c) => c.label)).toEqual(['Node', 'Avg Power', 'Power (W)', 'HBM in use']);
    expect(p.data).toEqual(['n0', 'n1']);
    expect(p.columns[1].getter('n0')).toBe('200.0 W');
    expect(p.columns[1].getter('n1')).toBe('—');
    const svgs = r.byTag('svg');
    expect(svgs).toHaveLength(2); // n1 has no points for either series
    expect(svgs[0].props['aria-label']).toBe('n0 power');
    expect(r.byTag('path')[0].props.d).toBe(sparklinePath(pts, 240, 36));
  });

  it('series with a row label and no HBM data: "Pod" column, no HBM column', () => {
    const v = setup();
    const b = { t: 'series', label: 'Pod', power: { 'train-p': [[0, 1], [30, 2]] }, vram: {}, avgPower: { 'train-p': 1.5 } };
    const r = render(h(v.Block, { b }));
    const p = only(r, CC.SimpleTable);
    expect(p.columns.map((c) => c.label)).toEqual(['Pod', 'Avg Power', 'Power (W)']);
  });

  it('sparklinePath needs two points and spans the box', () => {
    expect(sparklinePath([[0, 1]], 10, 10)).toBeNull();
    expect(sparklinePath([[0, 0], [10, 10]], 100, 50)).toBe('M0.0,50.0 L100.0,0.0');
  });
});

describe('Section memo', () => {
  it('skips re-rendering an unchanged section object', () => {
    const v = setup();
    const s = section('Stable', [kv([row('a', '1')])]);
    const r = render(h(v.Section, { s }));
    const inst = r.instances(v.Section)[0];
    expect(inst.renders).toBe(1);
    r.rerender(h(v.Section, { s }));
    r.rerender(h(v.Section, { s }));
    expect(inst.renders).toBe(1);
    expect(inst.skips).toBe(2);
    expect(only(r, CC.NameValueTable).rows[0].name).toBe('a');
  });

  it('re-renders when the section object changes', () => {
    const v = setup();
    const r = render(h(v.Section, { s: section('S', [kv([row('a', '1')])]) }));
    r.rerender(h(v.Section, { s: section('S', [kv([row('a', '2')])]) }));
    expect(r.instances(v.Section)[0].renders).toBe(2);
    expect(r.text()).toBe('Sa2');
  });

  it('a page refresh with one changed section re-renders only that section', () => {
    const v = setup();
    const a = section('A', []);
    const b1 = section('B', [kv([row('x', '1')])]);
    const b2 = section('B', [kv([row('x', '2')])]);
    const r = render(h(v.Page, { vm: page('T', null, [a, b1]) }));
    r.rerender(h(v.Page, { vm: page('T', null, [a, b2]) }));
    const counts = r.instances(v.Section).map((i) => [i.props.s.title, i.renders]);
    expect(counts).toEqual([['A', 1], ['B', 2]]);
  });
});

describe('a real view-model end to end', () => {
  beforeEach(() => clearViewMemo());

  it('Overview of a 2-node MI355X cluster renders every section through CommonComponents', () => {
    const v = setup();
    const nodes = [makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1')];
    const pods = [makeGpuPod('train-a', { gpus: 4 }), makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' })];
    const vm = overviewView(makeContext({ nodes, pods }));
    const r = render(h(v.Page, { vm, onRefresh: () => {} }));
    const titles = r.instances(CC.SectionBox).map((i) => i.props.title);
    expect(titles.length).toBeGreaterThan(2);
    expect(titles).toEqual(vm.items.filter((it) => it.t === 'section').map((it) => it.title));
    expect(r.instances(CC.PercentageBar).length).toBeGreaterThan(0);
    expect(r.html()).toContain('mi355x-1');
    expect(r.getByLabelText(vm.refresh.ariaLabel).tag).toBe('button');
  });
});

describe('harness React enforces the rules real React enforces', () => {
  it('a getSnapshot that returns a new object every call is rejected (infinite re-render in React)', () => {
    function Bad() {
      const v = React.useSyncExternalStore(() => () => {}, () => ({}));
      return h('div', null, String(!!v));
    }
    expect(() => render(h(Bad))).toThrow('getSnapshot should be cached');
  });

  it('a keyless element in an array child is rejected; variadic children need no key', () => {
    expect(() => render(h('ul', null, [h('li', null, 'a'), h('li', null, 'b')]))).toThrow('unique "key"');
    expect(() => render(h('ul', null, h('li', null, 'a'), h('li', null, 'b')))).not.toThrow();
  });

  it('hooks called in a different order on re-render are rejected', async () => {
    let flip = null;
    function Swap() {
      const s = React.useState(false);
      flip = s[1];
      if (s[0]) {
        React.useMemo(() => 1, []);
        React.useRef(0);
      } else {
        React.useRef(0);
        React.useMemo(() => 1, []);
      }
      return h('div', null, 'x');
    }
    const r = render(h(Swap));
    let err = null;
    try {
      flip(true);
      await r.settle();
    } catch (e) {
      err = e;
    }
    expect(String(err)).toContain('order of Hooks');
  });

  it('a state update of one component during another\'s render is rejected', () => {
    let setA = null;
    function A() {
      const s = React.useState(0);
      setA = s[1];
      return h('i', null, String(s[0]));
    }
    function B() {
      setA(1); // side effect in render
      return h('b', null, 'x');
    }
    expect(() => render(h('div', null, h(A), h(B)))).toThrow('while rendering');
  });

  it('a ref written while rendering is rejected; written in an effect it is fine', async () => {
    function Bad() {
      const r = React.useRef(0);
      r.current = r.current + 1; // side effect in render
      return h('i', null, 'x');
    }
    expect(() => render(h(Bad))).toThrow('ref.current written while rendering Bad');
    let seen = null;
    function Good(props) {
      const r = React.useRef(null);
      React.useEffect(function () { r.current = props.v; seen = r; }, [props.v]);
      return h('i', null, String(r.current)); // reading is allowed
    }
    const g = render(h(Good, { v: 7 }));
    await g.settle();
    expect(seen.current).toBe(7);
  });

  it('a hook skipped on re-render is rejected', async () => {
    let setFlag = null;
    function Cond() {
      const s = React.useState(false);
      setFlag = s[1];
      if (s[0]) return h('div', null, 'early');
      React.useMemo(() => 1, []);
      return h('div', null, 'late');
    }
    const r = render(h(Cond));
    let err = null;
    try {
      setFlag(true);
      await r.settle();
    } catch (e) {
      err = e;
    }
    expect(String(err)).toContain('Rendered fewer hooks than expected');
  });
});
