/**
 * Headlamp CommonComponents stand-ins for the Node-12 harness, built on the
 * React stand-in. Each renders the semantic element the reference's component
 * tests mock it with (reference src/components/OverviewPage.test.tsx:8-61) —
 * and that src/view/html.js emits for the same IR node — so specs assert on
 * one markup whichever renderer produced it:
 *   SectionBox → <section><h2>title</h2>…</section>, SectionHeader → <h1>,
 *   NameValueTable → <dl><div><dt>name</dt><dd>value</dd></div>…</dl>,
 *   SimpleTable → <table><thead>…</thead><tbody>…</tbody></table>,
 *   StatusLabel → <span data-status>, Loader → data-testid="loader",
 *   PercentageBar → data-testid="percentage-bar".
 * Component instances keep their props, so specs can also check what a page
 * handed each component (SimpleTable columns / getters / data, …).
 */
import { createElement as h } from './react.js';

export function SectionBox(p) {
  return h('section', null, h('h2', null, p.title), p.children);
}

export function SectionHeader(p) {
  return h('h1', null, p.title);
}

export function NameValueTable(p) {
  return h(
    'dl',
    null,
    p.rows.map(function (r, i) { return h('div', { key: i }, h('dt', null, r.name), h('dd', null, r.value)); })
  );
}

export function SimpleTable(p) {
  return h(
    'table',
    null,
    h('thead', null, h('tr', null, p.columns.map(function (c, j) { return h('th', { key: j }, c.label); }))),
    h(
      'tbody',
      null,
      p.data.map(function (item, i) {
        return h('tr', { key: i }, p.columns.map(function (c, j) { return h('td', { key: j }, c.getter(item)); }));
      })
    )
  );
}

export function StatusLabel(p) {
  return h('span', { 'data-status': p.status }, p.children);
}

export function Loader(p) {
  return h('div', { 'data-testid': 'loader' }, p.title);
}

export function PercentageBar(p) {
  return h(
    'div',
    { 'data-testid': 'percentage-bar', 'data-total': p.total },
    p.data.map(function (d, i) { return h('span', { key: i, 'data-name': d.name, 'data-value': d.value, 'data-fill': d.fill }, d.name + ': ' + d.value); })
  );
}
