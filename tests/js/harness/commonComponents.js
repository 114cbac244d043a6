/**
 * Headlamp CommonComponents stand-ins over ANY React's createElement: the
 * semantic elements the reference's component tests mock them with
 * (reference src/components/OverviewPage.test.tsx:8-61), which
 * src/view/html.js also emits. tests/js/stubs/CommonComponents.js builds
 * them on the harness React; tests/js/harness/dom.js on the real one.
 * @param {Function} h  React.createElement
 */
export function makeCommonComponents(h) {
  return {
    SectionBox: function SectionBox(p) {
      return h('section', null, h('h2', null, p.title), p.children);
    },
    SectionHeader: function SectionHeader(p) {
      return h('h1', null, p.title);
    },
    NameValueTable: function NameValueTable(p) {
      return h(
        'dl',
        null,
        p.rows.map(function (r, i) { return h('div', { key: i }, h('dt', null, r.name), h('dd', null, r.value)); })
      );
    },
    SimpleTable: function SimpleTable(p) {
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
    },
    StatusLabel: function StatusLabel(p) {
      return h('span', { 'data-status': p.status }, p.children);
    },
    Loader: function Loader(p) {
      return h('div', { 'data-testid': 'loader' }, p.title);
    },
    PercentageBar: function PercentageBar(p) {
      return h(
        'div',
        { 'data-testid': 'percentage-bar', 'data-total': p.total },
        p.data.map(function (d, i) { return h('span', { key: i, 'data-name': d.name, 'data-value': d.value, 'data-fill': d.fill }, d.name + ': ' + d.value); })
      );
    },
  };
}
