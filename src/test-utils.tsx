/**
 * Shared vitest stand-ins for Headlamp CommonComponents.
 *
 * Each component renders the plain semantic element that src/view/html.js
 * emits for the same IR node, so TSX tests and the Node-side specs assert on
 * one markup (the reference's component tests mock CommonComponents with the
 * same element mapping, SURVEY.md §4). Built with createElement from a small
 * table rather than per-component JSX.
 */
import React from 'react';

/* eslint-disable @typescript-eslint/no-explicit-any */
type Props = Record<string, any>;
const h = React.createElement;

/** Component → [tag, attributes] for the stand-ins that only wrap children. */
const WRAPPERS: Record<string, [string, Record<string, string>]> = {
  PercentageBar: ['div', { 'data-testid': 'percentage-bar' }],
};

function cells(columns: Props[], item: unknown) {
  return columns.map((c, j) => h('td', { key: j }, c.getter(item)));
}

export const commonComponentsMock: Record<string, (p: Props) => React.ReactElement> = {
  Loader: p => h('div', { 'data-testid': 'loader' }, p.title),
  SectionHeader: p => h('h1', null, p.title),
  SectionBox: p => h('section', null, h('h2', null, p.title), p.children),
  StatusLabel: p => h('span', { 'data-status': p.status }, p.children),
  NameValueTable: p =>
    h(
      'dl',
      null,
      (p.rows as Props[]).map((r, i) => h('div', { key: i }, h('dt', null, r.name), h('dd', null, r.value)))
    ),
  SimpleTable: p =>
    h(
      'table',
      null,
      h('thead', null, h('tr', null, (p.columns as Props[]).map((c, j) => h('th', { key: j }, c.label)))),
      h('tbody', null, (p.data as unknown[]).map((item, i) => h('tr', { key: i }, cells(p.columns, item))))
    ),
  ...Object.fromEntries(
    Object.entries(WRAPPERS).map(([name, [tag, attrs]]) => [name, (p: Props) => h(tag, attrs, p.children)])
  ),
};
