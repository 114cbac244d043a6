/**
 * Render adapter of the shared specs (tests/js/shared/) on the harness React
 * (tests/js/stubs/react.js): what `npm run test:node12`, `npm test` and the
 * pytest bridge run. tests/js/harness/dom.js is the same API on real React 18
 * + react-dom under jsdom (vitest.react.config.mts, networked CI only).
 *
 * A shared spec imports this API from 'amd-test-harness' and never a stub
 * internal: no component instances, no render counters.
 */
import React, { render as stubRender, textOf } from '../stubs/react.js';

export { React };
export const tier = 'harness';

// AMD_TEST_STRICT=1: every render under <StrictMode> (double render, effect replay).
const STRICT_ALL = typeof process !== 'undefined' && process.env.AMD_TEST_STRICT === '1';

export function render(element, options) {
  const r = stubRender(element, STRICT_ALL ? Object.assign({}, options, { strict: true }) : options);
  const handle = {
    settle: function (rounds) { return r.settle(rounds).then(function () { return handle; }); },
    text: function () { return r.text(); },
    html: function () { return r.html(); },
    /** The one element whose aria-label is exactly `label`. */
    byLabel: function (label) { return r.getByLabelText(label); },
    byTag: function (tag) { return r.byTag(tag); },
    /** Host elements carrying attribute `name`. */
    byAttr: function (name) { return r.queryAll(function (n) { return n.props[name] !== undefined; }); },
    /** An attribute as the DOM reports it (a string), or null. */
    attr: function (node, name) {
      const v = node.props[name === 'class' ? 'className' : name];
      return v === undefined || v === null || v === false ? null : String(v);
    },
    style: function (node) { return node.props.style || {}; },
    click: function (node) { r.click(node); return handle; },
    change: function (node, value) { r.change(node, value); return handle; },
    /** Leave a field (onBlur), with `value` typed into it when given. */
    blur: function (node, value) { r.blur(node, value); return handle; },
    /** What a form field shows: its controlled value, else its initial (uncontrolled) value. */
    value: function (node) { return r.fieldValue(node); },
    isDisabled: function (node) { return !!node.props.disabled; },
    textOf: function (node) { return textOf(node); },
    /** Run `fn` (an event-like update) and commit what it scheduled. */
    act: function (fn) {
      r.act(function () { fn(); });
      return handle;
    },
    /** Render a new element at the same root (props change, key change). */
    rerender: function (element2) {
      r.rerender(element2);
      return handle;
    },
    unmount: function () { r.unmount(); },
  };
  return handle;
}
