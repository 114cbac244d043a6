/**
 * Render adapter of the shared specs on REAL React 18 + react-dom, mounted in
 * jsdom with @testing-library/react — the reference's component tier
 * (reference vitest.config.mts:4-6, src/components/OverviewPage.test.tsx:8-61).
 * Selected by vitest.react.config.mts, which resolves 'react' to the real
 * package and mocks only '@kinvolk/headlamp-plugin/lib[/CommonComponents]'.
 * It needs the npm dev dependencies, so it runs in networked CI only; the
 * same specs run on the harness React offline (./stub.js).
 */
import * as ReactNS from 'react';
import { fireEvent, render as rtlRender, act } from '@testing-library/react';

const React = ReactNS.default || ReactNS;

export { React };
export const tier = 'react-dom';

// AMD_TEST_STRICT=1: every render under <StrictMode> (double render, effect replay).
const STRICT_ALL = typeof process !== 'undefined' && process.env.AMD_TEST_STRICT === '1';

export function render(element, options) {
  const strict = STRICT_ALL || !!(options && options.strict);
  const wrap = function (el) { return strict ? React.createElement(React.StrictMode, null, el) : el; };
  const r = rtlRender(wrap(element));
  const c = r.container;
  const handle = {
    /** Let pending requests resolve and React commit, `rounds` macrotask turns. */
    settle: async function (rounds) {
      const n = rounds || 20;
      for (let i = 0; i < n; i++) {
        await act(async function () {
          await new Promise(function (res) { setTimeout(res, 0); });
        });
      }
      return handle;
    },
    text: function () { return c.textContent; },
    html: function () { return c.innerHTML; },
    byLabel: function (label) {
      const hits = Array.prototype.filter.call(c.querySelectorAll('[aria-label]'), function (n) {
        return n.getAttribute('aria-label') === label;
      });
      if (hits.length !== 1) throw new Error((hits.length ? 'Found multiple' : 'Unable to find') + ' elements labelled ' + label);
      return hits[0];
    },
    byTag: function (tag) { return Array.prototype.slice.call(c.querySelectorAll(tag)); },
    byAttr: function (name) { return Array.prototype.slice.call(c.querySelectorAll('[' + name + ']')); },
    attr: function (node, name) { return node.getAttribute(name); },
    style: function (node) { return node.style; },
    click: function (node) { fireEvent.click(node); return handle; },
    change: function (node, value) { fireEvent.change(node, { target: { value: value } }); return handle; },
    blur: function (node, value) {
      if (value !== undefined) fireEvent.change(node, { target: { value: value } });
      fireEvent.blur(node);
      return handle;
    },
    value: function (node) { return node.value; },
    isDisabled: function (node) { return !!node.disabled; },
    textOf: function (node) { return node.textContent; },
    act: function (fn) {
      act(function () { fn(); });
      return handle;
    },
    rerender: function (element2) {
      r.rerender(wrap(element2));
      return handle;
    },
    unmount: function () { r.unmount(); },
  };
  return handle;
}
