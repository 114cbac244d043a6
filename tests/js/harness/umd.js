/**
 * Render adapter of the shared specs on REAL React 18.3.1 + react-dom,
 * offline: the UMD builds (./umd-react.js) rendering into the minimal DOM
 * (./minidom.js) through ReactDOM.createRoot, with React's own act(). The
 * same API as ./stub.js (harness React) and ./dom.js (jsdom +
 * @testing-library/react, networked CI): tools/plugin-loader.js selects this
 * one when AMD_TEST_TIER=react-umd (tests/test_js_real_react.py).
 */
import React, { ReactDOM } from './umd-react.js';
import { Event } from './minidom.js';

export { React };
export const tier = 'react-dom-umd';

const act = React.act;
// AMD_TEST_STRICT=1: every render under <StrictMode> (double render, effect replay).
const STRICT_ALL = process.env.AMD_TEST_STRICT === '1';

/** The DOM's own value setter, so React's value tracker sees a user's edit (as testing-library does). */
function setNativeValue(node, value) {
  let proto = Object.getPrototypeOf(node);
  while (proto && !Object.getOwnPropertyDescriptor(proto, 'value')) proto = Object.getPrototypeOf(proto);
  Object.getOwnPropertyDescriptor(proto, 'value').set.call(node, value);
}

export function render(element, options) {
  const strict = STRICT_ALL || !!(options && options.strict);
  const wrap = function (el) { return strict ? React.createElement(React.StrictMode, null, el) : el; };
  const c = document.createElement('div');
  document.body.appendChild(c);
  const root = ReactDOM.createRoot(c);
  act(function () { root.render(wrap(element)); });
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
    html: function () { return ''; },
    byLabel: function (label) {
      const hits = c.querySelectorAll('[aria-label]').filter(function (n) { return n.getAttribute('aria-label') === label; });
      if (hits.length !== 1) throw new Error((hits.length ? 'Found multiple' : 'Unable to find') + ' elements labelled ' + label);
      return hits[0];
    },
    byTag: function (tag) { return c.querySelectorAll(tag); },
    byAttr: function (name) { return c.querySelectorAll('[' + name + ']'); },
    attr: function (node, name) { return node.getAttribute(name); },
    style: function (node) { return node.style; },
    click: function (node) {
      act(function () { node.dispatchEvent(new Event('click', { bubbles: true, cancelable: true })); });
      return handle;
    },
    change: function (node, value) {
      act(function () {
        setNativeValue(node, value);
        node.dispatchEvent(new Event(node.localName === 'select' ? 'change' : 'input', { bubbles: true }));
      });
      return handle;
    },
    /** Leave a field (onBlur: React listens to focusout), after typing `value` into it when given. */
    blur: function (node, value) {
      act(function () {
        if (value !== undefined) {
          setNativeValue(node, value);
          node.dispatchEvent(new Event('input', { bubbles: true }));
        }
        node.dispatchEvent(new Event('focusout', { bubbles: true }));
      });
      return handle;
    },
    /** What a form field shows. */
    value: function (node) { return node.value; },
    isDisabled: function (node) { return !!node.disabled; },
    textOf: function (node) { return node.textContent; },
    act: function (fn) {
      act(function () { fn(); });
      return handle;
    },
    rerender: function (element2) {
      act(function () { root.render(wrap(element2)); });
      return handle;
    },
    unmount: function () {
      act(function () { root.unmount(); });
      if (c.parentNode) c.parentNode.removeChild(c);
    },
  };
  return handle;
}
