/**
 * A small React 18 stand-in for the Node-12 test harness (no npm registry
 * here, so the real React cannot be installed). It implements the subset of
 * React the plugin's shipped code uses — createElement, Fragment, memo,
 * createContext, useState / useReducer / useEffect / useLayoutEffect /
 * useMemo / useCallback / useRef / useContext / useSyncExternalStore — and a
 * reconciling renderer:
 *
 *   * component instances keep their hook state across renders (matched by
 *     key, else position, and type, like React);
 *   * `memo` components skip rendering when their props are shallow-equal
 *     and nothing below them is dirty (render counts are observable);
 *   * effects run after the render pass in React's commit order: layout
 *     before passive, children before parents, every cleanup of a phase
 *     before its new effects; a deleted subtree cleans up parent first;
 *   * <StrictMode> calls each component body twice and replays new effects
 *     (mount, cleanup, mount), as React 18's development build does;
 *   * state updates outside `act` are batched on a microtask.
 *
 * tests/js/shared/react-semantics.shared.test.js pins these rules; it runs
 * here and on real React 18.3.1 + react-dom — offline through the UMD builds
 * (tests/test_js_real_react.py), and in networked CI under jsdom
 * (vitest.react.config.mts) — so a divergence of this file from React fails.
 *
 * The rendered host tree ({tag, props, children}) can be queried
 * testing-library style (getByText, getByLabelText, getByTestId, …),
 * clicked, and serialised to HTML. Only what the plugin needs is modelled:
 * no refs to host nodes, no portals, no suspense, no concurrent mode.
 * The host tree's serialisation and queries are in ./hostTree.js.
 */

import { hostQueries, htmlOf, textOf } from './hostTree.js';

const ELEMENT = Symbol.for('stub.react.element');
const MEMO = Symbol.for('stub.react.memo');
const PROVIDER = Symbol.for('stub.react.provider');
const LIST = Symbol.for('stub.react.list');

export const Fragment = Symbol.for('stub.react.fragment');

// Children arrays built by createElement from its arguments; any OTHER array
// rendered as children (a .map() result, an array returned by a component)
// is a list whose elements need keys.
const VARIADIC = new WeakSet();

export function createElement(type, props) {
  const p = {};
  let key = null;
  if (props) {
    for (const k in props) {
      if (k === 'key') key = props.key === undefined || props.key === null ? null : String(props.key);
      else if (k !== 'ref') p[k] = props[k];
    }
  }
  if (arguments.length === 3) p.children = arguments[2];
  else if (arguments.length > 3) {
    p.children = Array.prototype.slice.call(arguments, 2);
    VARIADIC.add(p.children);
  }
  if (type === undefined || type === null) throw new Error('createElement: element type is ' + type);
  return { $$typeof: ELEMENT, type: type, key: key, props: p };
}

export function isValidElement(v) {
  return !!v && v.$$typeof === ELEMENT;
}

function shallowEqual(a, b) {
  if (a === b) return true;
  const ka = Object.keys(a);
  const kb = Object.keys(b);
  if (ka.length !== kb.length) return false;
  for (let i = 0; i < ka.length; i++) if (!Object.is(a[ka[i]], b[ka[i]])) return false;
  return true;
}

export function memo(type, compare) {
  return { $$typeof: MEMO, type: type, compare: compare || shallowEqual, displayName: 'Memo(' + (type.displayName || type.name) + ')' };
}

export function createContext(defaultValue) {
  const ctx = { _default: defaultValue };
  ctx.Provider = { $$typeof: PROVIDER, context: ctx };
  return ctx;
}

// ---------------------------------------------------------------------------
// Hooks
// ---------------------------------------------------------------------------

let current = null; // instance being rendered
let hookIndex = 0;
let replaying = false; // StrictMode's discarded first call of a component body
let currentRoot = null;
const ctxStack = [];

function hookSlot(init, kind) {
  if (!current) throw new Error('Invalid hook call: hooks can only be called inside a function component');
  const hooks = current.hooks;
  const kinds = current.hookKinds || (current.hookKinds = []);
  if (hookIndex >= hooks.length) {
    if (current.renders > 1) throw new Error('Rendered more hooks than during the previous render');
    hooks.push(init());
    kinds.push(kind);
  }
  // React: "React has detected a change in the order of Hooks".
  if (kinds[hookIndex] !== kind) throw new Error('Change in the order of Hooks: ' + kinds[hookIndex] + ' then ' + kind + ' at hook ' + hookIndex);
  return hooks[hookIndex++];
}

function depsChanged(prev, next) {
  if (!prev || !next) return true;
  if (prev.length !== next.length) return true;
  for (let i = 0; i < prev.length; i++) if (!Object.is(prev[i], next[i])) return true;
  return false;
}

export function useReducer(reducer, initialArg, init) {
  const inst = current;
  const slot = hookSlot(function () {
    const s = { state: init ? init(initialArg) : initialArg, dispatch: null };
    s.dispatch = function (action) {
      if (inst.unmounted) return;
      // React: "Cannot update a component while rendering a different component".
      if (current && current !== inst) {
        throw new Error('Cannot update ' + typeName(inst.type) + ' while rendering ' + typeName(current.type));
      }
      const next = s.reducer(s.state, action);
      if (Object.is(next, s.state)) return;
      s.state = next;
      markDirty(inst);
    };
    return s;
  }, 'useReducer');
  slot.reducer = reducer;
  return [slot.state, slot.dispatch];
}

function basicReducer(s, a) {
  return typeof a === 'function' ? a(s) : a;
}

export function useState(init) {
  return useReducer(basicReducer, init, typeof init === 'function' ? function (f) { return f(); } : undefined);
}

function effectHook(fn, deps, layout) {
  const inst = current;
  const slot = hookSlot(function () { return { deps: undefined, cleanup: null, first: true }; }, layout ? 'useLayoutEffect' : 'useEffect');
  if (replaying) return;
  if (slot.first || deps === undefined || depsChanged(slot.deps, deps)) {
    slot.first = false;
    slot.deps = deps;
    inst.root.pendingEffects.push({ inst: inst, slot: slot, fn: fn, depth: inst.depth, layout: layout });
  }
}

export function useEffect(fn, deps) {
  effectHook(fn, deps, false);
}

export function useLayoutEffect(fn, deps) {
  effectHook(fn, deps, true);
}

export function useMemo(fn, deps) {
  const slot = hookSlot(function () { return { deps: undefined, value: undefined, first: true }; }, 'useMemo');
  if (slot.first || depsChanged(slot.deps, deps)) {
    slot.first = false;
    slot.deps = deps;
    slot.value = fn();
  }
  return slot.value;
}

export function useCallback(fn, deps) {
  return useMemo(function () { return fn; }, deps);
}

export function useRef(v) {
  return hookSlot(function () {
    let value = v;
    return Object.defineProperty({}, 'current', {
      enumerable: true,
      get: function () { return value; },
      set: function (x) {
        // React: a ref holds what rendering does not depend on; writing one
        // while rendering breaks StrictMode's double render and concurrent
        // rendering. Write it in an effect or an event handler.
        if (current) throw new Error('ref.current written while rendering ' + typeName(current.type));
        value = x;
      },
    });
  }, 'useRef');
}

function readContext(ctx) {
  for (let i = ctxStack.length - 1; i >= 0; i--) if (ctxStack[i].context === ctx) return ctxStack[i].value;
  return ctx._default;
}

export function useContext(ctx) {
  if (!current) throw new Error('Invalid hook call: useContext outside a component');
  const v = readContext(ctx);
  current.ctxReads.set(ctx, v);
  return v;
}

export function useSyncExternalStore(subscribe, getSnapshot) {
  const inst = current;
  const slot = hookSlot(function () { return { subscribe: null, unsubscribe: null, value: undefined }; }, 'useSyncExternalStore');
  const value = getSnapshot();
  // React (dev) reads the snapshot twice: a store whose getSnapshot builds a
  // new object each call would re-render forever.
  if (!Object.is(getSnapshot(), value)) throw new Error('The result of getSnapshot should be cached to avoid an infinite loop');
  if (replaying) return value;
  slot.value = value;
  slot.getSnapshot = getSnapshot;
  if (slot.subscribe !== subscribe) {
    slot.subscribe = subscribe;
    // React 18 subscribes in a passive effect and re-checks the snapshot there.
    inst.root.pendingEffects.push({
      inst: inst,
      slot: slot,
      depth: inst.depth,
      layout: false,
      fn: function () {
        if (slot.unsubscribe) slot.unsubscribe();
        const check = function () {
          if (!Object.is(slot.getSnapshot(), slot.value)) markDirty(inst);
        };
        slot.unsubscribe = subscribe(check);
        check(); // the store may have changed between render and subscribe
        return function () {
          if (slot.unsubscribe) slot.unsubscribe();
          slot.unsubscribe = null;
        };
      },
    });
  }
  return value;
}

const React = {
  createElement: createElement,
  isValidElement: isValidElement,
  Fragment: Fragment,
  memo: memo,
  createContext: createContext,
  useState: useState,
  useReducer: useReducer,
  useEffect: useEffect,
  useLayoutEffect: useLayoutEffect,
  useMemo: useMemo,
  useCallback: useCallback,
  useRef: useRef,
  useContext: useContext,
  useSyncExternalStore: useSyncExternalStore,
  version: '18.3.1-stub',
};
export default React;

// ---------------------------------------------------------------------------
// Renderer
// ---------------------------------------------------------------------------

function typeName(t) {
  if (typeof t === 'string') return t;
  if (t === Fragment) return 'Fragment';
  if (t === LIST) return 'List';
  if (t && t.$$typeof === MEMO) return t.displayName;
  if (t && t.$$typeof === PROVIDER) return 'Context.Provider';
  return (t && (t.displayName || t.name)) || 'Anonymous';
}

function newInstance(root, parent, type, key) {
  return {
    root: root,
    parent: parent,
    depth: parent ? parent.depth + 1 : 0,
    type: type,
    key: key,
    props: null,
    hooks: [],
    kids: [],
    out: [],
    dirty: true,
    renders: 0,
    skips: 0,
    ctxReads: new Map(),
    unmounted: false,
    text: null,
  };
}

function markDirty(inst) {
  inst.dirty = true;
  inst.root.schedule();
}

/**
 * True when `inst` or anything below it has pending state, or (with
 * `checkCtx`, used at memo boundaries) read a context value that has
 * changed since. Providers inside the subtree push their current value so
 * descendants compare against what they would read now.
 */
function subtreeNeedsRender(inst, checkCtx) {
  if (inst.dirty) return true;
  if (checkCtx) {
    let changed = false;
    inst.ctxReads.forEach(function (v, ctx) {
      if (!Object.is(readContext(ctx), v)) changed = true;
    });
    if (changed) return true;
  }
  const provider = inst.type && inst.type.$$typeof === PROVIDER;
  if (provider) ctxStack.push({ context: inst.type.context, value: inst.props.value });
  try {
    for (let i = 0; i < inst.kids.length; i++) if (subtreeNeedsRender(inst.kids[i], checkCtx)) return true;
  } finally {
    if (provider) ctxStack.pop();
  }
  return false;
}

function childList(children) {
  if (children === undefined) return [];
  return Array.isArray(children) ? children : [children];
}

function identity(item, index) {
  if (isValidElement(item) && item.key !== null) return 'k:' + item.key;
  return 'i:' + index;
}

function sameType(inst, item) {
  if (typeof item === 'string' || typeof item === 'number') return inst.type === '#text';
  if (Array.isArray(item)) return inst.type === LIST;
  return inst.type === item.type;
}

function reconcileChildren(root, parent, children) {
  const list = childList(children);
  const keyed = parent.type === LIST || (Array.isArray(children) && !VARIADIC.has(children));
  const old = new Map();
  for (let i = 0; i < parent.kids.length; i++) old.set(parent.kids[i].ident, parent.kids[i]);
  const kids = [];
  const seen = {};
  for (let i = 0; i < list.length; i++) {
    const item = list[i];
    if (item === null || item === undefined || item === false || item === true || item === '') continue;
    // React warns for every keyless element of an array child.
    if (keyed && isValidElement(item) && (item.key === null || item.key === undefined)) {
      throw new Error('Each child in a list should have a unique "key" prop (' + typeName(item.type) + ')');
    }
    const id = identity(item, i);
    if (seen[id]) throw new Error('Duplicate key "' + id.slice(2) + '" among children of ' + typeName(parent.type));
    seen[id] = true;
    let inst = old.get(id);
    if (inst && !sameType(inst, item)) inst = null;
    if (inst) old.delete(id);
    if (typeof item === 'string' || typeof item === 'number') {
      inst = inst || newInstance(root, parent, '#text', null);
      inst.text = String(item);
      inst.out = [inst.text];
      inst.dirty = false;
    } else if (Array.isArray(item)) {
      inst = inst || newInstance(root, parent, LIST, null);
      inst.props = { children: item };
      renderInstance(inst);
    } else if (isValidElement(item)) {
      const fresh = !inst;
      inst = inst || newInstance(root, parent, item.type, item.key);
      const prevProps = inst.props;
      inst.props = item.props;
      renderInstance(inst, fresh ? null : prevProps);
    } else {
      throw new Error('Objects are not valid as a React child (found: ' + Object.keys(item).join(', ') + ')');
    }
    inst.ident = id;
    kids.push(inst);
  }
  old.forEach(function (inst) { unmount(inst); });
  parent.kids = kids;
  const out = [];
  for (let i = 0; i < kids.length; i++) for (let j = 0; j < kids[i].out.length; j++) out.push(kids[i].out[j]);
  return out;
}

/** After an event, a controlled field shows its current `value` prop, whether or not the handler changed it (React restores it). */
function restoreControlled(node) {
  const inst = node.instance;
  if (inst && !inst.unmounted && inst.props.value !== undefined) inst.field = inst.props.value;
}

function hostProps(props) {
  const p = {};
  for (const k in props) if (k !== 'children') p[k] = props[k];
  return p;
}

function renderInstance(inst, prevProps) {
  const t = inst.type;
  const root = inst.root;
  if (typeof t === 'string') {
    inst.renders++;
    // A form field's displayed value, as the DOM keeps it: set from value /
    // defaultValue at mount, then only by a controlled `value` or by the user
    // (change / blur below); a later defaultValue does not reach the screen.
    if (!('field' in inst)) inst.field = inst.props.value !== undefined ? inst.props.value : inst.props.defaultValue;
    else if (inst.props.value !== undefined) inst.field = inst.props.value;
    const children = reconcileChildren(root, inst, inst.props.children);
    inst.out = [{ tag: t, props: hostProps(inst.props), children: children, instance: inst }];
  } else if (t === Fragment || t === LIST) {
    inst.out = reconcileChildren(root, inst, inst.props.children);
  } else if (t && t.$$typeof === PROVIDER) {
    ctxStack.push({ context: t.context, value: inst.props.value });
    try {
      inst.out = reconcileChildren(root, inst, inst.props.children);
    } finally {
      ctxStack.pop();
    }
  } else if (t && t.$$typeof === MEMO) {
    if (prevProps && !inst.dirty && t.compare(prevProps, inst.props) && !subtreeNeedsRender(inst, true)) {
      inst.skips++;
      return;
    }
    inst.renders++;
    inst.out = reconcileChildren(root, inst, createElement(t.type, inst.props));
  } else if (typeof t === 'function') {
    const prev = current;
    const prevIdx = hookIndex;
    const prevReplay = replaying;
    current = inst;
    inst.renders++;
    let result;
    let used = 0;
    try {
      // <StrictMode> (React 18, development) calls every component body
      // twice per render and keeps the second result, so a render with side
      // effects shows up. The first call here queues no effects.
      const calls = root.strict ? 2 : 1;
      for (let c = 0; c < calls; c++) {
        replaying = c < calls - 1;
        hookIndex = 0;
        inst.ctxReads = new Map();
        result = t(inst.props);
        used = hookIndex;
      }
    } finally {
      current = prev;
      hookIndex = prevIdx;
      replaying = prevReplay;
    }
    // React: "Rendered fewer hooks than expected" (a hook behind a condition or an early return).
    if (used < inst.hooks.length) throw new Error('Rendered fewer hooks than expected in ' + typeName(t));
    if (result === undefined) throw new Error(typeName(t) + ' returned undefined (return null to render nothing)');
    inst.out = reconcileChildren(root, inst, result);
  } else {
    throw new Error('Unsupported element type: ' + String(t));
  }
  inst.dirty = false;
}

// React 18 runs a deleted subtree's effect cleanups parent before child
// (react-reconciler's "Deletion effects fire in parent -> child order"),
// layout cleanups during the commit, passive ones after it.
function unmount(inst) {
  if (inst.unmounted) return;
  const removed = [];
  walkInstances(inst, function (i) {
    if (!i.unmounted) removed.push(i);
  });
  removed.forEach(function (i) { i.unmounted = true; });
  [true, false].forEach(function (layout) {
    removed.forEach(function (i) {
      const kinds = i.hookKinds || [];
      for (let h = 0; h < i.hooks.length; h++) {
        const hk = i.hooks[h];
        const isLayout = kinds[h] === 'useLayoutEffect';
        if (isLayout !== layout || !hk || typeof hk.cleanup !== 'function') continue;
        const c = hk.cleanup;
        hk.cleanup = null;
        c();
      }
    });
  });
  removed.forEach(function (i) { i.root.unmounts++; });
}


function walkInstances(inst, fn) {
  fn(inst);
  for (let i = 0; i < inst.kids.length; i++) walkInstances(inst.kids[i], fn);
}

function flushMicrotasks() {
  return new Promise(function (r) { setImmediate(r); });
}

/**
 * Mount `element` and return a handle. All rendering is synchronous; state
 * updates from promises are flushed on a microtask or by `settle()`.
 */
export function render(element, options) {
  const root = {
    element: element,
    strict: !!(options && options.strict),
    top: null,
    pendingEffects: [],
    scheduled: false,
    batching: 0,
    unmounts: 0,
    commits: 0,
    error: null,
  };
  root.top = newInstance(root, null, Fragment, null);

  root.schedule = function () {
    if (root.batching > 0 || root.scheduled || root.top.unmounted) return;
    root.scheduled = true;
    Promise.resolve().then(function () {
      root.scheduled = false;
      try {
        flush();
      } catch (e) {
        root.error = e;
      }
    });
  };

  function cleanupOf(e) {
    if (e.inst.unmounted || typeof e.slot.cleanup !== 'function') return;
    const c = e.slot.cleanup;
    e.slot.cleanup = null;
    c();
  }

  function mountOf(e) {
    if (e.inst.unmounted) return;
    const r = e.fn();
    e.slot.cleanup = typeof r === 'function' ? r : null;
  }

  function runEffects() {
    const list = root.pendingEffects;
    root.pendingEffects = [];
    // React commit order: children's effects before their parents'; every
    // cleanup of a phase before any of its new effects; the layout phase
    // (inside the commit) before the passive one.
    list.sort(function (a, b) { return b.depth - a.depth; });
    const layout = list.filter(function (e) { return e.layout; });
    const passive = list.filter(function (e) { return !e.layout; });
    layout.forEach(cleanupOf);
    layout.forEach(mountOf);
    passive.forEach(cleanupOf);
    passive.forEach(mountOf);
    // <StrictMode> (React 18, development): newly mounted effects are torn
    // down and run again — layout cleanups, passive cleanups, layout effects,
    // passive effects — so effects must be idempotent.
    if (root.strict) {
      const fresh = list.filter(function (e) { return !e.slot.strictRemounted && !e.inst.unmounted; });
      fresh.forEach(function (e) { e.slot.strictRemounted = true; });
      const fl = fresh.filter(function (e) { return e.layout; });
      const fp = fresh.filter(function (e) { return !e.layout; });
      fl.forEach(cleanupOf);
      fp.forEach(cleanupOf);
      fl.forEach(mountOf);
      fp.forEach(mountOf);
    }
  }

  function pass() {
    const prev = currentRoot;
    currentRoot = root;
    try {
      root.top.props = { children: root.element };
      renderInstance(root.top);
      root.commits++;
      runEffects();
    } finally {
      currentRoot = prev;
    }
  }

  function flush() {
    if (root.top.unmounted) return;
    for (let i = 0; i < 100; i++) {
      if (!subtreeNeedsRender(root.top, false) && root.pendingEffects.length === 0) return;
      pass();
    }
    throw new Error('Too many re-renders (update loop?)');
  }

  root.batching++;
  try {
    pass();
  } finally {
    root.batching--;
  }
  flush();

  const handle = Object.assign(hostQueries(function () { return root.top.out; }), {
    /** Synchronously apply pending state updates. */
    flush: function () {
      if (root.error) {
        const e = root.error;
        root.error = null;
        throw e;
      }
      flush();
      return handle;
    },
    /** Run `fn` with updates batched, then flush (awaits a returned promise). */
    act: function (fn) {
      root.batching++;
      let r;
      try {
        r = fn();
      } catch (e) {
        root.batching--;
        throw e;
      }
      if (r && typeof r.then === 'function') {
        return r.then(
          function (v) { root.batching--; flush(); return v; },
          function (e) { root.batching--; throw e; }
        );
      }
      root.batching--;
      flush();
      return r;
    },
    /** Let pending promises (requests, timers at 0) run and flush, until quiet. */
    settle: async function (rounds) {
      const n = rounds || 20;
      for (let i = 0; i < n; i++) {
        await flushMicrotasks();
        handle.flush();
      }
      return handle;
    },
    rerender: function (el) {
      root.element = el;
      root.batching++;
      try {
        pass();
      } finally {
        root.batching--;
      }
      flush();
      return handle;
    },
    unmount: function () {
      unmount(root.top);
    },
    nodes: function () { return root.top.out; },
    html: function () { return root.top.out.map(htmlOf).join(''); },
    text: function () { return root.top.out.map(textOf).join(''); },
    stats: function () { return { commits: root.commits, unmounts: root.unmounts }; },
    /** Component instances of `type` (function, memo or host tag). */
    instances: function (type) {
      const out = [];
      walkInstances(root.top, function (i) { if (i.type === type && !i.unmounted) out.push(i); });
      return out;
    },
    click: function (node) {
      if (node.props.disabled) return handle;
      handle.act(function () {
        if (typeof node.props.onClick === 'function') node.props.onClick({ type: 'click', target: node, preventDefault: function () {} });
      });
      return handle;
    },
    change: function (node, value) {
      handle.act(function () {
        node.instance.field = value;
        if (typeof node.props.onChange === 'function') node.props.onChange({ type: 'change', target: { value: value } });
      });
      restoreControlled(node);
      return handle;
    },
    blur: function (node, value) {
      handle.act(function () {
        if (value !== undefined) node.instance.field = value;
        const v = node.instance.field === undefined ? '' : node.instance.field;
        if (typeof node.props.onBlur === 'function') node.props.onBlur({ type: 'blur', target: { value: v } });
      });
      restoreControlled(node);
      return handle;
    },
    /** What a form field shows (a string, like the DOM's `value`). */
    fieldValue: function (node) {
      const v = node.instance.field;
      return v === undefined || v === null ? '' : String(v);
    },
  });
  return handle;
}

export { textOf, htmlOf };
