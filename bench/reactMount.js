/**
 * Pages mounted on REAL React: react@18.3.1 + react-dom@18.3.1 production
 * UMD builds (what Headlamp serves users) committing with ReactDOM.flushSync
 * into the minimal DOM (tests/js/harness/minidom.js), through the shipped
 * renderer (src/view/react.js).
 */
import { createRenderer } from '../src/view/react.js';
import { ms, stats } from './common.js';

/** Real React 18.3.1 production builds + the shipped renderer, loaded on first use (umdDir: see reactDomMeasure). */
let realDom = null;
export async function realReact(umdDir) {
  if (!realDom) {
    const umd = await import('../tests/js/harness/umd-load.js');
    const cc = await import('../tests/js/harness/commonComponents.js');
    const loaded = umd.loadUmdReact(umdDir, 'production');
    const CC = cc.makeCommonComponents(loaded.React.createElement);
    realDom = { React: loaded.React, ReactDOM: loaded.ReactDOM, CC: CC, view: createRenderer(loaded.React, CC) };
  }
  return realDom;
}

/**
 * The same mount / re-render on REAL React: react@18.3.1 + react-dom@18.3.1
 * production UMD builds (what Headlamp serves users) committing with
 * ReactDOM.flushSync into the minimal DOM (tests/js/harness/minidom.js).
 * Median of `reps` mount + re-render + unmount cycles (the first warms the
 * JIT); elements = host elements in the container after the re-render.
 */
export async function reactDomMeasure(umdDir, vm, vm2, reps) {
  const R = await realReact(umdDir);
  const h = R.React.createElement;
  const mounts = [];
  const rerenders = [];
  let elements = 0;
  for (let i = 0; i < reps; i++) {
    const c = document.createElement('div');
    document.body.appendChild(c);
    const root = R.ReactDOM.createRoot(c);
    const t0 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(h(R.view.Page, { vm: vm })); });
    mounts.push(ms(process.hrtime(t0)));
    const t1 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(h(R.view.Page, { vm: vm2 })); });
    rerenders.push(ms(process.hrtime(t1)));
    elements = c.querySelectorAll('*').length;
    R.ReactDOM.flushSync(function () { root.unmount(); });
    document.body.removeChild(c);
  }
  return { mountMs: stats(mounts).p50, rerenderMs: stats(rerenders).p50, elements: elements, reps: reps };
}

/**
 * Mount `make()` into a fresh root on real React (flushSync), wait until the
 * container shows `waitText` when given (a page whose data arrives through an
 * effect: the reference's MetricsPage fetches in useEffect), then call
 * `beforeRerender()` (a watch event: a new context value) and render again.
 * Median over `reps` cycles of the mount and re-render wall times.
 */
export async function mountCycle(R, make, waitText, beforeRerender, reps, mustShow) {
  const mounts = [];
  const rerenders = [];
  let elements = 0;
  for (let i = 0; i < reps; i++) {
    const c = document.createElement('div');
    document.body.appendChild(c);
    const root = R.ReactDOM.createRoot(c);
    const t0 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(make()); });
    const errors = [];
    const consoleError = console.error;
    console.error = function () { errors.push(Array.prototype.join.call(arguments, ' ').slice(0, 500)); };
    try {
      const until = Date.now() + 60000;
      while (waitText && c.textContent.indexOf(waitText) < 0 && Date.now() < until && !errors.length) {
        await new Promise(function (r) { setImmediate(r); });
      }
    } finally {
      console.error = consoleError;
    }
    if (waitText && c.textContent.indexOf(waitText) < 0) {
      throw new Error('mountCycle: "' + waitText + '" never rendered' + (errors.length ? ': ' + errors.join(' | ') : ''));
    }
    mounts.push(ms(process.hrtime(t0)));
    if (mustShow && c.textContent.indexOf(mustShow) < 0) throw new Error('mountCycle: the page does not show "' + mustShow + '"');
    if (beforeRerender) beforeRerender();
    const t1 = process.hrtime();
    R.ReactDOM.flushSync(function () { root.render(make()); });
    rerenders.push(ms(process.hrtime(t1)));
    elements = c.querySelectorAll('*').length;
    R.ReactDOM.flushSync(function () { root.unmount(); });
    document.body.removeChild(c);
  }
  return { mountMs: stats(mounts).p50, rerenderMs: stats(rerenders).p50, elements: elements, reps: reps, mounts: mounts, rerenders: rerenders };
}
