/**
 * REAL React 18 + react-dom for bare Node, offline: the UMD development
 * builds of react@18.3.1 / react-dom@18.3.1 (the versions package.json pins),
 * taken from a directory that already holds them — AMD_REACT_UMD_DIR; the
 * pytest wrapper (tests/test_js_real_react.py) points it at the copies an
 * installed Python package vendors — and evaluated against the minimal DOM
 * in ./minidom.js, installed as the global window / document before
 * react-dom loads (it probes them at load time).
 *
 * tools/plugin-loader.js maps 'react' here when AMD_TEST_TIER=react-umd, so
 * the shipped plugin code and the shared specs get this React.
 */
import fs from 'fs';
import path from 'path';
import { createWindow } from './minidom.js';

const dir = process.env.AMD_REACT_UMD_DIR;
if (!dir) throw new Error('AMD_REACT_UMD_DIR is not set (a directory holding react@18.3.1.js and react-dom@18.3.1.js)');

if (typeof globalThis.window === 'undefined') {
  const w = createWindow();
  globalThis.window = w;
  globalThis.document = w.document;
  globalThis.navigator = w.navigator;
}
// React 18: updates are expected inside act() in a test environment.
globalThis.IS_REACT_ACT_ENVIRONMENT = true;
// async act() queues its flush on a MessageChannel when it cannot require
// Node's timers (a UMD build has no `require`); Node 12 has no global one.
// This one posts with setImmediate and holds no port open.
if (typeof globalThis.MessageChannel === 'undefined') {
  globalThis.MessageChannel = function MessageChannel() {
    const port1 = { onmessage: null };
    this.port1 = port1;
    this.port2 = {
      postMessage: function (data) {
        setImmediate(function () { if (port1.onmessage) port1.onmessage({ data: data }); });
      },
    };
  };
}

const sandbox = {};
function load(file) {
  const src = fs.readFileSync(path.join(dir, file), 'utf8');
  // The UMD wrapper registers on `this` when neither CommonJS nor AMD is around.
  new Function(src).call(sandbox); // eslint-disable-line no-new-func
}
load('react@18.3.1.js');
load('react-dom@18.3.1.js');

const React = sandbox.React;
export const ReactDOM = sandbox.ReactDOM;
if (!React || React.version !== '18.3.1' || !ReactDOM || !ReactDOM.createRoot) {
  throw new Error('react@18.3.1 / react-dom@18.3.1 UMD builds did not load from ' + dir);
}

export default React;
export const Children = React.Children;
export const Component = React.Component;
export const Fragment = React.Fragment;
export const StrictMode = React.StrictMode;
export const act = React.act;
export const createContext = React.createContext;
export const createElement = React.createElement;
export const isValidElement = React.isValidElement;
export const memo = React.memo;
export const useCallback = React.useCallback;
export const useContext = React.useContext;
export const useEffect = React.useEffect;
export const useLayoutEffect = React.useLayoutEffect;
export const useMemo = React.useMemo;
export const useReducer = React.useReducer;
export const useRef = React.useRef;
export const useState = React.useState;
export const useSyncExternalStore = React.useSyncExternalStore;
export const version = React.version;
