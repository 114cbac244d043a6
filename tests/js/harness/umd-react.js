/**
 * REAL React 18 + react-dom for bare Node, offline: the UMD development
 * builds of react@18.3.1 / react-dom@18.3.1 (the versions package.json pins),
 * taken from a directory that already holds them — AMD_REACT_UMD_DIR; the
 * pytest wrapper (tests/test_js_real_react.py) points it at the copies an
 * installed Python package vendors — and evaluated against the minimal DOM
 * in ./minidom.js (./umd-load.js).
 *
 * tools/plugin-loader.js maps 'react' here when AMD_TEST_TIER=react-umd, so
 * the shipped plugin code and the shared specs get this React.
 */
import { loadUmdReact } from './umd-load.js';

const dir = process.env.AMD_REACT_UMD_DIR;
if (!dir) throw new Error('AMD_REACT_UMD_DIR is not set (a directory holding react@18.3.1.js and react-dom@18.3.1.js)');

const loaded = loadUmdReact(dir, 'development');
// React 18: updates are expected inside act() in a test environment.
globalThis.IS_REACT_ACT_ENVIRONMENT = true;

const React = loaded.React;
export const ReactDOM = loaded.ReactDOM;

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
