/**
 * Load REAL React 18.3.1 + react-dom from their UMD builds, offline, into a
 * private sandbox over the minimal DOM (./minidom.js), installed as the global
 * window / document first (react-dom probes them at load time).
 *
 *   build 'development' — react@18.3.1.js / react-dom@18.3.1.js: act(), the
 *     dev warnings; the real-React spec tier (./umd-react.js).
 *   build 'production'  — the .min.js builds Headlamp ships to users: no
 *     act(), commits with ReactDOM.flushSync; the bench's real-React
 *     mount / re-render figure (bench/driver.js).
 */
import fs from 'fs';
import path from 'path';
import vm from 'vm';
import { createWindow } from './minidom.js';

const FILES = {
  development: ['react@18.3.1.js', 'react-dom@18.3.1.js'],
  production: ['react@18.3.1.min.js', 'react-dom@18.3.1.min.js'],
};

/** The window / document / navigator globals react-dom expects (kept if already there). */
export function installDom() {
  if (typeof globalThis.window === 'undefined') {
    const w = createWindow();
    globalThis.window = w;
    globalThis.document = w.document;
    globalThis.navigator = w.navigator;
  }
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
}

/**
 * @param {string} dir directory holding the UMD files
 * @param {'development'|'production'} build
 * @returns {{React: object, ReactDOM: object}}
 */
export function loadUmdReact(dir, build) {
  const files = FILES[build || 'development'];
  if (!files) throw new Error('unknown React build ' + build);
  if (!dir) throw new Error('no directory holding ' + files.join(' / '));
  installDom();
  const sandbox = {};
  for (let i = 0; i < files.length; i++) {
    const src = fs.readFileSync(path.join(dir, files[i]), 'utf8');
    // The UMD wrapper registers on `this` when neither CommonJS nor AMD is
    // around — on `self` in the .min.js builds, whose strict-mode IIFE leaves
    // `this` undefined: both are the sandbox.
    // Compiled as a script (not by the Function constructor), so it also loads in a process started with
    // --disallow-code-generation-from-strings (the opt-in render comparison, bench/compareRenders.js).
    vm.runInThisContext('(function (self) {' + src + '\n})', { filename: files[i] }).call(sandbox, sandbox);
  }
  const React = sandbox.React;
  const ReactDOM = sandbox.ReactDOM;
  if (!React || React.version !== '18.3.1' || !ReactDOM || !ReactDOM.createRoot) {
    throw new Error('react@18.3.1 / react-dom@18.3.1 UMD builds did not load from ' + dir);
  }
  return { React: React, ReactDOM: ReactDOM };
}
