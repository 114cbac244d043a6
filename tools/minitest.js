#!/usr/bin/env node
/**
 * minitest — a vitest-compatible test runner subset for Node 12.
 *
 * The container this repo is developed in has Node 12 and no npm registry,
 * so vitest cannot run here. Test files are written against the vitest
 * GLOBALS API (`describe`, `it`, `expect`, `vi`, `beforeEach`, `afterEach`;
 * vitest.config.mts sets `globals: true`) and run unchanged under both.
 *
 * Usage:
 *   node tools/minitest.js [--list] [--json OUT] file.test.js ...
 *
 * --list prints the test ids without running them (pytest collection);
 * --json writes [{id, file, name, ok, error, ms}] for the pytest bridge.
 */

import path from 'path';
import fs from 'fs';
import { pathToFileURL } from 'url';

// ---------------------------------------------------------------------------
// Registration
// ---------------------------------------------------------------------------

let currentFile = null;
const suiteStack = [];
const tests = [];

function hooks() {
  const be = [];
  const ae = [];
  for (let i = 0; i < suiteStack.length; i++) {
    be.push.apply(be, suiteStack[i].beforeEach);
    ae.unshift.apply(ae, suiteStack[i].afterEach);
  }
  return { be: be, ae: ae };
}

function describe(name, fn) {
  suiteStack.push({ name: name, beforeEach: [], afterEach: [] });
  try {
    fn();
  } finally {
    suiteStack.pop();
  }
}
describe.skip = function () {};

function it(name, fn) {
  const h = hooks();
  const full = suiteStack.map(function (s) { return s.name; }).concat([name]).join(' > ');
  tests.push({ file: currentFile, name: full, fn: fn, be: h.be, ae: h.ae });
}
it.skip = function () {};
it.each = function (table) {
  return function (name, fn) {
    table.forEach(function (row, i) {
      const args = Array.isArray(row) ? row : [row];
      let n = name;
      args.forEach(function (a) { n = n.replace(/%[sdij]/, typeof a === 'object' ? JSON.stringify(a) : String(a)); });
      if (n === name) n = name + ' [' + i + ']';
      it(n, function () { return fn.apply(null, args); });
    });
  };
};

function beforeEach(fn) {
  suiteStack[suiteStack.length - 1].beforeEach.push(fn);
}
function afterEach(fn) {
  suiteStack[suiteStack.length - 1].afterEach.push(fn);
}

// ---------------------------------------------------------------------------
// expect
// ---------------------------------------------------------------------------

function fmt(v) {
  try {
    if (typeof v === 'function') return '[Function]';
    if (v instanceof Error) return 'Error(' + v.message + ')';
    const s = JSON.stringify(v);
    return s === undefined ? String(v) : s.length > 300 ? s.slice(0, 300) + '…' : s;
  } catch (e) {
    return String(v);
  }
}

function deepEqual(a, b) {
  if (a === b) return true;
  if (typeof a === 'number' && typeof b === 'number' && isNaN(a) && isNaN(b)) return true;
  if (a === null || b === null || typeof a !== 'object' || typeof b !== 'object') {
    if (b && b.__asymmetric) return b.match(a);
    return false;
  }
  if (b.__asymmetric) return b.match(a);
  if (Array.isArray(a) !== Array.isArray(b)) return false;
  if (Array.isArray(a)) {
    if (a.length !== b.length) return false;
    for (let i = 0; i < a.length; i++) if (!deepEqual(a[i], b[i])) return false;
    return true;
  }
  const ka = Object.keys(a).filter(function (k) { return a[k] !== undefined; });
  const kb = Object.keys(b).filter(function (k) { return b[k] !== undefined; });
  if (ka.length !== kb.length) return false;
  for (let i = 0; i < kb.length; i++) if (!deepEqual(a[kb[i]], b[kb[i]])) return false;
  return true;
}

function subsetMatch(a, b) {
  if (b && b.__asymmetric) return b.match(a);
  if (b === null || typeof b !== 'object') return deepEqual(a, b);
  if (a === null || typeof a !== 'object') return false;
  for (const k in b) if (!subsetMatch(a[k], b[k])) return false;
  return true;
}

function AssertionError(msg) {
  const e = new Error(msg);
  e.name = 'AssertionError';
  return e;
}

function makeMatchers(actual, negate, label) {
  function check(pass, msg) {
    if (negate ? pass : !pass) throw AssertionError((label ? label + ': ' : '') + (negate ? 'NOT ' : '') + msg);
  }
  const m = {
    toBe: function (e) { check(Object.is(actual, e), 'expected ' + fmt(actual) + ' to be ' + fmt(e)); },
    toEqual: function (e) { check(deepEqual(actual, e), 'expected ' + fmt(actual) + ' to equal ' + fmt(e)); },
    toStrictEqual: function (e) { check(deepEqual(actual, e), 'expected ' + fmt(actual) + ' to strictly equal ' + fmt(e)); },
    toMatchObject: function (e) { check(subsetMatch(actual, e), 'expected ' + fmt(actual) + ' to match ' + fmt(e)); },
    toBeNull: function () { check(actual === null, 'expected ' + fmt(actual) + ' to be null'); },
    toBeUndefined: function () { check(actual === undefined, 'expected ' + fmt(actual) + ' to be undefined'); },
    toBeDefined: function () { check(actual !== undefined, 'expected value to be defined'); },
    toBeTruthy: function () { check(!!actual, 'expected ' + fmt(actual) + ' to be truthy'); },
    toBeFalsy: function () { check(!actual, 'expected ' + fmt(actual) + ' to be falsy'); },
    toBeNaN: function () { check(typeof actual === 'number' && isNaN(actual), 'expected NaN'); },
    toHaveLength: function (n) {
      check(actual !== null && actual !== undefined && actual.length === n,
        'expected length ' + (actual ? actual.length : actual) + ' to be ' + n);
    },
    toContain: function (e) {
      const ok = typeof actual === 'string' ? actual.indexOf(e) >= 0 : Array.isArray(actual) && actual.indexOf(e) >= 0;
      check(ok, 'expected ' + fmt(actual) + ' to contain ' + fmt(e));
    },
    toContainEqual: function (e) {
      check(Array.isArray(actual) && actual.some(function (x) { return deepEqual(x, e); }), 'expected ' + fmt(actual) + ' to contain equal ' + fmt(e));
    },
    toMatch: function (re) {
      const ok = typeof actual === 'string' && (re instanceof RegExp ? re.test(actual) : actual.indexOf(re) >= 0);
      check(ok, 'expected ' + fmt(actual) + ' to match ' + String(re));
    },
    toBeGreaterThan: function (n) { check(actual > n, 'expected ' + actual + ' > ' + n); },
    toBeGreaterThanOrEqual: function (n) { check(actual >= n, 'expected ' + actual + ' >= ' + n); },
    toBeLessThan: function (n) { check(actual < n, 'expected ' + actual + ' < ' + n); },
    toBeLessThanOrEqual: function (n) { check(actual <= n, 'expected ' + actual + ' <= ' + n); },
    toBeCloseTo: function (n, digits) {
      const d = digits === undefined ? 2 : digits;
      check(Math.abs(actual - n) < Math.pow(10, -d) / 2, 'expected ' + actual + ' to be close to ' + n);
    },
    toBeInstanceOf: function (c) { check(actual instanceof c, 'expected instance of ' + (c && c.name)); },
    toHaveProperty: function (k, v) {
      const has = actual !== null && actual !== undefined && Object.prototype.hasOwnProperty.call(Object(actual), k);
      check(has && (arguments.length < 2 || deepEqual(actual[k], v)), 'expected property ' + k + (arguments.length > 1 ? '=' + fmt(v) : ''));
    },
    toThrow: function (expected) {
      let threw = false;
      let err = null;
      try {
        actual();
      } catch (e) {
        threw = true;
        err = e;
      }
      let ok = threw;
      if (threw && expected !== undefined) {
        const msg = err && err.message !== undefined ? err.message : String(err);
        ok = expected instanceof RegExp ? expected.test(msg) : msg.indexOf(expected) >= 0;
      }
      check(ok, 'expected function to throw' + (expected !== undefined ? ' ' + String(expected) : '') + (err ? ' (got ' + err.message + ')' : ''));
    },
    toHaveBeenCalled: function () { check(actual.mock.calls.length > 0, 'expected mock to have been called'); },
    toHaveBeenCalledTimes: function (n) {
      check(actual.mock.calls.length === n, 'expected ' + n + ' calls, got ' + actual.mock.calls.length);
    },
    toHaveBeenCalledWith: function () {
      const args = Array.prototype.slice.call(arguments);
      check(actual.mock.calls.some(function (c) { return deepEqual(c, args); }),
        'expected a call with ' + fmt(args) + ', calls: ' + fmt(actual.mock.calls));
    },
    toHaveBeenLastCalledWith: function () {
      const args = Array.prototype.slice.call(arguments);
      const calls = actual.mock.calls;
      check(calls.length > 0 && deepEqual(calls[calls.length - 1], args),
        'expected the last call with ' + fmt(args) + ', calls: ' + fmt(calls));
    },
  };
  return m;
}

function expect(actual, label) {
  const m = makeMatchers(actual, false, label);
  m.not = makeMatchers(actual, true, label);
  m.resolves = wrapAsync(actual, false);
  m.rejects = wrapAsync(actual, true);
  return m;
}

function wrapAsync(promise, expectReject) {
  const out = {};
  const names = Object.keys(makeMatchers(null, false));
  names.forEach(function (n) {
    out[n] = function () {
      const args = arguments;
      return Promise.resolve(promise).then(
        function (v) {
          if (expectReject) throw AssertionError('expected promise to reject, resolved ' + fmt(v));
          return makeMatchers(v, false)[n].apply(null, args);
        },
        function (e) {
          if (!expectReject) throw AssertionError('expected promise to resolve, rejected ' + fmt(e));
          if (n === 'toThrow') {
            const msg = e && e.message !== undefined ? e.message : String(e);
            const exp = args[0];
            if (exp !== undefined && !(exp instanceof RegExp ? exp.test(msg) : msg.indexOf(exp) >= 0)) {
              throw AssertionError('expected rejection ' + String(exp) + ', got ' + msg);
            }
            return undefined;
          }
          return makeMatchers(e, false)[n].apply(null, args);
        }
      );
    };
  });
  return out;
}

expect.any = function (ctor) {
  return {
    __asymmetric: true,
    match: function (v) {
      if (ctor === String) return typeof v === 'string';
      if (ctor === Number) return typeof v === 'number';
      if (ctor === Boolean) return typeof v === 'boolean';
      if (ctor === Function) return typeof v === 'function';
      if (ctor === Object) return v !== null && typeof v === 'object';
      return v instanceof ctor;
    },
  };
};
expect.stringContaining = function (s) {
  return { __asymmetric: true, match: function (v) { return typeof v === 'string' && v.indexOf(s) >= 0; } };
};
expect.objectContaining = function (o) {
  return { __asymmetric: true, match: function (v) { return subsetMatch(v, o); } };
};

// ---------------------------------------------------------------------------
// vi
// ---------------------------------------------------------------------------

function fn(impl) {
  let base = impl;
  let onces = [];
  const mock = function () {
    const args = Array.prototype.slice.call(arguments);
    mock.mock.calls.push(args);
    const f = onces.length ? onces.shift() : base;
    const r = f ? f.apply(this, args) : undefined;
    mock.mock.results.push({ type: 'return', value: r });
    return r;
  };
  mock.mock = { calls: [], results: [] };
  mock._isMockFunction = true;
  mock.mockImplementation = function (f) { base = f; return mock; };
  mock.mockImplementationOnce = function (f) { onces.push(f); return mock; };
  mock.mockReturnValue = function (v) { base = function () { return v; }; return mock; };
  mock.mockReturnValueOnce = function (v) { onces.push(function () { return v; }); return mock; };
  mock.mockResolvedValue = function (v) { base = function () { return Promise.resolve(v); }; return mock; };
  mock.mockResolvedValueOnce = function (v) { onces.push(function () { return Promise.resolve(v); }); return mock; };
  mock.mockRejectedValue = function (e) { base = function () { return Promise.reject(e); }; return mock; };
  mock.mockRejectedValueOnce = function (e) { onces.push(function () { return Promise.reject(e); }); return mock; };
  mock.mockClear = function () { mock.mock.calls = []; mock.mock.results = []; return mock; };
  mock.mockReset = function () { mock.mockClear(); base = undefined; onces = []; return mock; };
  return mock;
}

// Fake timers: patch setTimeout/clearTimeout/setInterval/Date.now.
const real = { setTimeout: setTimeout, clearTimeout: clearTimeout, setInterval: setInterval, clearInterval: clearInterval, now: Date.now };
let fake = null;

function useFakeTimers() {
  if (fake) return vi;
  fake = { now: real.now(), id: 1, timers: [] };
  global.setTimeout = function (cb, ms) {
    const args = Array.prototype.slice.call(arguments, 2);
    const t = { id: fake.id++, at: fake.now + (ms || 0), cb: cb, args: args, every: 0 };
    fake.timers.push(t);
    return t.id;
  };
  global.setInterval = function (cb, ms) {
    const t = { id: fake.id++, at: fake.now + (ms || 0), cb: cb, args: [], every: ms || 1 };
    fake.timers.push(t);
    return t.id;
  };
  global.clearTimeout = global.clearInterval = function (id) {
    if (!fake) return;
    fake.timers = fake.timers.filter(function (t) { return t.id !== id; });
  };
  Date.now = function () { return fake.now; };
  return vi;
}

function useRealTimers() {
  global.setTimeout = real.setTimeout;
  global.clearTimeout = real.clearTimeout;
  global.setInterval = real.setInterval;
  global.clearInterval = real.clearInterval;
  Date.now = real.now;
  fake = null;
  return vi;
}

function advanceTimersByTime(ms) {
  if (!fake) throw new Error('advanceTimersByTime requires vi.useFakeTimers()');
  const target = fake.now + ms;
  for (;;) {
    fake.timers.sort(function (a, b) { return a.at - b.at || a.id - b.id; });
    const t = fake.timers[0];
    if (!t || t.at > target) break;
    fake.now = t.at;
    if (t.every) t.at += t.every;
    else fake.timers.shift();
    t.cb.apply(null, t.args);
  }
  fake.now = target;
  return vi;
}

function flushMicrotasks() {
  return new Promise(function (r) { real.setTimeout(r, 0); });
}

const vi = {
  fn: fn,
  useFakeTimers: useFakeTimers,
  useRealTimers: useRealTimers,
  advanceTimersByTime: advanceTimersByTime,
  advanceTimersByTimeAsync: function (ms) {
    // Interleave timer firing with microtask flushing so promise chains that
    // schedule further timers make progress (vitest semantics).
    const target = fake.now + ms;
    function step() {
      fake.timers.sort(function (a, b) { return a.at - b.at || a.id - b.id; });
      const t = fake.timers[0];
      if (!t || t.at > target) {
        fake.now = target;
        return flushMicrotasks();
      }
      fake.now = t.at;
      if (t.every) t.at += t.every;
      else fake.timers.shift();
      t.cb.apply(null, t.args);
      return flushMicrotasks().then(step);
    }
    return flushMicrotasks().then(step);
  },
  getTimerCount: function () { return fake ? fake.timers.length : 0; },
  setSystemTime: function (t) { if (fake) fake.now = typeof t === 'number' ? t : new Date(t).getTime(); },
  isMockFunction: function (f) { return !!(f && f._isMockFunction); },
};

global.describe = describe;
global.it = it;
global.test = it;
global.expect = expect;
global.beforeEach = beforeEach;
global.afterEach = afterEach;
global.vi = vi;
// Each file gets its own unnamed root suite (main() swaps it in before the
// file is imported), so file-level hooks apply to that file's tests only, as
// in vitest. The root suite's name must not appear in ids.
suiteStack.push({ name: '', beforeEach: [], afterEach: [] });
const origIt = it;
void origIt;

// ---------------------------------------------------------------------------
// Run
// ---------------------------------------------------------------------------

function idOf(t) {
  return t.file + '::' + t.name.replace(/^ > /, '');
}

function runWithTimeout(p, ms) {
  return new Promise(function (resolve, reject) {
    const h = real.setTimeout(function () { reject(new Error('test timed out after ' + ms + 'ms')); }, ms);
    Promise.resolve(p).then(
      function (v) { real.clearTimeout(h); resolve(v); },
      function (e) { real.clearTimeout(h); reject(e); }
    );
  });
}

async function runAll(list) {
  const results = [];
  for (let i = 0; i < list.length; i++) {
    const t = list[i];
    const start = process.hrtime();
    let ok = true;
    let error = null;
    try {
      for (let j = 0; j < t.be.length; j++) await t.be[j]();
      await runWithTimeout(t.fn(), 10000);
    } catch (e) {
      ok = false;
      error = e && e.stack ? e.stack.split('\n').slice(0, 6).join('\n') : String(e);
    }
    try {
      for (let j = 0; j < t.ae.length; j++) await t.ae[j]();
    } catch (e) {
      if (ok) {
        ok = false;
        error = 'afterEach: ' + (e && e.message);
      }
    }
    if (fake) useRealTimers();
    const d = process.hrtime(start);
    results.push({ id: idOf(t), file: t.file, name: t.name.replace(/^ > /, ''), ok: ok, error: error, ms: d[0] * 1e3 + d[1] / 1e6 });
  }
  return results;
}

async function main() {
  const argv = process.argv.slice(2);
  let list = false;
  let jsonOut = null;
  let filter = null;
  const files = [];
  for (let i = 0; i < argv.length; i++) {
    if (argv[i] === '--list') list = true;
    else if (argv[i] === '--json') jsonOut = argv[++i];
    else if (argv[i] === '--filter') filter = argv[++i];
    else files.push(argv[i]);
  }
  const root = process.cwd();
  for (let i = 0; i < files.length; i++) {
    const abs = path.resolve(files[i]);
    currentFile = path.relative(root, abs);
    suiteStack[0] = { name: '', beforeEach: [], afterEach: [] };
    await import(pathToFileURL(abs).href);
  }
  let selected = tests;
  if (filter) selected = tests.filter(function (t) { return idOf(t).indexOf(filter) >= 0; });
  if (list) {
    const ids = selected.map(idOf);
    if (jsonOut) fs.writeFileSync(jsonOut, JSON.stringify(ids));
    else process.stdout.write(ids.join('\n') + '\n');
    return;
  }
  const results = await runAll(selected);
  const failed = results.filter(function (r) { return !r.ok; });
  if (jsonOut) fs.writeFileSync(jsonOut, JSON.stringify(results));
  for (let i = 0; i < failed.length; i++) process.stdout.write('FAIL ' + failed[i].id + '\n' + failed[i].error + '\n');
  process.stdout.write(results.length - failed.length + ' passed, ' + failed.length + ' failed\n');
  process.exitCode = failed.length ? 1 : 0;
}

main().catch(function (e) {
  process.stderr.write(String(e && e.stack ? e.stack : e) + '\n');
  process.exitCode = 2;
});
