/**
 * The reference's page components in a realm of their own, inside a process
 * of its own (ADR 014). BENCHMARK ONLY: tools/render_compare.py
 * --allow-reference-exec mounts the reference's pages next to this plugin's.
 *
 * The reference's sources are untrusted public content. This file is the
 * whole of the process that runs them:
 *
 *   * the process (bench/refIsolated.js starts it) has no network (a network
 *     namespace of its own), a read-only root file system, no capabilities,
 *     RLIMIT_FSIZE 0, an environment of PATH alone, and V8's
 *     --disallow-code-generation-from-strings. It reads no file: this source,
 *     React, the DOM stand-in and the reference's transpiled modules arrive as
 *     strings on stdin, the cluster as JSON; it answers with numbers;
 *   * inside it, everything the reference can reach is built in a vm context
 *     from source text — the minimal DOM and CommonComponents stand-ins
 *     (bench/refHarness.js, bundled), react@18.3.1 / react-dom@18.3.1 from
 *     their UMD sources, the module table — and the data enters as JSON text
 *     parsed there. No host object is handed in: the host calls the realm's
 *     own functions with strings and numbers and times them. `audit()` walks
 *     everything reachable from the context's global object and reports any
 *     path to `process`, `require`, a host-realm function or a host-realm
 *     object (tests/js/refRealm.test.js, tests/test_render_compare.py).
 *
 * Every script evaluated in the context is wrapped in a function that binds
 * the context's globals as locals (`wrap`): a contextified global object
 * answers property lookups through an interceptor, which made React mount
 * about twice as slowly as in the main realm; bound lexically it runs at the
 * main realm's speed (`calibrate` measures both sides on the same tree).
 */
'use strict';

/** Global names the lexical prelude may bind (identifiers that strict code may declare). */
const UNBINDABLE = { eval: true, arguments: true, undefined: true, NaN: true, Infinity: true, globalThis: true };

function globalNames(vm, ctx) {
  const names = vm.runInContext('Object.getOwnPropertyNames(globalThis)', ctx);
  const out = [];
  for (let i = 0; i < names.length; i++) {
    const n = names[i];
    if (typeof n === 'string' && /^[A-Za-z_$][\w$]*$/.test(n) && !UNBINDABLE[n]) out.push(n);
  }
  return out;
}

/** `src` as a script whose free references to the context's current globals are lexical. */
function wrap(names, src) {
  const bind = names.length ? 'var ' + names.map(function (n) { return n + ' = globalThis.' + n; }).join(', ') + ';\n' : '';
  return '(function () {\n' + bind + src + '\n})();';
}

// ---------------------------------------------------------------------------
// Code that runs INSIDE the context (its source text is evaluated there)
// ---------------------------------------------------------------------------

/** Console, timers and the DOM globals, all of the context's own making. */
function realmPrelude() {
  var errors = [];
  var timers = [];
  var nextId = 0;
  function note() { errors.push(Array.prototype.join.call(arguments, ' ').slice(0, 500)); }
  globalThis.console = { error: note, warn: function () {}, log: function () {}, info: function () {}, debug: function () {} };
  // A timer queue the host drains: React's scheduler posts its work here.
  globalThis.setTimeout = function (fn) {
    var id = ++nextId;
    timers.push({ id: id, fn: fn, args: Array.prototype.slice.call(arguments, 2) });
    return id;
  };
  globalThis.clearTimeout = function (id) {
    timers = timers.filter(function (t) { return t.id !== id; });
  };
  globalThis.__realm = {
    errors: errors,
    drain: function () {
      var n = 0;
      while (timers.length && n < 10000) {
        var t = timers.shift();
        t.fn.apply(null, t.args);
        n++;
      }
      return n;
    },
  };
  var w = globalThis.__harness.createWindow();
  globalThis.window = w;
  globalThis.document = w.document;
  globalThis.navigator = w.navigator;
  globalThis.self = globalThis;
}

/**
 * The bench's API over the reference's modules (`__defs`, from the module
 * table): `resolve[id][spec]` is {file: id} or {ext: name}; `pages` maps a
 * page key to its module id. Every entry point takes and returns strings
 * and numbers.
 */
function realmBench(resolve, pages) {
  var CC = __harness.makeCommonComponents(React.createElement);
  var data = { ctx: null, base: null, metrics: null, nodes: null, pods: null };
  var ext = {
    react: React,
    '@kinvolk/headlamp-plugin/lib/CommonComponents': CC,
    '@kinvolk/headlamp-plugin/lib': { ApiProxy: { request: function () { return Promise.reject(new Error('no network in the render bench')); } } },
    '../api/IntelGpuDataContext': {
      useIntelGpuContext: function () {
        if (!data.ctx) throw new Error('useIntelGpuContext must be used within an IntelGpuDataProvider');
        return data.ctx;
      },
    },
  };
  var cache = {};
  function load(id) {
    if (cache[id]) return cache[id];
    if (!__defs[id]) throw new Error('realm: no module ' + id);
    var exp = {};
    cache[id] = exp;
    __defs[id](function (spec, wantDefault) {
      var r = resolve[id] && resolve[id][spec];
      if (!r) throw new Error('realm: ' + id + ' imports ' + spec + ', which is not resolved');
      var m = r.file ? load(r.file) : ext[r.ext];
      if (m === undefined) throw new Error('realm: no external ' + r.ext);
      if (!wantDefault) return m;
      return m && m.default !== undefined ? m.default : m;
    }, exp);
    return exp;
  }
  var k8s = load('api/k8s.ts');
  var real = load('api/metrics.ts');
  // fetchGpuMetrics answers from the synthetic cluster (as MetricsPage.test.tsx mocks it); the formatters are the reference's.
  var standIn = {};
  for (var k in real) standIn[k] = real[k];
  standIn.fetchGpuMetrics = function () { return Promise.resolve(data.metrics); };
  ext['../api/metrics'] = standIn;
  var comps = {};
  for (var p in pages) comps[p] = load(pages[p]).default;
  var container = null;
  var root = null;
  var current = null;
  globalThis.__bench = {
    /** The cluster, in the reference's shapes (JSON): its provider's context value, filtered by its own helpers. */
    setData: function (json) {
      var d = JSON.parse(json);
      data.nodes = d.nodes;
      data.pods = d.pods;
      data.metrics = d.metrics;
      data.base = {
        devicePlugins: d.devicePlugins,
        pluginInstalled: d.devicePlugins.length > 0 || d.pluginPods.length > 0,
        gpuNodes: k8s.filterIntelGpuNodes(d.nodes),
        gpuPods: k8s.filterGpuRequestingPods(d.pods),
        pluginPods: d.pluginPods,
        crdAvailable: true,
        loading: false,
        error: null,
        refresh: function () {},
      };
      data.ctx = data.base;
      return JSON.stringify({ gpuNodes: data.base.gpuNodes.length, gpuPods: data.base.gpuPods.length, chips: d.metrics.chips.length });
    },
    /** The provider's per-watch-event filtering of both whole lists (IntelGpuDataContext.tsx:200-208). */
    filter: function () {
      return k8s.filterIntelGpuNodes(data.nodes).length + k8s.filterGpuRequestingPods(data.pods).length;
    },
    mount: function (page) {
      current = comps[page];
      if (!current) throw new Error('realm: no page ' + page);
      data.ctx = data.base;
      container = document.createElement('div');
      document.body.appendChild(container);
      root = ReactDOM.createRoot(container);
      ReactDOM.flushSync(function () { root.render(React.createElement(current)); });
    },
    /** A watch event: a new context value (new arrays of the same objects). */
    event: function () {
      var b = data.base;
      var c = {};
      for (var f in b) c[f] = b[f];
      c.gpuNodes = b.gpuNodes.slice();
      c.gpuPods = b.gpuPods.slice();
      c.pluginPods = b.pluginPods.slice();
      c.devicePlugins = b.devicePlugins.slice();
      data.ctx = c;
    },
    rerender: function () {
      ReactDOM.flushSync(function () { root.render(React.createElement(current)); });
    },
    text: function () { return container.textContent; },
    elements: function () { return container.querySelectorAll('*').length; },
    unmount: function () {
      ReactDOM.flushSync(function () { root.unmount(); });
      document.body.removeChild(container);
      container = null;
      root = null;
    },
    drain: function () { return __realm.drain(); },
    errors: function () { return __realm.errors.splice(0).join(' | '); },
    /** The calibration tree (the same as bench/refIsolated.js mounts in the driver's realm). */
    calibrate: function (rows) {
      var h = React.createElement;
      var trs = [];
      for (var i = 0; i < rows; i++) trs.push(h('tr', { key: i }, h('td', null, 'node-' + i), h('td', null, String(i * 7))));
      container = document.createElement('div');
      document.body.appendChild(container);
      root = ReactDOM.createRoot(container);
      ReactDOM.flushSync(function () { root.render(h('table', null, h('tbody', null, trs))); });
      var n = container.querySelectorAll('*').length;
      ReactDOM.flushSync(function () { root.unmount(); });
      document.body.removeChild(container);
      return n;
    },
  };
}

// ---------------------------------------------------------------------------
// The realm, seen from the worker
// ---------------------------------------------------------------------------

/**
 * Build the realm: `init` = {harness: script expression (bench/refHarness.js
 * bundled), react, reactDom: UMD sources, modules: {id: transpiled body},
 * resolve, pages}. Returns {api, ctx}: `api` the context's own __bench
 * object (its functions take and return primitives).
 */
function createRealm(vm, init) {
  const ctx = vm.createContext(Object.create(null), { name: 'reference-realm', codeGeneration: { strings: false, wasm: false } });
  function run(src, filename) {
    new vm.Script(wrap(globalNames(vm, ctx), src), { filename: filename }).runInContext(ctx, { timeout: 20000 });
  }
  run('globalThis.pluginLib = {};\nglobalThis.__harness = (' + init.harness.trim().replace(/;$/, '') + '\n);', 'realm:harness');
  run('(' + realmPrelude.toString() + ')();', 'realm:prelude');
  // The UMD wrapper registers on `self` (the .min.js builds) or `this`: both the context's global.
  run('(function (self) {' + init.react + '\n}).call(globalThis, globalThis);', 'react@18.3.1.min.js');
  run('(function (self) {' + init.reactDom + '\n}).call(globalThis, globalThis);', 'react-dom@18.3.1.min.js');
  const ids = Object.keys(init.modules);
  let table = 'globalThis.__defs = {\n';
  for (let i = 0; i < ids.length; i++) {
    table += JSON.stringify(ids[i]) + ': function (__import, __exports) {"use strict";\n' + init.modules[ids[i]] + '\n},\n';
  }
  run(table + '};', 'realm:modules');
  run('(' + realmBench.toString() + ')(' + JSON.stringify(init.resolve) + ', ' + JSON.stringify(init.pages) + ');', 'realm:bench');
  // react-dom's UMD says "18.3.1-next-<commit>-<date>"
  const version = vm.runInContext('React.version + "/" + ReactDOM.version.split("-")[0]', ctx);
  if (version !== '18.3.1/18.3.1') throw new Error('realm: react / react-dom 18.3.1 did not load (' + version + ')');
  return { api: vm.runInContext('__bench', ctx), ctx: ctx };
}

/**
 * Everything reachable from the context's global object (own properties of
 * every kind, accessor functions, prototypes), checked for a way out: the
 * host's `process` or `require`, a function of the host realm (its
 * constructor compiles code in the host), an object whose prototype chain is
 * the host's. `host` = {process, require, Function, Object} of the caller.
 */
function audit(vm, ctx, host) {
  const seen = new Set();
  const queue = [vm.runInContext('globalThis', ctx)];
  const leaks = [];
  function visit(v, where) {
    if (v === null || (typeof v !== 'object' && typeof v !== 'function') || seen.has(v)) return;
    seen.add(v);
    if (v === host.process) leaks.push(where + ': process');
    else if (host.require && v === host.require) leaks.push(where + ': require');
    else if (v instanceof host.Function) leaks.push(where + ': a host-realm function');
    else if (v instanceof host.Object) leaks.push(where + ': a host-realm object');
    queue.push(v);
    paths.set(v, where);
  }
  const paths = new Map();
  paths.set(queue[0], 'globalThis');
  seen.add(queue[0]);
  while (queue.length && leaks.length < 20) {
    const o = queue.shift();
    const at = paths.get(o) || '?';
    visit(Object.getPrototypeOf(o), at + '.__proto__');
    const keys = Object.getOwnPropertyNames(o).concat(Object.getOwnPropertySymbols(o));
    for (let i = 0; i < keys.length; i++) {
      const d = Object.getOwnPropertyDescriptor(o, keys[i]);
      if (!d) continue;
      const name = at + '.' + String(keys[i]);
      if ('value' in d) visit(d.value, name);
      visit(d.get, name + '<get>');
      visit(d.set, name + '<set>');
    }
  }
  return { objects: seen.size, leaks: leaks };
}

/** Mount / wait / re-render / unmount of one page, timed here (ms), as bench/reactMount.js mountCycle does in the driver. */
async function cycle(api, c, yieldFn) {
  const ms = function (t) { return t[0] * 1e3 + t[1] / 1e6; };
  const t0 = process.hrtime();
  api.mount(c.page);
  let errors = '';
  for (let spins = 0; c.waitText && api.text().indexOf(c.waitText) < 0 && spins < 100000 && !errors; spins++) {
    await yieldFn();
    api.drain();
    errors = api.errors();
  }
  if (c.waitText && api.text().indexOf(c.waitText) < 0) {
    throw new Error('realm: "' + c.waitText + '" never rendered' + (errors ? ': ' + errors : ''));
  }
  const mount = ms(process.hrtime(t0));
  if (c.mustShow && api.text().indexOf(c.mustShow) < 0) throw new Error('realm: the page does not show "' + c.mustShow + '"');
  api.event();
  const t1 = process.hrtime();
  api.rerender();
  const rerender = ms(process.hrtime(t1));
  const elements = api.elements();
  api.unmount();
  return { mount: mount, rerender: rerender, elements: elements };
}

/** The worker's own isolation, tried: a write to a few places, a TCP connection out. */
function probe(fs, net) {
  const out = { writes: {}, connect: null };
  const targets = ['/tmp/.ref-probe', '/dev/shm/.ref-probe', process.cwd() + '/.ref-probe'];
  for (let i = 0; i < targets.length; i++) {
    try {
      fs.writeFileSync(targets[i], 'x');
      out.writes[targets[i]] = 'written';
    } catch (e) {
      out.writes[targets[i]] = e.code || String(e);
    }
  }
  return new Promise(function (resolve) {
    const s = net.connect({ host: '1.1.1.1', port: 80 });
    const done = function (v) { out.connect = v; s.destroy(); resolve(out); };
    s.setTimeout(3000, function () { done('timeout'); });
    s.on('error', function (e) { done(e.code || String(e)); });
    s.on('connect', function () { done('connected'); });
  });
}

/**
 * JSON lines in on stdin ({id, cmd, ...}), JSON lines out ({id, ok, result | error}).
 * Commands: init, setData, filter, cycle, calibrate, audit, probe.
 */
function serve(vm, proc, req) {
  let realm = null;
  let buf = '';
  const yieldFn = function () { return new Promise(function (r) { setImmediate(r); }); };
  function reply(id, ok, v) {
    proc.stdout.write(JSON.stringify(ok ? { id: id, ok: true, result: v } : { id: id, ok: false, error: String(v && v.stack || v) }) + '\n');
  }
  async function handle(m) {
    const ms = function (t) { return t[0] * 1e3 + t[1] / 1e6; };
    switch (m.cmd) {
      case 'init':
        realm = createRealm(vm, m);
        return { node: proc.version };
      case 'setData': {
        const t0 = proc.hrtime();
        const r = JSON.parse(realm.api.setData(m.json));
        r.contextBuildMs = ms(proc.hrtime(t0));
        return r;
      }
      case 'filter': {
        const t0 = proc.hrtime();
        realm.api.filter();
        return ms(proc.hrtime(t0));
      }
      case 'cycle':
        return cycle(realm.api, m, yieldFn);
      case 'calibrate': {
        const times = [];
        let elements = 0;
        for (let i = 0; i < m.reps; i++) {
          const t0 = proc.hrtime();
          elements = realm.api.calibrate(m.rows);
          times.push(ms(proc.hrtime(t0)));
        }
        return { times: times, elements: elements };
      }
      case 'audit':
        return audit(vm, realm.ctx, { process: proc, require: req, Function: Function, Object: Object });
      case 'probe':
        return probe(req('fs'), req('net'));
      default:
        throw new Error('unknown command ' + m.cmd);
    }
  }
  let chain = Promise.resolve();
  proc.stdin.setEncoding('utf8');
  proc.stdin.on('data', function (chunk) {
    buf += chunk;
    let nl;
    while ((nl = buf.indexOf('\n')) >= 0) {
      const line = buf.slice(0, nl);
      buf = buf.slice(nl + 1);
      if (!line.trim()) continue;
      const m = JSON.parse(line);
      chain = chain.then(function () { return handle(m); }).then(function (v) { reply(m.id, true, v); }, function (e) { reply(m.id, false, e); });
    }
  });
  proc.stdin.on('end', function () { chain.then(function () { proc.exit(0); }); });
}

module.exports = { audit: audit, createRealm: createRealm, cycle: cycle, globalNames: globalNames, serve: serve, wrap: wrap };
