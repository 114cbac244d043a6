#!/usr/bin/env node
/**
 * Offline plugin bundler: src/index.tsx and everything it imports → one
 * self-contained script (default `dist-offline/main.js`; `headlamp-plugin build`
 * writes `dist/main.js`), the file Headlamp loads for a plugin.
 *
 *   node tools/bundle.js [--entry src/index.tsx] [--out dist-offline/main.js] [--package] [--stamp]
 *   node tools/bundle.js --digest      # print the archive's sha256 for this tree, write nothing
 *   node tools/bundle.js --check       # exit 1 unless artifacthub-pkg.yml carries that digest
 *
 * The reference builds its bundle with `headlamp-plugin build` (vite;
 * /root/reference/package.json:16-18, CI /root/reference/.github/workflows/ci.yaml:169-170).
 * That CLI is an npm package and this build environment has no registry, so
 * this file does the part of that job the plugin needs, with no dependency:
 *
 *   * module graph from the entry, relative specifiers resolved like
 *     tools/plugin-loader.js (./x → x.tsx | x.ts | x.js | x/index.*);
 *   * TypeScript: the .ts/.tsx shims are written in the JavaScript subset of
 *     TypeScript (types live in .d.ts files), so the only TypeScript syntax
 *     is `import type`, which is dropped;
 *   * ES modules → functions in a module table (import bindings resolved
 *     through getters, so exports are live), executed once, in import order;
 *   * host modules are not bundled: they resolve to the globals Headlamp
 *     hands every plugin (`pluginLib`) — the externals `headlamp-plugin
 *     build` declares for the same imports (EXTERNALS below).
 *
 * Anything else (an `import`/`export` form this does not understand, a bare
 * specifier that is not a host module) is an error, not a silent pass-through.
 *
 * This bundle is the shipped artifact: `--package` wraps it into the archive
 * the release uploads (.github/workflows/release.yaml), `--stamp` writes that
 * archive's version, URL and sha256 into artifacthub-pkg.yml (the reference
 * commits the real digest, /root/reference/artifacthub-pkg.yml:101-105), and
 * tools/verify_archive.js evaluates the archive's own main.js and checks
 * every registration. The archive is a function of the tree alone (fixed
 * tar headers, tools/deflate.js instead of zlib), so the CPU gate re-derives
 * the committed digest. CI still runs `npm run build` (headlamp-plugin's
 * vite build) as a check that the real toolchain compiles the sources.
 */
import crypto from 'crypto';
import fs from 'fs';
import path from 'path';
import { fileURLToPath } from 'url';
import { gzipStable } from './deflate.js';

const ROOT = path.resolve(path.dirname(fileURLToPath(import.meta.url)), '..');

/** Host modules → expression over the `pluginLib` object Headlamp provides. */
export const EXTERNALS = {
  '@kinvolk/headlamp-plugin/lib': 'pluginLib',
  '@kinvolk/headlamp-plugin/lib/CommonComponents': 'pluginLib.CommonComponents',
  react: 'pluginLib.React',
};

const TRY = ['', '.tsx', '.ts', '.js', '/index.tsx', '/index.ts', '/index.js'];
const IDENT = /^[A-Za-z_$][\w$]*$/;

function resolveFile(fromFile, spec) {
  const base = path.resolve(path.dirname(fromFile), spec);
  for (let i = 0; i < TRY.length; i++) {
    const f = base + TRY[i];
    if (fs.existsSync(f) && fs.statSync(f).isFile()) return f;
  }
  throw new Error('bundle: cannot resolve ' + JSON.stringify(spec) + ' from ' + path.relative(ROOT, fromFile));
}

/** `a, b as c` → [[local, exported]] (import: [imported, local]). */
function specList(body, where) {
  return body
    .split(',')
    .map(function (s) { return s.trim(); })
    .filter(function (s) { return s.length > 0; })
    .map(function (s) {
      const m = /^([A-Za-z_$][\w$]*)(?:\s+as\s+([A-Za-z_$][\w$]*))?$/.exec(s);
      if (!m) throw new Error('bundle: unsupported specifier ' + JSON.stringify(s) + ' in ' + where);
      return [m[1], m[2] || m[1]];
    });
}

/** Names bound by `{ a, b: c, ...rest }` / `[a, b]` / `name`. */
function boundNames(target, where) {
  const t = target.trim();
  if (IDENT.test(t)) return [t];
  const inner = t.slice(1, -1);
  return inner
    .split(',')
    .map(function (s) { return s.trim(); })
    .filter(function (s) { return s.length > 0; })
    .map(function (s) {
      const rest = /^\.\.\.([A-Za-z_$][\w$]*)$/.exec(s);
      if (rest) return rest[1];
      const m = /^(?:[A-Za-z_$][\w$]*\s*:\s*)?([A-Za-z_$][\w$]*)(?:\s*=.*)?$/.exec(s);
      if (!m) throw new Error('bundle: unsupported destructuring ' + JSON.stringify(s) + ' in ' + where);
      return m[1];
    });
}

/**
 * One module's source → { code, deps } where code is the body of
 * `function (__exports, __req) { … }`.
 */
export function transformModule(source, file, resolveDep) {
  const where = path.relative(ROOT, file);
  const getters = []; // [exported, expression]
  const deps = [];
  let nextTmp = 0;
  function req(spec) {
    if (Object.prototype.hasOwnProperty.call(EXTERNALS, spec)) return '__ext(' + JSON.stringify(spec) + ')';
    if (!(spec.startsWith('./') || spec.startsWith('../'))) {
      throw new Error('bundle: bare import ' + JSON.stringify(spec) + ' in ' + where + ' is not a host module');
    }
    const id = resolveDep(file, spec);
    deps.push(id);
    return '__req(' + JSON.stringify(id) + ')';
  }
  let s = String(source).replace(/^import type [^;]*;[ \t]*$/gm, '');
  s = s.replace(/^import\s+([\s\S]*?)\s+from\s+'([^']+)';?/gm, function (m, clause, spec) {
    const src = req(spec);
    const out = [];
    let c = clause.trim();
    const ns = /^\*\s+as\s+([A-Za-z_$][\w$]*)$/.exec(c);
    if (ns) return 'const ' + ns[1] + ' = ' + src + ';';
    let def = null;
    const d = /^([A-Za-z_$][\w$]*)\s*(?:,\s*([\s\S]*))?$/.exec(c);
    if (d) {
      def = d[1];
      c = (d[2] || '').trim();
    }
    const tmp = '__m' + nextTmp++;
    out.push('const ' + tmp + ' = ' + src + ';');
    if (def) out.push('const ' + def + ' = __default(' + tmp + ');');
    if (c) {
      if (c[0] !== '{' || c[c.length - 1] !== '}') throw new Error('bundle: unsupported import ' + JSON.stringify(m) + ' in ' + where);
      specList(c.slice(1, -1), where).forEach(function (p) {
        out.push('const ' + p[1] + ' = ' + tmp + '.' + p[0] + ';');
        out.push('if (!(' + JSON.stringify(p[0]) + ' in ' + tmp + ')) __missing(' + JSON.stringify(p[0]) + ', ' + JSON.stringify(spec) + ', ' + JSON.stringify(where) + ');');
      });
    }
    return out.join(' ');
  });
  s = s.replace(/^import\s+'([^']+)';?/gm, function (m, spec) { return req(spec) + ';'; });
  s = s.replace(/^export\s+\{([^}]*)\}\s+from\s+'([^']+)';?/gm, function (m, body, spec) {
    const tmp = '__re' + getters.length;
    specList(body, where).forEach(function (p) { getters.push([p[1], tmp + '.' + p[0]]); });
    return 'const ' + tmp + ' = ' + req(spec) + ';';
  });
  s = s.replace(/^export\s+\{([^}]*)\};?/gm, function (m, body) {
    specList(body, where).forEach(function (p) { getters.push([p[1], p[0]]); });
    return '';
  });
  s = s.replace(/^export\s+default\s+/gm, '__exports.default = ');
  s = s.replace(/^export\s+(const|let|var)\s+(\{[^}]*\}|\[[^\]]*\]|[A-Za-z_$][\w$]*)/gm, function (m, kw, target) {
    boundNames(target, where).forEach(function (n) { getters.push([n, n]); });
    return kw + ' ' + target;
  });
  s = s.replace(/^export\s+((?:async\s+)?function\*?|class)\s+([A-Za-z_$][\w$]*)/gm, function (m, kw, name) {
    getters.push([name, name]);
    return kw + ' ' + name;
  });
  const left = /^(import|export)\b.*$/m.exec(s);
  if (left) throw new Error('bundle: unsupported statement in ' + where + ': ' + left[0]);
  if (/\bimport\s*\(|\bimport\.meta\b/.test(s)) throw new Error('bundle: dynamic import / import.meta in ' + where);
  const head = getters
    .map(function (g) { return '__export(__exports, ' + JSON.stringify(g[0]) + ', function () { return ' + g[1] + '; });'; })
    .join('\n');
  return { code: "'use strict';\n" + head + '\n' + s, deps: deps };
}

/**
 * Bundle the graph rooted at `entry` (absolute path) → script text.
 * @returns {{code: string, modules: string[]}}
 */
export function bundle(entry) {
  const order = [];
  const mods = {};
  function id(file) { return path.relative(ROOT, file).split(path.sep).join('/'); }
  function resolveDep(fromFile, spec) { return id(resolveFile(fromFile, spec)); }
  function visit(file) {
    const key = id(file);
    if (mods[key]) return;
    mods[key] = transformModule(fs.readFileSync(file, 'utf8'), file, resolveDep);
    mods[key].deps.forEach(function (d) { visit(path.join(ROOT, d)); });
    order.push(key);
  }
  visit(entry);
  const pkg = JSON.parse(fs.readFileSync(path.join(ROOT, 'package.json'), 'utf8'));
  const parts = [];
  parts.push('/* ' + pkg.name + ' ' + pkg.version + ' — Headlamp plugin bundle built by tools/bundle.js from ' + id(entry) + ' (' + order.length + ' modules). */');
  parts.push('(function (pluginLib) {');
  parts.push("  'use strict';");
  parts.push('  if (!pluginLib) throw new Error(' + JSON.stringify(pkg.name + ': Headlamp plugin library (pluginLib) not found') + ');');
  parts.push('  var __defs = Object.create(null);');
  parts.push('  var __cache = Object.create(null);');
  parts.push('  var __externals = {');
  Object.keys(EXTERNALS).forEach(function (k) {
    parts.push('    ' + JSON.stringify(k) + ': function () { return ' + EXTERNALS[k] + '; },');
  });
  parts.push('  };');
  parts.push('  function __export(o, k, get) { Object.defineProperty(o, k, { enumerable: true, get: get }); }');
  parts.push('  function __default(m) { return m && m.__esModule !== true && m.default !== undefined ? m.default : m; }');
  parts.push('  function __missing(name, spec, from) { throw new Error("bundle: \'" + name + "\' is not exported by " + spec + " (imported by " + from + ")"); }');
  parts.push('  function __ext(spec) { var v = __externals[spec](); if (v === undefined || v === null) throw new Error("host module " + spec + " missing from pluginLib"); return v; }');
  parts.push('  function __req(id) {');
  parts.push('    var m = __cache[id];');
  parts.push('    if (m) return m;');
  parts.push('    m = __cache[id] = {};');
  parts.push('    __defs[id](m, __req, __ext);');
  parts.push('    return m;');
  parts.push('  }');
  order.forEach(function (key) {
    parts.push('  // ---- ' + key);
    parts.push('  __defs[' + JSON.stringify(key) + '] = function (__exports, __req, __ext) {');
    parts.push(mods[key].code);
    parts.push('  };');
  });
  parts.push('  return __req(' + JSON.stringify(id(entry)) + ');');
  parts.push("})(typeof pluginLib !== 'undefined' ? pluginLib : (typeof globalThis !== 'undefined' ? globalThis.pluginLib : undefined));");
  return { code: parts.join('\n') + '\n', modules: order };
}

/** One ustar header + body (padded to 512-byte blocks). */
function tarEntry(name, body, mtime) {
  const h = Buffer.alloc(512, 0);
  function put(off, len, str) { h.write(str, off, len, 'ascii'); }
  function oct(off, len, n) { put(off, len, n.toString(8).padStart(len - 1, '0') + '\0'); }
  if (Buffer.byteLength(name) > 100) throw new Error('bundle: tar name too long: ' + name);
  put(0, 100, name);
  oct(100, 8, 0o644);
  oct(108, 8, 0);
  oct(116, 8, 0);
  oct(124, 12, body.length);
  oct(136, 12, mtime);
  put(148, 8, '        '); // checksum placeholder (spaces) while summing
  put(156, 1, '0');
  put(257, 6, 'ustar\0');
  put(263, 2, '00');
  let sum = 0;
  for (let i = 0; i < 512; i++) sum += h[i];
  put(148, 8, sum.toString(8).padStart(6, '0') + '\0 ');
  const pad = Buffer.alloc((512 - (body.length % 512)) % 512, 0);
  return Buffer.concat([h, body, pad]);
}

/**
 * The installable plugin archive: `<name>/main.js` + `<name>/package.json`,
 * the layout Headlamp loads from its plugins directory and `headlamp-plugin
 * package` produces; gzip-compressed by tools/deflate.js with fixed tar
 * headers (mtime 0), so the bytes depend on the bundle and package.json only.
 * Returns {name, bytes, sha256}.
 */
export function archiveOf(code) {
  const pkg = JSON.parse(fs.readFileSync(path.join(ROOT, 'package.json'), 'utf8'));
  const meta = { name: pkg.name, version: pkg.version, description: pkg.description, license: pkg.license, main: 'main.js' };
  const mtime = 0;
  const tar = Buffer.concat([
    tarEntry(pkg.name + '/main.js', Buffer.from(code, 'utf8'), mtime),
    tarEntry(pkg.name + '/package.json', Buffer.from(JSON.stringify(meta, null, 2) + '\n', 'utf8'), mtime),
    Buffer.alloc(1024, 0),
  ]);
  const gz = gzipStable(tar);
  return { name: pkg.name + '-' + pkg.version + '.tar.gz', version: pkg.version, bytes: gz, sha256: crypto.createHash('sha256').update(gz).digest('hex') };
}

/** Write archiveOf(code) into outDir → {file, sha256} (the checksum artifacthub-pkg.yml's archive-checksum takes). */
export function packageArchive(code, outDir) {
  const a = archiveOf(code);
  const file = path.join(outDir, a.name);
  fs.mkdirSync(outDir, { recursive: true });
  fs.writeFileSync(file, a.bytes);
  return { file: file, sha256: a.sha256 };
}

/** The archive this tree ships: src/index.tsx bundled and packaged, in memory. */
export function treeArchive() {
  return archiveOf(bundle(path.join(ROOT, 'src', 'index.tsx')).code);
}

const PKG_YML = path.join(ROOT, 'artifacthub-pkg.yml');
const CHECKSUM_RE = /^(\s*headlamp\/plugin\/archive-checksum:\s*)"sha256:[0-9a-f]{64}"\s*$/m;
const URL_RE = /^(\s*headlamp\/plugin\/archive-url:\s*")([^"]*\/)v\d+\.\d+\.\d+\/([^"/]*?)-\d+\.\d+\.\d+\.tar\.gz"\s*$/m;

/** artifacthub-pkg.yml text with version, archive URL and checksum set to archive `a`. */
export function stampText(text, a) {
  if (!CHECKSUM_RE.test(text)) throw new Error('bundle: no archive-checksum "sha256:<64 hex>" line in artifacthub-pkg.yml');
  if (!URL_RE.test(text)) throw new Error('bundle: no archive-url ".../vX.Y.Z/<name>-X.Y.Z.tar.gz" line in artifacthub-pkg.yml');
  if (!/^version: "[^"]*"\s*$/m.test(text)) throw new Error('bundle: no top-level version: "X.Y.Z" line in artifacthub-pkg.yml');
  return text
    .replace(/^version: "[^"]*"/m, 'version: "' + a.version + '"')
    .replace(URL_RE, function (m, pre, base) { return pre + base + 'v' + a.version + '/' + a.name + '"'; })
    .replace(CHECKSUM_RE, function (m, pre) { return pre + '"sha256:' + a.sha256 + '"'; });
}

/** The archive-checksum artifacthub-pkg.yml carries (hex), or null. */
export function committedDigest(text) {
  const m = /headlamp\/plugin\/archive-checksum:\s*"sha256:([0-9a-f]{64})"/.exec(text);
  return m ? m[1] : null;
}

function main(argv) {
  let entry = path.join(ROOT, 'src', 'index.tsx');
  let out = path.join(ROOT, 'dist-offline', 'main.js');
  let pack = false;
  let stamp = false;
  let mode = 'build';
  for (let i = 0; i < argv.length; i++) {
    if (argv[i] === '--entry') entry = path.resolve(argv[++i]);
    else if (argv[i] === '--out') out = path.resolve(argv[++i]);
    else if (argv[i] === '--package') pack = true;
    else if (argv[i] === '--stamp') pack = stamp = true;
    else if (argv[i] === '--digest') mode = 'digest';
    else if (argv[i] === '--check') mode = 'check';
    else {
      process.stderr.write('usage: node tools/bundle.js [--entry src/index.tsx] [--out dist-offline/main.js] [--package] [--stamp] | --digest | --check\n');
      return 2;
    }
  }
  if (mode !== 'build') {
    const a = treeArchive();
    if (mode === 'digest') {
      process.stdout.write('sha256:' + a.sha256 + '\n');
      return 0;
    }
    const text = fs.readFileSync(PKG_YML, 'utf8');
    if (stampText(text, a) !== text) {
      process.stderr.write('artifacthub-pkg.yml does not describe this tree\'s archive ' + a.name + ' (sha256:' + a.sha256 +
        ', committed ' + committedDigest(text) + '); run: node tools/bundle.js --package --stamp\n');
      return 1;
    }
    process.stdout.write('artifacthub-pkg.yml matches ' + a.name + ' sha256:' + a.sha256 + '\n');
    return 0;
  }
  const b = bundle(entry);
  fs.mkdirSync(path.dirname(out), { recursive: true });
  const tmp = out + '.tmp' + process.pid;
  fs.writeFileSync(tmp, b.code);
  fs.renameSync(tmp, out);
  process.stdout.write(path.relative(process.cwd(), out) + ': ' + b.modules.length + ' modules, ' + b.code.length + ' bytes\n');
  if (pack) {
    const a = packageArchive(b.code, path.dirname(out));
    process.stdout.write(path.relative(process.cwd(), a.file) + ': sha256:' + a.sha256 + '\n');
    if (stamp) {
      if (entry !== path.join(ROOT, 'src', 'index.tsx')) throw new Error('bundle: --stamp describes the shipped entry, src/index.tsx');
      fs.writeFileSync(PKG_YML, stampText(fs.readFileSync(PKG_YML, 'utf8'), archiveOf(b.code)));
      process.stdout.write('artifacthub-pkg.yml: stamped sha256:' + a.sha256 + '\n');
    }
  }
  return 0;
}

if (process.argv[1] && path.resolve(process.argv[1]) === fileURLToPath(import.meta.url)) {
  process.exitCode = main(process.argv.slice(2));
}
