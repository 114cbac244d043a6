#!/usr/bin/env node
/**
 * Offline stand-in for the part of ESLint's `no-unused-vars` that catches
 * real drift in this code base (ESLint itself needs the npm registry; CI runs
 * it, `.eslintrc.cjs`). Token-level (bench/tsxLex.js), per file:
 *
 *   * an imported binding that the file never uses;
 *   * a top-level `function` / `const` / `let` that is neither exported nor
 *     used anywhere else in its file;
 *   * a file longer than MAX_LINES (the module-size budget, VERDICT r3).
 *
 *   node tools/lint_js.js DIR_OR_FILE...    → one line per finding, exit 1 if any
 */
import fs from 'fs';
import path from 'path';
import { tokenize } from '../bench/tsxLex.js';

export const MAX_LINES = 700;

function walk(p, out) {
  if (fs.statSync(p).isDirectory()) {
    fs.readdirSync(p).sort().forEach(function (f) {
      if (f !== 'node_modules' && f[0] !== '.') walk(path.join(p, f), out);
    });
  } else if (/\.js$/.test(p) && !/\.min\.js$/.test(p)) {
    out.push(p);
  }
  return out;
}

/** Every identifier token of `src`, template-literal expressions included. */
function identifiers(src) {
  const used = {};
  (function scan(s) {
    // Significant tokens (no whitespace / comments), to look one back and one ahead.
    const ts = tokenize(s).filter(function (t) { return t.t !== 'ws' && t.t !== 'comment'; });
    for (let i = 0; i < ts.length; i++) {
      const t = ts[i];
      if (t.t === 'tmpl') {
        t.parts.forEach(function (p, k) { if (k % 2) scan(p); });
        continue;
      }
      if (t.t !== 'ident') continue;
      const prev = ts[i - 1];
      const next = ts[i + 1];
      // `x.get(…)` and `{ get: … }` name a property, not an imported `get`.
      if (prev && prev.v === '.') continue;
      if (prev && (prev.v === '{' || prev.v === ',') && next && next.v === ':') continue;
      used[t.v] = (used[t.v] || 0) + 1;
    }
  })(src);
  return used;
}

/** Bindings of one import clause (`A`, `{ b, c as d }`, `* as ns`, `A, { b }`). */
function importBindings(clause) {
  let c = clause.trim();
  const out = [];
  const ns = /^(?:([A-Za-z_$][\w$]*)\s*,\s*)?\*\s+as\s+([A-Za-z_$][\w$]*)$/.exec(c);
  if (ns) return ns[1] ? [ns[1], ns[2]] : [ns[2]];
  const def = /^([A-Za-z_$][\w$]*)\s*(?:,\s*([\s\S]*))?$/.exec(c);
  if (def) {
    out.push(def[1]);
    c = (def[2] || '').trim();
  }
  if (c[0] === '{') {
    c.slice(1, -1).split(',').map(function (x) { return x.trim(); }).filter(Boolean).forEach(function (x) {
      out.push(/([A-Za-z_$][\w$]*)\s*$/.exec(x)[1]);
    });
  }
  return out;
}

/** Findings for one file's source. */
export function lintSource(file, src) {
  const findings = [];
  const lines = src.split('\n').length - (src.endsWith('\n') ? 1 : 0);
  if (lines > MAX_LINES) findings.push(file + ': ' + lines + ' lines (budget ' + MAX_LINES + ')');
  const imports = [];
  const body = src.replace(/^import\s+([\s\S]*?)\s+from\s+'[^']+';?/gm, function (m, clause) {
    importBindings(clause).forEach(function (b) { imports.push(b); });
    return '';
  });
  let used;
  try {
    used = identifiers(body);
  } catch (e) {
    return findings.concat([file + ': cannot tokenize (' + e.message + ')']);
  }
  imports.forEach(function (b) {
    if (!used[b]) findings.push(file + ': import ' + b + ' is never used');
  });
  const exported = {};
  body.replace(/^export\s*\{([^}]*)\}/gm, function (m, names) {
    names.split(',').forEach(function (x) { const a = /^\s*([A-Za-z_$][\w$]*)/.exec(x); if (a) exported[a[1]] = true; });
    return m;
  });
  const decl = /^(export\s+)?(?:async\s+)?(?:function\s*\*?|const|let)\s+([A-Za-z_$][\w$]*)/gm;
  let m;
  while ((m = decl.exec(body))) {
    if (m[1] || exported[m[2]]) continue;
    if ((used[m[2]] || 0) < 2) findings.push(file + ': ' + m[2] + ' is declared but never used');
  }
  return findings;
}

function main() {
  const files = [];
  process.argv.slice(2).forEach(function (p) { walk(p, files); });
  let all = [];
  files.forEach(function (f) { all = all.concat(lintSource(f, fs.readFileSync(f, 'utf8'))); });
  all.forEach(function (x) { process.stdout.write(x + '\n'); });
  process.stdout.write('[lint_js] ' + files.length + ' files, ' + all.length + ' findings\n');
  process.exit(all.length ? 1 : 0);
}

if (process.argv[1] && path.resolve(process.argv[1]) === path.resolve(new URL(import.meta.url).pathname)) main();
