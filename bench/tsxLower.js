/**
 * The lowering passes of bench/tsx.js: `a?.b` / `a?.[k]` / `a?.(x)` and
 * `a ?? b` → ES2019 (helpers that evaluate the left side once), and ES
 * modules → a function module (`__import(spec)` / `__exports`).
 */
import { KEYWORD_BEFORE_EXPR, isClose, isOpen, matching, sig, tokenize } from './tsxLex.js';

// ---------------------------------------------------------------------------
// ?. and ?? → ES2019
// ---------------------------------------------------------------------------

const NC_LEFT_STOPS = ['(', '[', '{', ',', ';', '=', ':', '?', '=>', '&&', '||', '??', '...', '!', '+=', '-='];
const NC_RIGHT_STOPS = [')', ']', '}', ',', ';', ':', '?', '??', '||', '&&'];

function text(toks, a, b) {
  return toks.slice(a, b).map(function (x) { return x.v; }).join('');
}

/**
 * Start of the member / call chain ending at token `k` (inclusive):
 * primary ( .name | ?.name | (…) | […] )*, walked right to left.
 */
function chainStart(toks, k) {
  let j = k;
  for (;;) {
    const t = toks[j];
    if (t.t === 'punct' && (t.v === ')' || t.v === ']')) {
      const o = openOf(toks, j);
      const p = sig(toks, o, -1);
      const pv = p >= 0 ? toks[p] : null;
      if (pv && pv.t === 'punct' && pv.v === '?.') { j = sig(toks, p, -1); continue; }
      // a call or an index continues to the callee / object; else the bracket is the primary
      if (pv && ((pv.t === 'ident' && !KEYWORD_BEFORE_EXPR[pv.v]) || (pv.t === 'punct' && (pv.v === ')' || pv.v === ']')))) {
        j = p;
        continue;
      }
      return o;
    }
    if (t.t === 'ident' || t.t === 'str' || t.t === 'num' || t.t === 'tmpl') {
      if (t.t === 'ident' && KEYWORD_BEFORE_EXPR[t.v]) throw new Error('tsx: keyword in chain ' + t.v);
      const p = sig(toks, j, -1);
      if (p >= 0 && toks[p].t === 'punct' && (toks[p].v === '.' || toks[p].v === '?.')) {
        j = sig(toks, p, -1);
        continue;
      }
      return j;
    }
    throw new Error('tsx: cannot chain from ' + t.v);
  }
}

function openOf(toks, close) {
  let d = 0;
  for (let j = close; j >= 0; j--) {
    if (isClose(toks[j])) d++;
    else if (isOpen(toks[j])) {
      d--;
      if (d === 0) return j;
    }
  }
  throw new Error('tsx: unbalanced ' + toks[close].v);
}

/** End (exclusive) of the member / call chain continuing at token `k`. */
function chainEnd(toks, k) {
  let j = k;
  for (;;) {
    const n = sig(toks, j - 1, 1);
    if (n >= toks.length) return j;
    const t = toks[n];
    if (t.t === 'punct' && (t.v === '.' || t.v === '?.')) {
      const m = sig(toks, n, 1);
      if (toks[m].t === 'ident') { j = m + 1; continue; }
      if (toks[m].v === '(' || toks[m].v === '[') { j = matching(toks, m) + 1; continue; }
      return j;
    }
    if (t.t === 'punct' && (t.v === '(' || t.v === '[')) { j = matching(toks, n) + 1; continue; }
    return j;
  }
}

/** Rewrite optional chains and nullish coalescing (innermost / leftmost first). */
export function lowerOptional(src) {
  for (let guard = 0; guard < 10000; guard++) {
    const toks = tokenize(src);
    // template literals: lower their expressions in place
    let changed = false;
    for (let k = 0; k < toks.length; k++) {
      if (toks[k].t !== 'tmpl') continue;
      const parts = toks[k].parts;
      let v = '`';
      for (let i = 0; i < parts.length; i++) v += i % 2 ? '${' + lowerOptional(parts[i]) + '}' : parts[i];
      v += '`';
      if (v !== toks[k].v) {
        toks[k] = { t: 'tmpl', v: v, parts: parts };
        changed = true;
      }
    }
    if (changed) src = text(toks, 0, toks.length);
    const T = tokenize(src);
    let at = -1;
    for (let k = 0; k < T.length; k++) {
      if (T[k].t === 'punct' && (T[k].v === '?.' || T[k].v === '??')) { at = k; break; }
    }
    if (at < 0) return src;
    if (T[at].v === '?.') {
      const lhsEnd = sig(T, at, -1);
      const lhsStart = chainStart(T, lhsEnd);
      const restStart = sig(T, at, 1);
      let restEnd;
      if (T[restStart].t === 'ident') restEnd = chainEnd(T, restStart + 1);
      else if (T[restStart].v === '(' || T[restStart].v === '[') restEnd = chainEnd(T, matching(T, restStart) + 1);
      else throw new Error('tsx: bad optional chain');
      const rest = text(T, restStart, restEnd);
      const body = T[restStart].t === 'ident' ? '__o.' + rest : '__o' + rest;
      src = text(T, 0, lhsStart) + '__oc(' + text(T, lhsStart, lhsEnd + 1) + ', function (__o) { return ' + body + '; })' +
        text(T, restEnd, T.length);
    } else {
      // left operand: back to a lower-precedence token at depth 0
      let a = at - 1;
      for (; a >= 0; a--) {
        const t = T[a];
        if (isClose(t)) { a = openOf(T, a); continue; }
        if (isOpen(t)) break;
        if (t.t === 'punct' && NC_LEFT_STOPS.indexOf(t.v) >= 0) break;
        if (t.t === 'ident' && (t.v === 'return' || t.v === 'case' || t.v === 'throw')) break;
      }
      let b = at + 1;
      for (; b < T.length; b++) {
        const t = T[b];
        if (isOpen(t)) { b = matching(T, b); continue; }
        if (isClose(t)) break;
        if (t.t === 'punct' && NC_RIGHT_STOPS.indexOf(t.v) >= 0) break;
      }
      const left = text(T, a + 1, at).trim();
      const right = text(T, at + 1, b).trim();
      src = text(T, 0, a + 1) + ' __nc(' + left + ', function () { return ' + right + '; })' + text(T, b, T.length);
    }
  }
  throw new Error('tsx: optional lowering did not converge');
}

// ---------------------------------------------------------------------------
// ES module → function module
// ---------------------------------------------------------------------------

export const HELPERS = 'function __oc(o, f) { return o === null || o === undefined ? undefined : f(o); }\n' +
  'function __nc(v, f) { return v === null || v === undefined ? f() : v; }\n';

/** `import` / `export` statements → `__import(spec)` / `__exports`. */
export function lowerModules(src) {
  const exportsTail = [];
  let s = src.replace(/^[ \t]*import\s+([\s\S]*?)\s+from\s+'([^']+)';?/gm, function (m, clause, spec) {
    const out = [];
    let c = clause.trim();
    const def = /^([A-Za-z_$][\w$]*)\s*(?:,\s*([\s\S]*))?$/.exec(c);
    if (def) {
      out.push('const ' + def[1] + ' = __import(' + JSON.stringify(spec) + ', true);');
      c = (def[2] || '').trim();
    }
    if (c) {
      if (c[0] !== '{') throw new Error('tsx: unsupported import ' + m);
      const names = c.slice(1, -1).split(',').map(function (x) { return x.trim(); }).filter(Boolean).map(function (x) {
        const a = /^(?:type\s+)?([A-Za-z_$][\w$]*)(?:\s+as\s+([A-Za-z_$][\w$]*))?$/.exec(x);
        if (!a) throw new Error('tsx: unsupported import name ' + x);
        return a[2] ? a[1] + ': ' + a[2] : a[1];
      });
      out.push('const { ' + names.join(', ') + ' } = __import(' + JSON.stringify(spec) + ');');
    }
    return out.join(' ');
  });
  s = s.replace(/^[ \t]*import\s+'([^']+)';?/gm, function (m, spec) { return '__import(' + JSON.stringify(spec) + ');'; });
  s = s.replace(/^[ \t]*export\s+default\s+function\s+([A-Za-z_$][\w$]*)/gm, function (m, name) {
    exportsTail.push('__exports.default = ' + name + ';');
    return 'function ' + name;
  });
  s = s.replace(/^[ \t]*export\s+(async\s+)?function\s+([A-Za-z_$][\w$]*)/gm, function (m, as, name) {
    exportsTail.push('__exports.' + name + ' = ' + name + ';');
    return (as || '') + 'function ' + name;
  });
  s = s.replace(/^[ \t]*export\s+(const|let|var)\s+([A-Za-z_$][\w$]*)/gm, function (m, kw, name) {
    exportsTail.push('__exports.' + name + ' = ' + name + ';');
    return kw + ' ' + name;
  });
  s = s.replace(/^[ \t]*export\s+default\s+/gm, '__exports.default = ');
  const left = /^[ \t]*(import|export)\b.*$/m.exec(s);
  if (left) throw new Error('tsx: unsupported module statement: ' + left[0]);
  return s + '\n' + exportsTail.join('\n') + '\n';
}
