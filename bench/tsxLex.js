/**
 * The lexer of bench/tsx.js (the benchmark's TSX → JavaScript transformer):
 * tokens with their kinds, the scanners for strings, templates and regular
 * expressions, and the token-walking helpers the type erasure and the
 * optional-chain lowering share.
 */

export const PUNCT3 = ['...', '===', '!==', '**=', '<<=', '>>=', '>>>', '&&=', '||=', '??='];
export const PUNCT2 = ['=>', '==', '!=', '<=', '>=', '&&', '||', '??', '?.', '++', '--', '+=', '-=', '*=', '/=', '%=', '&=',
  '|=', '^=', '<<', '>>', '**'];
export const KEYWORD_BEFORE_EXPR = { return: 1, case: 1, typeof: 1, void: 1, delete: 1, throw: 1, in: 1, of: 1, new: 1, else: 1,
  do: 1, instanceof: 1, yield: 1, await: 1, default: 1 };

export function isIdStart(c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c === '_' || c === '$';
}
export function isIdPart(c) {
  return isIdStart(c) || (c >= '0' && c <= '9');
}

/** True when the token `prev` (or the start) leaves the scanner in expression position. */
export function exprPosition(prev) {
  if (!prev) return true;
  if (prev.t === 'ident') return !!KEYWORD_BEFORE_EXPR[prev.v];
  if (prev.t === 'punct') return [')', ']', '}', '++', '--'].indexOf(prev.v) < 0;
  return false;
}

/**
 * Tokens of `src`: {t, v} with t in ws | comment | ident | num | str | tmpl |
 * regex | punct. A template literal is one token; `parts` alternates quasi
 * text and expression source.
 */
export function tokenize(src) {
  const out = [];
  let i = 0;
  let prev = null;
  const n = src.length;
  function push(t, v, extra) {
    const tok = Object.assign({ t: t, v: v }, extra || {});
    out.push(tok);
    if (t !== 'ws' && t !== 'comment') prev = tok;
  }
  while (i < n) {
    const c = src[i];
    if (c === ' ' || c === '\t' || c === '\n' || c === '\r') {
      let j = i;
      while (j < n && /\s/.test(src[j])) j++;
      push('ws', src.slice(i, j));
      i = j;
    } else if (c === '/' && src[i + 1] === '/') {
      let j = src.indexOf('\n', i);
      if (j < 0) j = n;
      push('comment', src.slice(i, j));
      i = j;
    } else if (c === '/' && src[i + 1] === '*') {
      const j = src.indexOf('*/', i + 2);
      if (j < 0) throw new Error('tsx: unterminated comment');
      push('comment', src.slice(i, j + 2));
      i = j + 2;
    } else if (c === '"' || c === "'") {
      const j = skipString(src, i);
      push('str', src.slice(i, j));
      i = j;
    } else if (c === '`') {
      const r = scanTemplate(src, i);
      push('tmpl', src.slice(i, r.end), { parts: r.parts });
      i = r.end;
    } else if (isIdStart(c)) {
      let j = i;
      while (j < n && isIdPart(src[j])) j++;
      push('ident', src.slice(i, j));
      i = j;
    } else if (c >= '0' && c <= '9') {
      let j = i;
      while (j < n && /[0-9a-fA-FxXoObB._n]/.test(src[j])) j++;
      push('num', src.slice(i, j));
      i = j;
    } else if (c === '/' && exprPosition(prev)) {
      const j = scanRegex(src, i);
      push('regex', src.slice(i, j));
      i = j;
    } else {
      let p = null;
      const three = src.substr(i, 3);
      const two = src.substr(i, 2);
      if (PUNCT3.indexOf(three) >= 0) p = three;
      else if (PUNCT2.indexOf(two) >= 0 && !(two === '?.' && /[0-9]/.test(src[i + 2] || ''))) p = two;
      else p = c;
      push('punct', p);
      i += p.length;
    }
  }
  return out;
}

/** End of the regex literal at `i` (flags included). */
export function scanRegex(src, i) {
  let j = i + 1;
  let cls = false;
  while (j < src.length) {
    if (src[j] === '\\') { j += 2; continue; }
    if (src[j] === '[') cls = true;
    else if (src[j] === ']') cls = false;
    else if (src[j] === '/' && !cls) break;
    else if (src[j] === '\n') throw new Error('tsx: unterminated regex');
    j++;
  }
  j++;
  while (j < src.length && isIdPart(src[j])) j++;
  return j;
}

export function skipString(src, i) {
  const q = src[i];
  let j = i + 1;
  while (j < src.length && src[j] !== q) {
    if (src[j] === '\\') j++;
    else if (src[j] === '\n') throw new Error('tsx: unterminated string');
    j++;
  }
  return j + 1;
}

/** A template literal at `i`: {end, parts: [quasi, expr, quasi, ...]} (raw source). */
export function scanTemplate(src, i) {
  const parts = [];
  let j = i + 1;
  let q = j;
  while (j < src.length) {
    if (src[j] === '\\') { j += 2; continue; }
    if (src[j] === '`') {
      parts.push(src.slice(q, j));
      return { end: j + 1, parts: parts };
    }
    if (src[j] === '$' && src[j + 1] === '{') {
      parts.push(src.slice(q, j));
      const e = matchBrace(src, j + 1);
      parts.push(src.slice(j + 2, e));
      j = e + 1;
      q = j;
      continue;
    }
    j++;
  }
  throw new Error('tsx: unterminated template');
}

/** Index of the `}` closing the `{` at `open` (strings, templates and comments skipped). */
export function matchBrace(src, open) {
  let depth = 0;
  let j = open;
  while (j < src.length) {
    const c = src[j];
    if (c === '"' || c === "'") { j = skipString(src, j); continue; }
    if (c === '`') { j = scanTemplate(src, j).end; continue; }
    if (c === '/' && src[j + 1] === '/') { j = src.indexOf('\n', j); if (j < 0) break; continue; }
    if (c === '/' && src[j + 1] === '*') { j = src.indexOf('*/', j) + 2; continue; }
    if (c === '{') depth++;
    else if (c === '}') {
      depth--;
      if (depth === 0) return j;
    }
    j++;
  }
  throw new Error('tsx: unbalanced {');
}

// ---------------------------------------------------------------------------
// TypeScript erasure (token level)
// ---------------------------------------------------------------------------

export function sig(toks, k, dir) {
  let j = k + dir;
  while (j >= 0 && j < toks.length && (toks[j].t === 'ws' || toks[j].t === 'comment')) j += dir;
  return j;
}

export function isOpen(t) { return t.t === 'punct' && (t.v === '(' || t.v === '[' || t.v === '{'); }
export function isClose(t) { return t.t === 'punct' && (t.v === ')' || t.v === ']' || t.v === '}'); }

/** Index of the token closing the bracket at `k`. */
export function matching(toks, k) {
  let d = 0;
  for (let j = k; j < toks.length; j++) {
    if (isOpen(toks[j])) d++;
    else if (isClose(toks[j])) {
      d--;
      if (d === 0) return j;
    }
  }
  throw new Error('tsx: unbalanced ' + toks[k].v);
}

/** Index of the `>` closing a type-argument `<` at `k`, or -1 when it is no type argument list. */
export function typeArgsEnd(toks, k) {
  let d = 0;
  for (let j = k; j < toks.length; j++) {
    const t = toks[j];
    if (t.t === 'ws' || t.t === 'comment' || t.t === 'ident' || t.t === 'str' || t.t === 'num') continue;
    if (t.t !== 'punct') return -1;
    if (t.v === '<') d++;
    else if (t.v === '>') {
      d--;
      if (d === 0) return j;
    } else if (t.v === '>>') {
      d -= 2;
      if (d <= 0) return d === 0 ? j : -1;
    } else if (['|', '&', ',', '[', ']', '.', '{', '}', ':', ';', '?', '(', ')', '=>'].indexOf(t.v) < 0) return -1;
  }
  return -1;
}

/**
 * End (exclusive) of a type starting at token `k`: the first token at depth 0
 * that is in `stops` (brackets and `<…>` nest).
 */
export function typeEnd(toks, k, stops) {
  let d = 0;
  let angle = 0;
  for (let j = k; j < toks.length; j++) {
    const t = toks[j];
    if (t.t !== 'punct') continue;
    if (d === 0 && angle === 0 && j > k && stops.indexOf(t.v) >= 0) return j;
    if (isOpen(t)) d++;
    else if (isClose(t)) {
      if (d === 0) return j;
      d--;
    } else if (t.v === '<') angle++;
    else if (t.v === '>' && angle > 0) angle--;
    else if (t.v === '=>' && d === 0 && angle === 0 && stops.indexOf('=>') >= 0 && j > k) return j;
  }
  return toks.length;
}

export function blank(toks, a, b) {
  for (let j = a; j < b; j++) toks[j] = { t: 'ws', v: toks[j].t === 'ws' && /\n/.test(toks[j].v) ? '\n' : '' };
}
