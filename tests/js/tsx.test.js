/**
 * bench/tsx.js — the benchmark's TSX → JavaScript transformer (the opt-in
 * render comparison mounts the reference's own pages with it,
 * bench/referenceRender.js). Its transforms on small inputs of this
 * repository's own (the realm the reference's modules run in is checked by
 * tests/test_render_compare.py). Nothing here
 * reads or runs the reference's sources: they are untrusted public content
 * (ADR 014), executed only by tools/render_compare.py --allow-reference-exec.
 */
import { lowerModules, lowerOptional, stripTypes, transformJsx, transpile } from '../../bench/tsx.js';

/** Transpile one module and run it here, its imports answered from `imports` (this repository's fixtures only). */
function run(src, imports) {
  const exp = {};
  // eslint-disable-next-line no-new-func
  new Function('__import', '__exports', transpile(src))(function (spec, wantDefault) {
    const m = imports[spec];
    return wantDefault && m && m.default !== undefined ? m.default : m;
  }, exp);
  return exp;
}

const React = {
  Fragment: 'F',
  createElement: function (type, props) {
    return { type: type, props: props, children: Array.prototype.slice.call(arguments, 2) };
  },
};

describe('tsx: JSX → React.createElement', () => {
  it('elements, attributes, spread, fragments, expression containers and JSX text', () => {
    const m = run(`
      import React from 'react';
      export function view(p: { n: number; rest: Record<string, string> }) {
        return (
          <>
            <div className="a" aria-label="x y" data-n={p.n} {...p.rest} hidden>
              Hello &amp; welcome{' '}
              <b>{p.n > 1 ? 'many' : 'one'}</b>
              {/* a comment */}
            </div>
            <Child value={<i>nested</i>} />
          </>
        );
      }
      function Child() { return null; }
    `, { react: React });
    const el = m.view({ n: 2, rest: { id: 'r' } });
    expect(el.type).toBe('F');
    const div = el.children[0];
    expect(div.type).toBe('div');
    expect(div.props).toEqual({ className: 'a', 'aria-label': 'x y', 'data-n': 2, id: 'r', hidden: true });
    expect(div.children[0]).toBe('Hello & welcome');
    expect(div.children[1]).toBe(' ');
    expect(div.children[2]).toEqual({ type: 'b', props: null, children: ['many'] });
    expect(div.children).toHaveLength(3);
    expect(el.children[1].props.value.type).toBe('i');
  });

  it('a < b is a comparison, Map<K, V>() a generic call, not JSX', () => {
    const src = 'const a = 1 < 2;\nconst m = new Map<string, string[]>();\nconst s = useState<Foo | null>(null);';
    const out = stripTypes(transformJsx(src));
    expect(out).toContain('1 < 2');
    expect(out).toContain('new Map()');
    expect(out).toContain('useState(null)');
  });
});

describe('tsx: TypeScript erasure', () => {
  it('interfaces, type aliases, annotations, casts, type predicates, catch bindings, non-null', () => {
    const src = `
      export interface A { x: number; y?: string; z: Array<{ k: string }> }
      export type T = 'a' | 'b';
      export function f(value: unknown, n: number = 2, o?: A): value is A {
        const r: Record<string, number> = { a: 1 };
        const v = (value as Record<string, unknown>)['x'] as number | undefined;
        try { throw new Error('e'); } catch (e: unknown) { r.c = 3; }
        const g = (q: string): number => q.length;
        return r.a + (v || 0) + g('ab') + new Map<string, number>([['k', n]]).get('k')!;
      }
      export const K = 'x' as const;
    `;
    const m = run(src, {});
    expect(m.f({ x: 1 })).toBe(6);
    expect(m.K).toBe('x');
    expect(stripTypes(src)).not.toContain('interface');
  });
});

describe('tsx: optional chaining and nullish coalescing → ES2019', () => {
  it('chains, calls, index access, spread and nesting keep their semantics', () => {
    const m = run(`
      export function t(o: any) {
        return [o?.a?.b ?? 'd', o?.list?.length ?? 0, o?.['k'], o?.f?.(2), { ...o?.s }, (o?.n ?? 1) + 1, o?.m.get('x') ?? 'none'];
      }
    `, {});
    expect(m.t(null)).toEqual(['d', 0, undefined, undefined, {}, 2, 'none']);
    expect(m.t({ a: { b: 0 }, list: [1, 2], k: 'v', f: (x) => x * 2, s: { z: 1 }, n: 0, m: new Map([['x', 'y']]) }))
      .toEqual([0, 2, 'v', 4, { z: 1 }, 1, 'y']);
  });

  it('the left side is evaluated once', () => {
    let calls = 0;
    const m = run('export function t(f: () => any) { return f()?.x ?? f(); }', {});
    expect(m.t(() => { calls++; return { x: 7 }; })).toBe(7);
    expect(calls).toBe(1);
  });

  it('template literal expressions are lowered too', () => {
    expect(lowerOptional('const s = `${a?.b ?? "x"}!`;')).not.toContain('?.');
  });
});

describe('tsx: modules', () => {
  it('imports (default, named, renamed, type-only) and exports', () => {
    const out = lowerModules("import A, { b, type C, d as e } from 'm';\nexport default function F() {}\nexport const K = 1;");
    expect(out).toContain("const A = __import(\"m\", true);");
    expect(out).toContain('const { b, C, d: e } = __import("m");');
    expect(out).toContain('__exports.default = F;');
    expect(out).toContain('__exports.K = K;');
  });

  it('transpile: one module body over __import / __exports', () => {
    const body = transpile("import { two } from './b';\nexport const three: number = two + 1;\n");
    const exp = {};
    // eslint-disable-next-line no-new-func
    new Function('__import', '__exports', body)(function () { return { two: 2 }; }, exp);
    expect(exp.three).toBe(3);
  });
});

describe('the render comparison refuses to run the reference unless asked, in a sandboxed process', () => {
  it('assertReferenceSandbox: the opt-in, then the process flag', async () => {
    const { assertReferenceSandbox } = await import('../../bench/compareRenders.js');
    expect(() => assertReferenceSandbox({})).toThrow('--allow-reference-exec');
    expect(() => assertReferenceSandbox({ allowReferenceExec: 'yes' })).toThrow('--allow-reference-exec');
    // The spec runner is not started with --disallow-code-generation-from-strings.
    expect(() => assertReferenceSandbox({ allowReferenceExec: true })).toThrow('--disallow-code-generation-from-strings');
  });
});
