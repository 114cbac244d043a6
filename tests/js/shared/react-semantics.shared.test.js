/**
 * React 18 semantics the plugin relies on, as runner-agnostic specs: the
 * same file checks the harness React (tests/js/harness/stub.js) and real
 * React 18.3.1 + react-dom — offline through the UMD builds
 * (tests/js/harness/umd.js, tests/test_js_real_react.py) and under jsdom in
 * networked CI (tests/js/harness/dom.js). A spec that passes on react-dom and
 * fails on the harness is a fidelity bug of the harness.
 *
 * Covered: commit order of layout / passive effects and their cleanups
 * (mount, update, deletion), StrictMode's double render and effect replay,
 * automatic batching, functional updates, memo bail-out and context through
 * a memo boundary, key-driven remounts, hook identity (useRef, useCallback,
 * useMemo), and useSyncExternalStore's snapshot comparison and unsubscribe.
 * Components count their own renders in test-local variables; nothing reads
 * harness internals.
 */
import { React, render, tier } from 'amd-test-harness';

const h = React.createElement;

describe('React semantics: effect commit order (' + tier + ')', () => {
  it('on mount: layout effects before passive ones, children before parents', async () => {
    const log = [];
    function Child() {
      React.useLayoutEffect(() => { log.push('layout child'); }, []);
      React.useEffect(() => { log.push('passive child'); }, []);
      return h('span', null, 'c');
    }
    function Parent() {
      React.useLayoutEffect(() => { log.push('layout parent'); }, []);
      React.useEffect(() => { log.push('passive parent'); }, []);
      return h('div', null, h(Child));
    }
    const r = render(h(Parent));
    await r.settle();
    expect(log).toEqual(['layout child', 'layout parent', 'passive child', 'passive parent']);
    r.unmount();
  });

  it('on update: every cleanup of a phase runs before any of its new effects', async () => {
    const log = [];
    function Child(p) {
      React.useEffect(() => {
        log.push('effect child ' + p.v);
        return () => log.push('cleanup child ' + p.v);
      }, [p.v]);
      return h('span', null, String(p.v));
    }
    function Parent(p) {
      React.useEffect(() => {
        log.push('effect parent ' + p.v);
        return () => log.push('cleanup parent ' + p.v);
      }, [p.v]);
      return h('div', null, h(Child, { v: p.v }));
    }
    const r = render(h(Parent, { v: 1 }));
    await r.settle();
    log.length = 0;
    r.rerender(h(Parent, { v: 2 }));
    await r.settle();
    expect(log).toEqual(['cleanup child 1', 'cleanup parent 1', 'effect child 2', 'effect parent 2']);
    expect(r.text()).toBe('2');
    r.unmount();
  });

  it('on deletion: cleanups run parent before child, layout before passive', async () => {
    const log = [];
    function Child() {
      React.useLayoutEffect(() => () => log.push('layout child'), []);
      React.useEffect(() => () => log.push('passive child'), []);
      return h('span', null, 'c');
    }
    function Parent() {
      React.useLayoutEffect(() => () => log.push('layout parent'), []);
      React.useEffect(() => () => log.push('passive parent'), []);
      return h('div', null, h(Child));
    }
    const r = render(h('section', null, h(Parent)));
    await r.settle();
    r.rerender(h('section', null, null));
    await r.settle();
    expect(log).toEqual(['layout parent', 'layout child', 'passive parent', 'passive child']);
    r.unmount();
  });

  it('an effect without deps runs after every commit; one with [] only once', async () => {
    let every = 0;
    let once = 0;
    function C(p) {
      React.useEffect(() => { every++; });
      React.useEffect(() => { once++; }, []);
      return h('span', null, String(p.v));
    }
    const r = render(h(C, { v: 1 }));
    await r.settle();
    r.rerender(h(C, { v: 2 }));
    await r.settle();
    r.rerender(h(C, { v: 3 }));
    await r.settle();
    expect(every).toBe(3);
    expect(once).toBe(1);
    r.unmount();
  });
});

describe('React semantics: StrictMode, development build (' + tier + ')', () => {
  it('calls a component body twice per render', async () => {
    let bodies = 0;
    function C() {
      bodies++;
      return h('span', null, 'x');
    }
    const r = render(h(C), { strict: true });
    await r.settle();
    expect(bodies).toBe(2);
    r.unmount();
  });

  it('mounts each new effect, tears it down and mounts it again; later updates run once', async () => {
    const log = [];
    function C(p) {
      React.useEffect(() => {
        log.push('mount ' + p.v);
        return () => log.push('cleanup ' + p.v);
      }, [p.v]);
      return h('span', null, String(p.v));
    }
    const r = render(h(C, { v: 1 }), { strict: true });
    await r.settle();
    expect(log).toEqual(['mount 1', 'cleanup 1', 'mount 1']);
    log.length = 0;
    r.rerender(h(C, { v: 2 }));
    await r.settle();
    expect(log).toEqual(['cleanup 1', 'mount 2']);
    r.unmount();
    expect(log).toEqual(['cleanup 1', 'mount 2', 'cleanup 2']);
  });
});

describe('React semantics: state updates (' + tier + ')', () => {
  it('two updates in one event handler commit in one render', async () => {
    let bodies = 0;
    function C() {
      bodies++;
      const [a, setA] = React.useState(0);
      const [b, setB] = React.useState(0);
      return h('button', { 'aria-label': 'both', onClick: () => { setA(a + 1); setB(b + 10); } }, a + ':' + b);
    }
    const r = render(h(C));
    await r.settle();
    const before = bodies;
    r.click(r.byLabel('both'));
    await r.settle();
    expect(r.text()).toBe('1:10');
    expect(bodies).toBe(before + 1);
    r.unmount();
  });

  it('updates from a resolved promise are batched too (automatic batching)', async () => {
    let bodies = 0;
    function C() {
      bodies++;
      const [a, setA] = React.useState(0);
      const [b, setB] = React.useState(0);
      React.useEffect(() => {
        Promise.resolve().then(() => {
          setA(1);
          setB(2);
        });
      }, []);
      return h('span', null, a + ':' + b);
    }
    const r = render(h(C));
    await r.settle();
    expect(r.text()).toBe('1:2');
    expect(bodies).toBe(2);
    r.unmount();
  });

  it('functional updates compose; a lazy initial state is computed once', async () => {
    let inits = 0;
    function C() {
      const [n, setN] = React.useState(() => {
        inits++;
        return 0;
      });
      return h('button', { 'aria-label': 'inc', onClick: () => { setN((x) => x + 1); setN((x) => x + 1); } }, String(n));
    }
    const r = render(h(C));
    await r.settle();
    r.click(r.byLabel('inc'));
    await r.settle();
    r.click(r.byLabel('inc'));
    await r.settle();
    expect(r.text()).toBe('4');
    expect(inits).toBe(1);
    r.unmount();
  });

  it('a state update from an effect re-renders once more and then settles', async () => {
    let bodies = 0;
    function C() {
      bodies++;
      const [ready, setReady] = React.useState(false);
      React.useEffect(() => { setReady(true); }, []);
      return h('span', null, ready ? 'ready' : 'pending');
    }
    const r = render(h(C));
    await r.settle();
    expect(r.text()).toBe('ready');
    expect(bodies).toBe(2);
    r.unmount();
  });
});

describe('React semantics: memo, context and keys (' + tier + ')', () => {
  it('memo skips a child whose props are shallow-equal; a plain child re-renders', async () => {
    const counts = { memo: 0, plain: 0 };
    const Memo = React.memo(function Memo(p) {
      counts.memo++;
      return h('i', null, p.label);
    });
    function Plain() {
      counts.plain++;
      return h('b', null, 'p');
    }
    function Parent() {
      const [n, setN] = React.useState(0);
      return h('div', null,
        h('button', { 'aria-label': 'bump', onClick: () => setN(n + 1) }, String(n)),
        h(Memo, { label: 'same' }),
        h(Plain));
    }
    const r = render(h(Parent));
    await r.settle();
    r.click(r.byLabel('bump'));
    await r.settle();
    expect(counts).toEqual({ memo: 1, plain: 2 });
    r.unmount();
  });

  it('a context change reaches a consumer below a memo boundary', async () => {
    const Ctx = React.createContext('default');
    let consumer = 0;
    function Reader() {
      consumer++;
      return h('span', null, React.useContext(Ctx));
    }
    const Wall = React.memo(function Wall() {
      return h('div', null, h(Reader));
    });
    function App() {
      const [v, setV] = React.useState('a');
      return h(Ctx.Provider, { value: v },
        h('button', { 'aria-label': 'set', onClick: () => setV('b') }, 'set'),
        h(Wall));
    }
    const r = render(h(App));
    await r.settle();
    expect(r.text()).toBe('seta');
    r.click(r.byLabel('set'));
    await r.settle();
    expect(r.text()).toBe('setb');
    expect(consumer).toBe(2);
    r.unmount();
  });

  it('a consumer with no provider above it reads the default value', async () => {
    const Ctx = React.createContext('fallback');
    function Reader() {
      return h('span', null, React.useContext(Ctx));
    }
    const r = render(h(Reader));
    await r.settle();
    expect(r.text()).toBe('fallback');
    r.unmount();
  });

  it('a changed key remounts: state resets and the effect cleans up and mounts again', async () => {
    const log = [];
    function Counter(p) {
      const [n, setN] = React.useState(0);
      React.useEffect(() => {
        log.push('mount ' + p.id);
        return () => log.push('cleanup ' + p.id);
      }, []);
      return h('button', { 'aria-label': 'inc', onClick: () => setN(n + 1) }, p.id + '=' + n);
    }
    const r = render(h(Counter, { key: 'a', id: 'a' }));
    await r.settle();
    r.click(r.byLabel('inc'));
    await r.settle();
    expect(r.text()).toBe('a=1');
    r.rerender(h(Counter, { key: 'b', id: 'b' }));
    await r.settle();
    expect(r.text()).toBe('b=0');
    expect(log).toEqual(['mount a', 'cleanup a', 'mount b']);
    r.unmount();
  });

  it('keyed list items keep their state when the list is reordered', async () => {
    function Item(p) {
      const [clicks, setClicks] = React.useState(0);
      return h('button', { 'aria-label': 'item ' + p.id, onClick: () => setClicks(clicks + 1) }, p.id + clicks);
    }
    function List(p) {
      return h('div', null, p.ids.map((id) => h(Item, { key: id, id: id })));
    }
    const r = render(h(List, { ids: ['x', 'y'] }));
    await r.settle();
    r.click(r.byLabel('item y'));
    await r.settle();
    r.rerender(h(List, { ids: ['y', 'x'] }));
    await r.settle();
    expect(r.text()).toBe('y1x0');
    r.unmount();
  });
});

describe('React semantics: hook identity (' + tier + ')', () => {
  it('useRef and useCallback keep their identity; useMemo recomputes only when a dep changes', async () => {
    const refs = [];
    const cbs = [];
    let computed = 0;
    function C(p) {
      const ref = React.useRef(null);
      const cb = React.useCallback(() => p.a, [p.a]);
      const memo = React.useMemo(() => {
        computed++;
        return p.a * 2;
      }, [p.a]);
      refs.push(ref);
      cbs.push(cb);
      return h('span', null, String(memo));
    }
    const r = render(h(C, { a: 1, b: 1 }));
    await r.settle();
    r.rerender(h(C, { a: 1, b: 2 }));
    await r.settle();
    r.rerender(h(C, { a: 5, b: 2 }));
    await r.settle();
    expect(refs[0] === refs[1] && refs[1] === refs[2]).toBe(true);
    expect(cbs[0] === cbs[1]).toBe(true);
    expect(cbs[1] === cbs[2]).toBe(false);
    expect(computed).toBe(2);
    expect(r.text()).toBe('10');
    r.unmount();
  });

  it('a ref written in an effect is read by the next render', async () => {
    function C(p) {
      const prev = React.useRef('none');
      const shown = prev.current;
      React.useEffect(() => { prev.current = p.v; });
      return h('span', null, shown + '->' + p.v);
    }
    const r = render(h(C, { v: 'a' }));
    await r.settle();
    r.rerender(h(C, { v: 'b' }));
    await r.settle();
    expect(r.text()).toBe('a->b');
    r.unmount();
  });
});

describe('React semantics: useSyncExternalStore (' + tier + ')', () => {
  function makeStore(initial) {
    let snap = initial;
    const subs = new Set();
    return {
      subs: subs,
      subscribe: (fn) => {
        subs.add(fn);
        return () => subs.delete(fn);
      },
      get: () => snap,
      set: (v) => {
        snap = v;
        subs.forEach((fn) => fn());
      },
      poke: () => subs.forEach((fn) => fn()),
    };
  }

  it('re-renders on a new snapshot, not on a notification with the same one; unsubscribes on unmount', async () => {
    const store = makeStore({ n: 1 });
    let bodies = 0;
    function C() {
      bodies++;
      const s = React.useSyncExternalStore(store.subscribe, store.get);
      return h('span', null, String(s.n));
    }
    const r = render(h(C));
    await r.settle();
    expect(store.subs.size).toBe(1);
    const before = bodies;
    // Store changes inside act(), as React expects in a test (outside it, React
    // 18.3 warns and may render an external-store update twice).
    r.act(() => store.poke());
    await r.settle();
    expect(bodies).toBe(before);
    r.act(() => store.set({ n: 2 }));
    await r.settle();
    expect(r.text()).toBe('2');
    expect(bodies).toBe(before + 1);
    r.unmount();
    expect(store.subs.size).toBe(0);
  });

  it('a store change between render and subscribe is not lost', async () => {
    const store = makeStore('old');
    function C() {
      const s = React.useSyncExternalStore(store.subscribe, store.get);
      React.useLayoutEffect(() => {
        if (store.get() === 'old') store.set('changed-before-subscribe');
      }, []);
      return h('span', null, s);
    }
    const r = render(h(C));
    await r.settle();
    expect(r.text()).toBe('changed-before-subscribe');
    r.unmount();
  });
});

describe('React semantics: form fields (' + tier + ')', () => {
  it('an uncontrolled field keeps what the user typed; a later defaultValue does not reach the screen', () => {
    const r = render(h('input', { 'aria-label': 'f', defaultValue: 'a' }));
    expect(r.value(r.byLabel('f'))).toBe('a');
    r.change(r.byLabel('f'), 'typed');
    r.rerender(h('input', { 'aria-label': 'f', defaultValue: 'b' }));
    expect(r.value(r.byLabel('f'))).toBe('typed');
    r.unmount();
  });

  it('a controlled field shows its value: what the handler stores, or its old value when the handler ignores the edit', () => {
    function Field(props) {
      const st = React.useState('x');
      return h('input', { 'aria-label': 'f', value: st[0], onChange: (e) => { if (props.accept) st[1](e.target.value.toUpperCase()); } });
    }
    const a = render(h(Field, { accept: true }));
    a.change(a.byLabel('f'), 'abc');
    expect(a.value(a.byLabel('f'))).toBe('ABC');
    a.unmount();
    const b = render(h(Field, { accept: false }));
    b.change(b.byLabel('f'), 'abc');
    expect(b.value(b.byLabel('f'))).toBe('x');
    b.unmount();
  });

  it('a remount (new key) starts from the new defaultValue', () => {
    const r = render(h('input', { key: 1, 'aria-label': 'f', defaultValue: 'a' }));
    r.change(r.byLabel('f'), 'typed');
    r.rerender(h('input', { key: 2, 'aria-label': 'f', defaultValue: 'b' }));
    expect(r.value(r.byLabel('f'))).toBe('b');
    r.unmount();
  });
});
