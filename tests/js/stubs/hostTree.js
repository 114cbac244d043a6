/**
 * The host tree the harness React (./react.js) renders — {tag, props,
 * children} nodes and strings — serialised (text, HTML) and queried
 * testing-library style (getByText, getByLabelText, getByTestId, …).
 */

export function textOf(node) {
  if (typeof node === 'string') return node;
  let s = '';
  for (let i = 0; i < node.children.length; i++) s += textOf(node.children[i]);
  return s;
}

const VOID = { br: true, input: true, hr: true, img: true };

function esc(s) {
  return String(s).replace(/&/g, '&amp;').replace(/</g, '&lt;').replace(/>/g, '&gt;').replace(/"/g, '&quot;');
}

function attrs(props) {
  let s = '';
  const keys = Object.keys(props).sort();
  for (let i = 0; i < keys.length; i++) {
    const k = keys[i];
    const v = props[k];
    if (v === null || v === undefined || v === false || typeof v === 'function' || k === 'style') continue;
    s += ' ' + k + (v === true ? '' : '="' + esc(v) + '"');
  }
  return s;
}

export function htmlOf(node) {
  if (typeof node === 'string') return esc(node);
  const inner = node.children.map(htmlOf).join('');
  if (VOID[node.tag]) return '<' + node.tag + attrs(node.props) + '>';
  return '<' + node.tag + attrs(node.props) + '>' + inner + '</' + node.tag + '>';
}

function walk(nodes, fn) {
  for (let i = 0; i < nodes.length; i++) {
    const n = nodes[i];
    if (typeof n === 'string') continue;
    fn(n);
    walk(n.children, fn);
  }
}

function matches(text, m) {
  const t = text.replace(/\s+/g, ' ').trim();
  return m instanceof RegExp ? m.test(t) : t === m;
}

/** The testing-library style queries over the host nodes `nodes()` returns. */
export function hostQueries(nodes) {
  const handle = {
    /** Host nodes (deepest first match semantics like testing-library). */
    queryAll: function (pred) {
      const out = [];
      walk(nodes(), function (n) { if (pred(n)) out.push(n); });
      return out;
    },
    getAllByText: function (m) {
      const hits = handle.queryAll(function (n) {
        if (!matches(textOf(n), m)) return false;
        // deepest: no host child matches as well
        for (let i = 0; i < n.children.length; i++) {
          const c = n.children[i];
          if (typeof c !== 'string' && matches(textOf(c), m)) return false;
        }
        return true;
      });
      if (hits.length === 0) throw new Error('Unable to find an element with the text: ' + String(m));
      return hits;
    },
    getByText: function (m) {
      const hits = handle.getAllByText(m);
      if (hits.length > 1) throw new Error('Found multiple elements with the text: ' + String(m));
      return hits[0];
    },
    queryByText: function (m) {
      try {
        return handle.getByText(m);
      } catch (e) {
        return null;
      }
    },
    getByLabelText: function (label) {
      const hits = handle.queryAll(function (n) { return n.props['aria-label'] !== undefined && matches(String(n.props['aria-label']), label); });
      if (hits.length !== 1) throw new Error((hits.length ? 'Found multiple' : 'Unable to find') + ' elements labelled ' + String(label));
      return hits[0];
    },
    getAllByTestId: function (id) {
      const hits = handle.queryAll(function (n) { return n.props['data-testid'] === id; });
      if (hits.length === 0) throw new Error('Unable to find data-testid=' + id);
      return hits;
    },
    getByTestId: function (id) {
      const hits = handle.getAllByTestId(id);
      if (hits.length > 1) throw new Error('Found multiple data-testid=' + id);
      return hits[0];
    },
    byTag: function (tag) {
      return handle.queryAll(function (n) { return n.tag === tag; });
    },
  };
  return handle;
}
