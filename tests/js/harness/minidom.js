/**
 * A minimal DOM for running react-dom 18 under bare Node (no jsdom offline):
 * documents, elements, text and comment nodes, attributes, inline styles,
 * capture / bubble event dispatch, and the form-control properties React's
 * input / select wrappers use (value with a prototype accessor, so React's
 * value tracker attaches; select.options; option.selected). Only what
 * react-dom's client renderer and the shared specs touch is modelled.
 */

const ELEMENT_NODE = 1;
const TEXT_NODE = 3;
const COMMENT_NODE = 8;
const DOCUMENT_NODE = 9;
const DOCUMENT_FRAGMENT_NODE = 11;
const HTML_NS = 'http://www.w3.org/1999/xhtml';

export class Event {
  constructor(type, init) {
    const o = init || {};
    this.type = type;
    this.bubbles = !!o.bubbles;
    this.cancelable = !!o.cancelable;
    this.defaultPrevented = false;
    this.target = null;
    this.currentTarget = null;
    this.eventPhase = 0;
    this.timeStamp = Date.now();
    this.isTrusted = false;
    this._stop = false;
    this._stopNow = false;
  }
  preventDefault() { if (this.cancelable) this.defaultPrevented = true; }
  stopPropagation() { this._stop = true; }
  stopImmediatePropagation() { this._stop = true; this._stopNow = true; }
}

class Target {
  constructor() { this._listeners = {}; }
  addEventListener(type, fn, opts) {
    if (!fn) return;
    const capture = opts === true || !!(opts && opts.capture);
    const list = this._listeners[type] || (this._listeners[type] = []);
    for (let i = 0; i < list.length; i++) if (list[i].fn === fn && list[i].capture === capture) return;
    list.push({ fn: fn, capture: capture });
  }
  removeEventListener(type, fn, opts) {
    const capture = opts === true || !!(opts && opts.capture);
    const list = this._listeners[type];
    if (!list) return;
    this._listeners[type] = list.filter(function (l) { return !(l.fn === fn && l.capture === capture); });
  }
  _fire(evt, capturePhase) {
    const list = (this._listeners[evt.type] || []).slice();
    evt.currentTarget = this;
    for (let i = 0; i < list.length; i++) {
      if (list[i].capture !== capturePhase) continue;
      list[i].fn.call(this, evt);
      if (evt._stopNow) return;
    }
  }
  dispatchEvent(evt) {
    evt.target = this;
    const path = [];
    for (let n = this.parentNode; n; n = n.parentNode) path.push(n);
    const win = this.ownerDocument && this.ownerDocument.defaultView;
    if (path.length && path[path.length - 1].nodeType === DOCUMENT_NODE && win) path.push(win);
    evt.eventPhase = 1;
    for (let i = path.length - 1; i >= 0 && !evt._stop; i--) path[i]._fire(evt, true);
    evt.eventPhase = 2;
    if (!evt._stop) this._fire(evt, true);
    if (!evt._stop) this._fire(evt, false);
    evt.eventPhase = 3;
    if (evt.bubbles) for (let i = 0; i < path.length && !evt._stop; i++) path[i]._fire(evt, false);
    evt.eventPhase = 0;
    evt.currentTarget = null;
    return !evt.defaultPrevented;
  }
}

export class Node extends Target {
  constructor(doc, type, name) {
    super();
    this.ownerDocument = doc;
    this.nodeType = type;
    this.nodeName = name;
    this.parentNode = null;
    this.childNodes = [];
  }
  get firstChild() { return this.childNodes[0] || null; }
  get lastChild() { return this.childNodes[this.childNodes.length - 1] || null; }
  get parentElement() { return this.parentNode && this.parentNode.nodeType === ELEMENT_NODE ? this.parentNode : null; }
  get nextSibling() {
    const p = this.parentNode;
    if (!p) return null;
    return p.childNodes[p.childNodes.indexOf(this) + 1] || null;
  }
  get previousSibling() {
    const p = this.parentNode;
    if (!p) return null;
    return p.childNodes[p.childNodes.indexOf(this) - 1] || null;
  }
  hasChildNodes() { return this.childNodes.length > 0; }
  appendChild(c) { return this.insertBefore(c, null); }
  insertBefore(c, ref) {
    if (c.nodeType === DOCUMENT_FRAGMENT_NODE) {
      const kids = c.childNodes.slice();
      for (let i = 0; i < kids.length; i++) this.insertBefore(kids[i], ref);
      return c;
    }
    if (c.parentNode) c.parentNode.removeChild(c);
    const at = ref ? this.childNodes.indexOf(ref) : -1;
    if (ref && at < 0) throw new Error('insertBefore: the reference node is not a child');
    if (at < 0) this.childNodes.push(c);
    else this.childNodes.splice(at, 0, c);
    c.parentNode = this;
    return c;
  }
  removeChild(c) {
    const i = this.childNodes.indexOf(c);
    if (i < 0) throw new Error('removeChild: not a child');
    this.childNodes.splice(i, 1);
    c.parentNode = null;
    return c;
  }
  contains(n) {
    for (let x = n; x; x = x.parentNode) if (x === this) return true;
    return false;
  }
  get textContent() {
    if (this.nodeType === TEXT_NODE || this.nodeType === COMMENT_NODE) return this.nodeValue;
    let s = '';
    for (let i = 0; i < this.childNodes.length; i++) if (this.childNodes[i].nodeType !== COMMENT_NODE) s += this.childNodes[i].textContent;
    return s;
  }
  set textContent(v) {
    if (this.nodeType === TEXT_NODE || this.nodeType === COMMENT_NODE) {
      this.nodeValue = String(v);
      return;
    }
    while (this.childNodes.length) this.removeChild(this.childNodes[0]);
    if (v !== '' && v !== null && v !== undefined) this.appendChild(this.ownerDocument.createTextNode(String(v)));
  }
  /** `tag` or `[attr]` (what the harness adapters ask for), descendants in document order. */
  querySelectorAll(sel) {
    const attr = /^\[([^\]=]+)\]$/.exec(sel);
    const want = attr ? null : sel.toLowerCase();
    const out = [];
    (function walk(n) {
      for (let i = 0; i < n.childNodes.length; i++) {
        const c = n.childNodes[i];
        if (c.nodeType !== ELEMENT_NODE) continue;
        if (attr ? c.hasAttribute(attr[1]) : want === '*' || c.localName === want) out.push(c);
        walk(c);
      }
    })(this);
    return out;
  }
  querySelector(sel) { return this.querySelectorAll(sel)[0] || null; }
}

export class Text extends Node {
  constructor(doc, data) {
    super(doc, TEXT_NODE, '#text');
    this.nodeValue = data;
  }
  get data() { return this.nodeValue; }
  set data(v) { this.nodeValue = String(v); }
}

export class Comment extends Node {
  constructor(doc, data) {
    super(doc, COMMENT_NODE, '#comment');
    this.nodeValue = data;
  }
  get data() { return this.nodeValue; }
}

/** element.style: declarations as own properties, the CSSStyleDeclaration methods on the prototype. */
class Style {
  setProperty(k, v) { this[k] = String(v); }
  removeProperty(k) { delete this[k]; }
  getPropertyValue(k) { return Object.prototype.hasOwnProperty.call(this, k) ? this[k] : ''; }
}

function makeStyle() {
  return new Style();
}

export class Element extends Node {
  constructor(doc, tag, ns) {
    const html = !ns || ns === HTML_NS;
    super(doc, ELEMENT_NODE, html ? tag.toUpperCase() : tag);
    this.namespaceURI = ns || HTML_NS;
    this.localName = html ? tag.toLowerCase() : tag;
    this.tagName = this.nodeName;
    this._attrs = new Map();
    this.style = makeStyle();
    this._value = null; // input / select / textarea value once set as a property
    this._selected = null; // option
  }
  getAttribute(k) { return this._attrs.has(k) ? this._attrs.get(k) : null; }
  setAttribute(k, v) { this._attrs.set(k, String(v)); }
  removeAttribute(k) { this._attrs.delete(k); }
  hasAttribute(k) { return this._attrs.has(k); }
  getAttributeNS(ns, k) { return this.getAttribute(k); }
  setAttributeNS(ns, k, v) { this.setAttribute(k, v); }
  removeAttributeNS(ns, k) { this.removeAttribute(k); }
  get attributes() {
    const out = [];
    this._attrs.forEach(function (v, k) { out.push({ name: k, value: v }); });
    return out;
  }
  get children() { return this.childNodes.filter(function (c) { return c.nodeType === ELEMENT_NODE; }); }
  /** input.type defaults to "text" (React's change plugin keys text inputs on it). */
  get type() {
    if (this.hasAttribute('type')) return this.getAttribute('type').toLowerCase();
    if (this.localName === 'input') return 'text';
    if (this.localName === 'button') return 'submit';
    if (this.localName === 'select') return this.multiple ? 'select-multiple' : 'select-one';
    return '';
  }
  set type(v) { this.setAttribute('type', v); }
  get disabled() { return this.hasAttribute('disabled'); }
  set disabled(v) { if (v) this.setAttribute('disabled', ''); else this.removeAttribute('disabled'); }
  focus() { this.ownerDocument.activeElement = this; }
  blur() { if (this.ownerDocument.activeElement === this) this.ownerDocument.activeElement = this.ownerDocument.body; }

  // Form controls. React's value tracker reads the accessor from the prototype.
  get value() {
    if (this.localName === 'select') {
      const opts = this.options;
      for (let i = 0; i < opts.length; i++) if (opts[i].selected) return opts[i].value;
      return opts.length ? opts[0].value : '';
    }
    if (this.localName === 'option') return this.hasAttribute('value') ? this.getAttribute('value') : this.textContent;
    if (this._value !== null) return this._value;
    return this.hasAttribute('value') ? this.getAttribute('value') : '';
  }
  set value(v) {
    const s = String(v);
    if (this.localName === 'select') {
      const opts = this.options;
      for (let i = 0; i < opts.length; i++) opts[i]._selected = opts[i].value === s;
      return;
    }
    if (this.localName === 'option') {
      this.setAttribute('value', s);
      return;
    }
    this._value = s;
  }
  // The value attribute: an uncontrolled field's initial value (React sets defaultValue).
  get defaultValue() { return this.hasAttribute('value') ? this.getAttribute('value') : ''; }
  set defaultValue(v) { this.setAttribute('value', v); }
  get options() { return this.localName === 'select' ? this.querySelectorAll('option') : undefined; }
  get selectedIndex() {
    const opts = this.options || [];
    for (let i = 0; i < opts.length; i++) if (opts[i].selected) return i;
    return -1;
  }
  get selected() {
    if (this._selected !== null) return this._selected;
    return this.hasAttribute('selected');
  }
  set selected(v) {
    this._selected = !!v;
    // A single select holds one selected option.
    let sel = this.parentNode;
    while (sel && sel.localName !== 'select') sel = sel.parentNode;
    if (v && sel && !sel.multiple) {
      const opts = sel.options;
      for (let i = 0; i < opts.length; i++) if (opts[i] !== this) opts[i]._selected = false;
    }
  }
}

export class Document extends Node {
  constructor() {
    super(null, DOCUMENT_NODE, '#document');
    this.ownerDocument = null;
    this.documentElement = new Element(this, 'html');
    this.body = new Element(this, 'body');
    this.head = new Element(this, 'head');
    this.appendChild(this.documentElement);
    this.documentElement.appendChild(this.head);
    this.documentElement.appendChild(this.body);
    this.activeElement = this.body;
    this.defaultView = null;
    // react-dom's isEventSupported('input') looks for the handler property.
    this.oninput = null;
  }
  createElement(tag) { return new Element(this, tag, HTML_NS); }
  createElementNS(ns, tag) { return new Element(this, tag, ns); }
  createTextNode(s) { return new Text(this, String(s)); }
  createComment(s) { return new Comment(this, String(s)); }
  createDocumentFragment() { return new Node(this, DOCUMENT_FRAGMENT_NODE, '#document-fragment'); }
}

/** A window + document pair: what react-dom probes for at load time and while committing. */
export function createWindow() {
  const document = new Document();
  const window = new Target();
  window.document = document;
  window.Event = Event;
  window.Node = Node;
  window.Element = Element;
  window.HTMLElement = Element;
  window.HTMLIFrameElement = function HTMLIFrameElement() {};
  window.navigator = { userAgent: 'Node.js (minidom)' };
  window.location = { protocol: 'file:', href: 'file:///', pathname: '/', hash: '' };
  window.top = window;
  window.self = window;
  window.event = undefined;
  document.defaultView = window;
  return window;
}
