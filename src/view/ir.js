/**
 * View IR — the declarative page description every view-model returns.
 *
 * A page is a list of items (loaders and sections); a section holds blocks
 * (name/value tables, simple tables, percentage bars, per-GPU slot strips,
 * the xGMI matrix, time series). The TSX layer maps each node 1:1 onto a
 * Headlamp CommonComponent (SectionBox, NameValueTable, SimpleTable,
 * StatusLabel, PercentageBar, Loader); `html.js` maps it onto the same
 * semantic HTML the reference's component tests mock those components with
 * (src/components/OverviewPage.test.tsx:8-61), so the page logic is testable
 * without React.
 */

/** @typedef {'success'|'warning'|'error'} Status */

/** @param {Status} status @param {string|number} text */
export function status(st, text) {
  return { t: 'status', status: st, text: String(text) };
}

/** Inline allocation/power bar: text like "3/8 (38%)". */
export function bar(used, total, pctValue, color, text) {
  return { t: 'bar', used: used, total: total, pct: pctValue, color: color, text: text };
}

/** Multi-line cell: [{label, text}] rendered as "<strong>label</strong>: text". */
export function lines(items) {
  return { t: 'lines', lines: items };
}

export function kv(rows) {
  return { t: 'kv', rows: rows };
}

export function row(name, value) {
  return { name: name, value: value };
}

/** @param {string[]} columns @param {Array<Array<any>>} rows @param {string[]} [keys] */
export function table(columns, rows, keys) {
  return { t: 'table', columns: columns, rows: rows, keys: keys || null };
}

/** PercentageBar: data [{name, value, fill}] of `total`. */
export function pctbar(label, data, total) {
  return { t: 'pctbar', label: label, data: data, total: total };
}

export function section(title, blocks, key) {
  return { t: 'section', title: title, key: key || title, blocks: blocks };
}

export function loader(title) {
  return { t: 'loader', title: title };
}

/**
 * Page-level pager over a long list (GPU nodes): which slice is shown, and
 * the name filter that selected it. A page item, not a section block, so the
 * renderer can wire its buttons to the page's own state.
 * @param {{page: number, pages: number, from: number, to: number, total: number, matched: number,
 *          filter: string, perPage: number}} p
 * @param {string} noun  what is counted ("GPU nodes")
 */
export function pager(p, noun, sorting) {
  const item = {
    // `label` names the controls and stays the same when the noun counts
    // something narrower (a power-ranked page counts "GPU nodes reporting").
    t: 'pager', key: 'pager', noun: noun, label: (sorting && sorting.label) || noun, page: p.page, pages: p.pages, from: p.from, to: p.to,
    total: p.total, matched: p.matched, filter: p.filter, perPage: p.perPage,
  };
  if (p.beyond) item.beyond = true;
  // Offered orders ({value, label}[]) and the current one, when the list can be ranked.
  if (sorting && sorting.sorts) {
    item.sort = sorting.sort;
    item.sorts = sorting.sorts;
  }
  return item;
}

/**
 * True when a pager has nothing to control: the whole list on one page, no
 * filter typed and the default order. Renderers then draw its count line
 * alone (a cluster of a few nodes mounts no filter box, order menu or
 * previous / next buttons); any of the three brings the controls back.
 */
export function pagerIdle(p) {
  const filtered = typeof p.filter === 'string' && p.filter.trim() !== '';
  const sorted = !!p.sorts && p.sorts.length > 0 && !!p.sort && p.sort !== p.sorts[0].value;
  return p.pages <= 1 && !filtered && !sorted && !p.beyond;
}

/** "Showing 17–32 of 1000 GPU nodes" (with the filter's match count when one is set). */
export function pagerText(p) {
  const f = p.filter ? p.filter.trim() : '';
  const of = f ? p.matched + ' matching "' + f + '" (' + p.total + ' ' + p.noun + ')' : p.total + ' ' + p.noun;
  if (p.matched === 0) return 'No ' + p.noun + (f ? ' match "' + f + '"' : '');
  // A ranked page past the end (the count shrank): the component moves to the last page.
  if (p.beyond) return 'Moving to page ' + p.pages + ' of ' + p.pages + ' (' + of + ')';
  return 'Showing ' + (p.from + 1) + '–' + p.to + ' of ' + of + (p.pages > 1 ? ' · page ' + (p.page + 1) + ' of ' + p.pages : '');
}

/**
 * @param {string|null} title  page header (null while the page is only a loader)
 * @param {{label: string, ariaLabel: string, disabled: boolean}|null} refresh
 * @param {any[]} items
 */
export function page(title, refresh, items) {
  return { t: 'page', title: title, refresh: refresh, items: items };
}

// ---------------------------------------------------------------------------
// Memoisation
// ---------------------------------------------------------------------------

// Time-dependent output (ages: "42s", "7m", "3h", "12d") stays valid until
// the first label it shows changes. While a section or row is built, the
// earliest such instant is collected here (noteExpiry), so a cached value can
// be reused until then instead of being rebuilt on every clock tick.
// `building`: a value is being built; `until`: its earliest label change so
// far; `lastUntil`: the horizon of the value computeWithHorizon just built.
// Plain variables, saved and restored around nested builds: a cold page
// build makes a few dozen memo entries, and an object per entry for its
// horizon was a measurable share of it.
let building = false;
let until = Infinity;
let lastUntil = Infinity;

/** Record that the value being built changes at epoch-ms `t`. */
export function noteExpiry(t) {
  if (building && t < until) until = t;
}

/** `compute()`, noting the earliest label change inside it in `lastUntil` (and in the enclosing build). */
function computeWithHorizon(compute) {
  const savedBuilding = building;
  const savedUntil = until;
  building = true;
  until = Infinity;
  let value;
  let mine;
  try {
    value = compute();
  } finally {
    mine = until;
    building = savedBuilding;
    until = savedUntil;
  }
  noteExpiry(mine); // a nested value bounds the enclosing one
  lastUntil = mine;
  return value;
}

function sameDeps(a, b) {
  if (a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) if (a[i] !== b[i]) return false;
  return true;
}

function fresh(e, deps, now) {
  if (!e || !sameDeps(e.deps, deps)) return false;
  if (now === undefined) return true;
  return now >= e.from && now < e.until;
}

/**
 * Identity-keyed memo with a bounded number of slots. `memo(key, deps, fn)`
 * returns the previous value for `key` when every dep is `===` to last time.
 * The store keeps unchanged lists by identity (structural sharing), so
 * sections whose inputs did not change are returned as the SAME IR objects —
 * which `React.memo` (react.js Section) and `renderSection`'s cache then skip.
 *
 * `memo(key, deps, fn, now)` also holds the value only until the first age
 * label inside it changes (see noteExpiry), instead of keying on the clock.
 */
export function createMemo(limit) {
  const max = limit || 256;
  const slots = new Map();
  function memo(key, deps, compute, now) {
    const e = slots.get(key);
    if (fresh(e, deps, now)) {
      noteExpiry(e.until);
      return e.value;
    }
    const value = computeWithHorizon(compute);
    // Most recently built last (the LRU order): an entry being replaced moves to the end.
    if (e) slots.delete(key);
    slots.set(key, { deps: deps, value: value, until: lastUntil, from: now === undefined ? -Infinity : now });
    if (slots.size > max) slots.delete(slots.keys().next().value);
    return value;
  }
  memo.clear = function () { slots.clear(); };
  memo.size = function () { return slots.size; };
  return memo;
}

/**
 * Per-object cache of derived values (table rows of a pod, a node), keyed on
 * the Kubernetes object itself: a watch event that changes one pod rebuilds
 * that pod's row only. Same contract as `memo` (deps + age expiry); entries
 * go away with their objects.
 */
export function createObjectCache() {
  let cache = new WeakMap();
  function cached(obj, deps, compute, now) {
    const e = cache.get(obj);
    if (fresh(e, deps, now)) {
      noteExpiry(e.until);
      return e.value;
    }
    const value = computeWithHorizon(compute);
    cache.set(obj, { deps: deps, value: value, until: lastUntil, from: now === undefined ? -Infinity : now });
    return value;
  }
  cached.clear = function () { cache = new WeakMap(); };
  return cached;
}

// ---------------------------------------------------------------------------
// Shared captions (React, HTML and text renderers)
// ---------------------------------------------------------------------------

/**
 * Caption of the xGMI matrix: whether the link topology was measured or is
 * the platform model, and what throughput was measured — per link only when
 * a series pinned each row to its peer (topology.js placeThroughput), else
 * per GPU with the neighbour order said to be unknown.
 */
export function matrixCaption(b) {
  // Blocks of pages/nodes.js matrixBlock carry the facts; a hand-made block only its grid.
  const m = b.linksPerGpu !== undefined ? b : b.matrix;
  const peak = m.size > 1 ? ' ' + (b.linkGBs !== undefined ? b.linkGBs : m.cells[0][1].peakGBs) : '';
  const perGpu = b.throughputPerGpu !== undefined ? b.throughputPerGpu : !!gridGpuStats(b.matrix);
  const kind = (b.measuredTopology ? 'measured' : 'assumed MI355X full mesh') +
    (b.measuredThroughput ? '; link throughput measured' : perGpu ? '; xGMI throughput measured per GPU, neighbour order not reported' : '');
  return (
    'xGMI topology (' + kind + ') — ' +
    (b.fullMesh ? 'full mesh, ' + m.linksPerGpu + ' links/GPU' : 'partial') +
    ' · ' + m.linksPerGpu + '×' + peak + ' GB/s per GPU · ring collectives bound at ' + m.ringBusGBs + ' GB/s per link'
  );
}

/**
 * The measured side of an xGMI matrix in one phrase — " · measured: max X,
 * mean Y GB/s over N links" when throughput sits on links, " · measured per
 * GPU: max X, mean Y GB/s over N GPUs" when only totals do, '' when nothing
 * was measured: what a closed matrix still says.
 */
export function matrixSummary(b) {
  // pages/nodes.js matrixBlock reads the statistics from the link maps; a
  // hand-made block (tests, text renderer) has only its grid.
  const st = b.linkStats !== undefined ? b.linkStats : gridLinkStats(b.matrix);
  if (st) return ' · measured: max ' + st.maxGBs.toFixed(0) + ', mean ' + st.meanGBs.toFixed(0) + ' GB/s over ' + st.links + ' links';
  const gs = b.gpuStats !== undefined ? b.gpuStats : gridGpuStats(b.matrix);
  return gs ? ' · measured per GPU: max ' + gs.maxGBs.toFixed(0) + ', mean ' + gs.meanGBs.toFixed(0) + ' GB/s over ' + gs.gpus + ' GPUs' : '';
}

const captionCache = new Map();
const summaryCache = typeof WeakMap === 'function' ? new WeakMap() : null;

/**
 * matrixCaption(b) + matrixSummary(b), the line a matrix shows open or
 * closed, formatted once per distinct content: the caption per combination
 * of its facts, the summary per statistics object (topology.js linkFacts
 * keeps one per link map). A hand-made block (no facts) is formatted as is.
 */
export function matrixLine(b) {
  if (b.linksPerGpu === undefined) return matrixCaption(b) + matrixSummary(b);
  const key = (b.measuredTopology ? 1 : 0) + (b.measuredThroughput ? 2 : 0) + (b.throughputPerGpu ? 4 : 0) + (b.fullMesh ? 8 : 0) +
    '|' + b.linksPerGpu + '|' + b.linkGBs + '|' + b.ringBusGBs;
  let caption = captionCache.get(key);
  if (caption === undefined) {
    caption = matrixCaption(b);
    captionCache.set(key, caption);
  }
  const st = b.linkStats || b.gpuStats;
  if (!st || !summaryCache) return caption + (st ? matrixSummary(b) : '');
  let summary = summaryCache.get(st);
  if (summary === undefined) {
    summary = matrixSummary(b);
    summaryCache.set(st, summary);
  }
  return caption + summary;
}

function gridLinkStats(m) {
  let n = 0;
  let sum = 0;
  let max = 0;
  for (let i = 0; i < m.size; i++) {
    for (let j = 0; j < m.size; j++) {
      const c = m.cells[i][j];
      if (c.kind !== 'xgmi' || typeof c.measuredGBs !== 'number') continue;
      n++;
      sum += c.measuredGBs;
      if (c.measuredGBs > max) max = c.measuredGBs;
    }
  }
  return n ? { links: n, meanGBs: sum / n, maxGBs: max } : null;
}

/** Per-GPU totals of a grid (its `self` cells). */
function gridGpuStats(m) {
  let n = 0;
  let sum = 0;
  let max = 0;
  for (let i = 0; i < m.size; i++) {
    const v = m.cells[i][i].measuredGBs;
    if (typeof v !== 'number') continue;
    n++;
    sum += v;
    if (v > max) max = v;
  }
  return n ? { gpus: n, meanGBs: sum / n, maxGBs: max } : null;
}

/** Text of one xGMI matrix cell: a GPU's total "Σ N" on the diagonal, GB/s on a link, else its kind. */
export function matrixCellText(c, xgmiMark) {
  if (c.kind === 'self') return c.measuredGBs !== null && c.measuredGBs !== undefined ? '\u03a3' + c.measuredGBs.toFixed(0) : '\u2014';
  return c.measuredGBs !== null ? c.measuredGBs.toFixed(0) : c.kind === 'xgmi' ? xgmiMark : c.kind;
}

/** One slot's owner as `data-slots` lists it: "namespace/pod", or "free". */
export function slotOwner(s) {
  return s.pod ? (s.namespace ? s.namespace + '/' : '') + s.pod : 'free';
}

/** slotOwner(a) === slotOwner(b), without building the strings. */
function sameOwner(a, b) {
  if (!a.pod || !b.pod) return !a.pod && !b.pod;
  return a.pod === b.pod && (a.namespace || '') === (b.namespace || '');
}

function slotLabel(s) {
  return s.partition === null || s.partition === undefined ? String(s.index) : s.board + '·' + s.partition;
}

/**
 * A slot strip's owners in runs: "GPU 0–3 ml/train-a · GPU 4 free · …"
 * (consecutive slots of one owner fold into one run).
 */
export function slotsText(slots) {
  // Runs compare the owners' fields (no owner string per slot: a strip is
  // drawn per GPU node card on every mount).
  let out = '';
  for (let i = 0; i < slots.length;) {
    const from = slots[i];
    let j = i + 1;
    while (j < slots.length && sameOwner(slots[j], from)) j++;
    const a = slotLabel(from);
    out += (i ? ' · GPU ' : 'GPU ') + (j - 1 === i ? a : a + '–' + slotLabel(slots[j - 1])) + ' ' + slotOwner(from);
    i = j;
  }
  return out;
}

// ---------------------------------------------------------------------------
// Query helpers (tests, benchmark row counting)
// ---------------------------------------------------------------------------

export function sections(vm) {
  const out = [];
  if (!vm) return out;
  const items = vm.t === 'section' ? [vm] : vm.items || [];
  for (let i = 0; i < items.length; i++) if (items[i].t === 'section') out.push(items[i]);
  return out;
}

export function sectionTitles(vm) {
  return sections(vm).map(function (s) { return s.title; });
}

export function findSection(vm, title) {
  const ss = sections(vm);
  for (let i = 0; i < ss.length; i++) if (ss[i].title === title) return ss[i];
  return null;
}

/** The page's pager item, or null. */
export function pagerOf(vm) {
  if (!vm || !vm.items) return null;
  for (let i = 0; i < vm.items.length; i++) if (vm.items[i].t === 'pager') return vm.items[i];
  return null;
}

export function loaders(vm) {
  if (!vm || !vm.items) return [];
  return vm.items.filter(function (i) { return i.t === 'loader'; }).map(function (i) { return i.title; });
}

/** Value of the first kv row named `name` in a section (or whole page). */
export function rowValue(scope, name) {
  const ss = scope && scope.t === 'page' ? sections(scope) : [scope];
  for (let s = 0; s < ss.length; s++) {
    if (!ss[s]) continue;
    const blocks = ss[s].blocks || [];
    for (let b = 0; b < blocks.length; b++) {
      if (blocks[b].t !== 'kv') continue;
      const rows = blocks[b].rows;
      for (let r = 0; r < rows.length; r++) if (rows[r].name === name) return rows[r].value;
    }
  }
  return undefined;
}

export function rowNames(sec) {
  const out = [];
  if (!sec) return out;
  for (let b = 0; b < sec.blocks.length; b++) {
    if (sec.blocks[b].t !== 'kv') continue;
    for (let r = 0; r < sec.blocks[b].rows.length; r++) out.push(sec.blocks[b].rows[r].name);
  }
  return out;
}

export function firstTable(sec) {
  if (!sec) return null;
  for (let b = 0; b < sec.blocks.length; b++) if (sec.blocks[b].t === 'table') return sec.blocks[b];
  return null;
}

export function firstBlock(sec, t) {
  if (!sec) return null;
  for (let b = 0; b < sec.blocks.length; b++) if (sec.blocks[b].t === t) return sec.blocks[b];
  return null;
}

/** Plain text of a cell value. */
export function text(v) {
  if (v === null || v === undefined) return '';
  if (typeof v === 'string' || typeof v === 'number') return String(v);
  if (v.t === 'status') return v.text;
  if (v.t === 'bar') return v.text;
  if (v.t === 'lines') return v.lines.map(function (l) { return l.label ? l.label + ': ' + l.text : l.text; }).join('\n');
  return '';
}

/**
 * Count what a page renders: table rows, name/value rows, sections, and
 * per-GPU cells. This is the "rows rendered" half of the benchmark metric.
 */
export function countRows(vm) {
  const c = { sections: 0, tableRows: 0, kvRows: 0, gpuCells: 0 };
  const ss = sections(vm);
  for (let s = 0; s < ss.length; s++) {
    c.sections++;
    const blocks = ss[s].blocks;
    for (let b = 0; b < blocks.length; b++) {
      const bl = blocks[b];
      if (bl.t === 'table') c.tableRows += bl.rows.length;
      else if (bl.t === 'kv') c.kvRows += bl.rows.length;
      else if (bl.t === 'slots') c.gpuCells += bl.slots.length;
      else if (bl.t === 'matrix') c.gpuCells += bl.matrix.size * bl.matrix.size;
    }
  }
  return c;
}
