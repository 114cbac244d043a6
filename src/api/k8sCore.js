/**
 * The AMD constants (resource names, CRD, labels, operator namespace,
 * MI355X platform facts), the generic Kubernetes helpers every model module
 * uses, the list envelope, the 70/90 % thresholds and the formatters.
 * Pure, I/O-free, ES2019.
 *
 * Reference: src/api/k8s.ts:13-31 (constants, C2.1), :315-323 (list
 * envelope, C2.12), :337-364 (formatters, C2.14).
 */

// Constants
// ---------------------------------------------------------------------------

/** AMD GPU Operator CRD (verify: amd.com/v1alpha1 DeviceConfig, namespaced). */
export const AMD_GPU_OPERATOR_API_GROUP = 'amd.com';

export const AMD_GPU_OPERATOR_API_VERSION = 'v1alpha1';

export const DEVICE_CONFIG_KIND = 'DeviceConfig';

export const DEVICE_CONFIG_PLURAL = 'deviceconfigs';

export const DEVICE_CONFIG_LIST_PATH =
  '/apis/' + AMD_GPU_OPERATOR_API_GROUP + '/' + AMD_GPU_OPERATOR_API_VERSION + '/' + DEVICE_CONFIG_PLURAL;

/** Whole-GPU extended resource advertised by the AMD k8s device plugin. */
export const AMD_GPU_RESOURCE = 'amd.com/gpu';

/** Every AMD extended resource shares this prefix (partition resources too). */
export const AMD_RESOURCE_PREFIX = 'amd.com/';

/**
 * Partition resources exposed with the device plugin's "mixed" naming
 * strategy, e.g. `amd.com/cpx_nps4` (verify per operator release).
 */
export const AMD_PARTITION_RESOURCE_RE = /^amd\.com\/(spx|dpx|qpx|cpx)_(nps[1-8])$/;

/** Label set by the GPU Operator's Node Feature Discovery rule. */
export const AMD_NFD_GPU_LABEL = 'feature.node.kubernetes.io/amd-gpu';

/** Node-labeller labels (verify: `amd.com/gpu.<prop>`, legacy `beta.amd.com/gpu.<prop>`). */
export const AMD_LABELLER_PREFIX = 'amd.com/gpu.';

export const AMD_LABELLER_LEGACY_PREFIX = 'beta.amd.com/gpu.';

export const LABEL_PRODUCT_NAME = 'amd.com/gpu.product-name';

export const LABEL_FAMILY = 'amd.com/gpu.family';

export const LABEL_DEVICE_ID = 'amd.com/gpu.device-id';

export const LABEL_VRAM = 'amd.com/gpu.vram';

export const LABEL_CU_COUNT = 'amd.com/gpu.cu-count';

export const LABEL_DRIVER_VERSION = 'amd.com/gpu.driver-version';

export const LABEL_COMPUTE_PARTITION = 'amd.com/compute-partitioning-mode';

export const LABEL_MEMORY_PARTITION = 'amd.com/memory-partitioning-mode';

/** Namespace the AMD GPU Operator deploys its operands into (verify). */
export const AMD_GPU_OPERATOR_NAMESPACE = 'kube-amd-gpu';

/** `name=` pod labels of the standalone k8s-device-plugin DaemonSets (verify). */
export const AMD_DEVICE_PLUGIN_POD_LABEL = 'amdgpu-dp-ds';

export const AMD_NODE_LABELLER_POD_LABEL = 'amdgpu-labeller-ds';

/**
 * Plugin-pod discovery requests. Issued in PARALLEL by the data layer
 * (the reference issues its three selectors serially,
 * src/api/IntelGpuDataContext.tsx:155-165). One set-based selector replaces
 * two equality selectors, and it leaves out the operator namespace, which the
 * second request lists whole: the two answers are disjoint, so on a large
 * cluster (two or three operand pods per GPU node) no pod is sent twice.
 */
export const PLUGIN_POD_LABEL_SELECTOR = 'name in (' + AMD_DEVICE_PLUGIN_POD_LABEL + ',' + AMD_NODE_LABELLER_POD_LABEL + ')';
export const PLUGIN_POD_FIELD_SELECTOR = 'metadata.namespace!=' + AMD_GPU_OPERATOR_NAMESPACE;

export const PLUGIN_POD_QUERIES = [
  '/api/v1/pods?labelSelector=' + encodeURIComponent(PLUGIN_POD_LABEL_SELECTOR) +
    '&fieldSelector=' + encodeURIComponent(PLUGIN_POD_FIELD_SELECTOR),
  '/api/v1/namespaces/' + AMD_GPU_OPERATOR_NAMESPACE + '/pods',
];

/**
 * The same two selections as list + watch options of Headlamp's
 * `Pod.useList()` (providerCore.js OperatorPodFeed), in PLUGIN_POD_QUERIES
 * order: what the Device Plugins route watches instead of every pod of the
 * cluster. A host whose `useList` does not apply these options delivers
 * objects outside them: the feed counts those (selectors.js countOutside),
 * and the provider swaps the watches for the scoped requests (ADR 012).
 */
export const OPERATOR_POD_LISTS = Object.freeze([
  Object.freeze({ namespace: '', labelSelector: PLUGIN_POD_LABEL_SELECTOR, fieldSelector: PLUGIN_POD_FIELD_SELECTOR }),
  Object.freeze({ namespace: AMD_GPU_OPERATOR_NAMESPACE }),
]);

/** MI355X platform facts (MI355X_MICROARCH.md chip-level table). */
export const MI355X = Object.freeze({
  product: 'AMD Instinct MI355X',
  shortName: 'MI355X',
  arch: 'gfx950 (CDNA4)',
  hbmBytes: 294896 * 1024 * 1024, // 288 GiB HBM3E less 16 MiB: what the device reports (amd-smi total_vram 294896 MB)
  hbmLabel: '288 GB HBM3E',
  hbmPeakTBs: 8.0,
  computeUnits: 256,
  xcds: 8,
  gpusPerNode: 8,
  xgmiLinksPerGpu: 7,
  xgmiLinkGBs: 153,
  tdpWatts: 1400,
  // Junction (hotspot) throttle threshold: amd-smi slowdown_hotspot_temperature
  // on an MI355X (tests/fixtures/mi355x/amd_smi_static.json).
  junctionSlowdownC: 100,
});

/** Allocation / power colour thresholds (reference NodesPage.tsx:38, MetricsPage.tsx:52-53). */
export const WARN_PCT = 70;

export const ERROR_PCT = 90;

/** @param {unknown} v @returns {v is Record<string, unknown>} */
export function isObject(v) {
  return v !== null && typeof v === 'object' && !Array.isArray(v);
}

const optString = function (v) { return v === undefined || v === null || typeof v === 'string'; };

/**
 * A Kubernetes object the views can name: metadata with a non-empty string
 * name, and a namespace / uid that are strings when present. What fails this
 * (a half-written object, a wrong-shaped watch event) is never classified as
 * a GPU node, GPU pod, operator pod or DeviceConfig, so no page renders its
 * name — a view never hands React an object where it expects text.
 */
export function isNamedObject(v) {
  if (!isObject(v) || !isObject(v.metadata)) return false;
  const m = v.metadata;
  return typeof m.name === 'string' && m.name !== '' && optString(m.namespace) && optString(m.uid);
}

/** Safe nested getter: get(obj, ['a','b']) without optional chaining. */
export function get(obj, path, dflt) {
  let cur = obj;
  for (let i = 0; i < path.length; i++) {
    if (cur === null || cur === undefined || typeof cur !== 'object') return dflt;
    cur = cur[path[i]];
  }
  return cur === undefined || cur === null ? dflt : cur;
}

/** Parse a Kubernetes integer quantity ("8", "8k" is not valid for devices). */
export function parseCount(v) {
  if (v === undefined || v === null) return 0;
  const n = parseInt(String(v), 10);
  return isFinite(n) && n > 0 ? n : 0;
}

/** Headlamp `useList()` returns KubeObject wrappers that keep raw JSON in `.jsonData`. */
export function unwrapKubeObject(item) {
  if (item && typeof item === 'object' && 'jsonData' in item && item.jsonData && typeof item.jsonData === 'object') {
    return item.jsonData;
  }
  return item;
}

export function unwrapAll(items) {
  if (!Array.isArray(items)) return [];
  const out = new Array(items.length);
  for (let i = 0; i < items.length; i++) out[i] = unwrapKubeObject(items[i]);
  return out;
}

export function labelsOf(obj) {
  const l = get(obj, ['metadata', 'labels'], null);
  return isObject(l) ? l : {};
}

/** @returns {boolean} true for `{ items: [...] }` list responses. */
export function isKubeList(value) {
  return isObject(value) && Array.isArray(value.items);
}

/** Rounded percentage, 0 when the denominator is 0. */
export function pct(used, total) {
  if (!(total > 0)) return 0;
  return Math.round((used / total) * 100);
}

/** success <70 %, warning ≥70 %, error ≥90 %. */
export function pctToStatus(p) {
  if (p >= ERROR_PCT) return 'error';
  if (p >= WARN_PCT) return 'warning';
  return 'success';
}

/** Bar colours matching the thresholds (AMD red for healthy "in use"). */
export const BAR_COLORS = { ok: '#ed1c24', okInferred: '#f27478', warn: '#f57c00', err: '#d32f2f', track: '#e0e0e0', mute: '#9e9e9e' };

export function pctToColor(p) {
  if (p >= ERROR_PCT) return BAR_COLORS.err;
  if (p >= WARN_PCT) return BAR_COLORS.warn;
  return BAR_COLORS.ok;
}

/** Age as Ns / Nm / Nh / Nd (reference k8s.ts:337-348 semantics). `now` is injectable for tests. */
const timeCache = new Map();

/** Epoch ms of an RFC 3339 timestamp (NaN when unparseable); parsed once per string. */
export function parseTime(timestamp) {
  let t = timeCache.get(timestamp);
  if (t === undefined) {
    t = new Date(timestamp).getTime();
    if (timeCache.size > 65536) timeCache.clear();
    timeCache.set(timestamp, t);
  }
  return t;
}

/**
 * The instant (epoch ms) at which `formatAge(timestamp, now)` next shows a
 * different label: the next whole second, minute, hour or day of age
 * (Infinity when the label never changes).
 */
export function nextAgeChange(timestamp, now) {
  if (!timestamp) return Infinity;
  const t = parseTime(timestamp);
  if (!isFinite(t)) return Infinity;
  const n = now === undefined ? Date.now() : now;
  const secs = Math.max(0, Math.floor((n - t) / 1000));
  if (secs < 60) return t + (secs + 1) * 1000;
  const mins = Math.floor(secs / 60);
  if (mins < 60) return t + (mins + 1) * 60000;
  const hours = Math.floor(mins / 60);
  if (hours < 24) return t + (hours + 1) * 3600000;
  return t + (Math.floor(hours / 24) + 1) * 86400000;
}

export function formatAge(timestamp, now) {
  if (!timestamp) return 'unknown';
  const t = parseTime(timestamp);
  if (!isFinite(t)) return 'unknown';
  const diffMs = (now === undefined ? Date.now() : now) - t;
  const secs = Math.max(0, Math.floor(diffMs / 1000));
  if (secs < 60) return secs + 's';
  const mins = Math.floor(secs / 60);
  if (mins < 60) return mins + 'm';
  const hours = Math.floor(mins / 60);
  if (hours < 24) return hours + 'h';
  return Math.floor(hours / 24) + 'd';
}

/** Display name for an AMD extended resource key. */
export function formatGpuResourceName(key) {
  if (key === AMD_GPU_RESOURCE) return 'GPU';
  const m = AMD_PARTITION_RESOURCE_RE.exec(key);
  if (m) return 'GPU partition (' + m[1].toUpperCase() + '/' + m[2].toUpperCase() + ')';
  return key.indexOf(AMD_RESOURCE_PREFIX) === 0 ? key.slice(AMD_RESOURCE_PREFIX.length) : key;
}

/**
 * Bytes → "288 GiB" / "2.3 TiB". Binary units: the MI355X's "288 GB" of HBM3E
 * is 288 GiB (measured on the device), and the exporter reports MiB.
 */
const BYTE_UNITS = ['B', 'KiB', 'MiB', 'GiB', 'TiB', 'PiB'];

export function formatBytes(b) {
  if (!(b >= 0) || b === null) return '—';
  let v = b;
  let u = 0;
  while (v >= 1024 && u < BYTE_UNITS.length - 1) {
    v /= 1024;
    u++;
  }
  // Three significant digits, trailing zeros dropped: "288 GiB", "2.25 TiB", "4.5 TiB".
  const digits = v >= 100 || u === 0 ? 0 : v >= 10 ? 1 : 2;
  let t = v.toFixed(digits);
  if (digits > 0) {
    let end = t.length;
    while (t.charCodeAt(end - 1) === 48) end--; // '0'
    if (t.charCodeAt(end - 1) === 46) end--; // '.'
    t = t.slice(0, end);
  }
  return t + ' ' + BYTE_UNITS[u];
}

/** Watts with one decimal, as `toFixed(1)` writes them (whole watts, the usual reading, without the call). */
export function formatWatts(w) {
  return (Number.isSafeInteger(w) ? w + '.0' : w.toFixed(1)) + ' W';
}

export function formatPercent(used, max) {
  if (!(max > 0)) return '—';
  return Math.round((used / max) * 100) + '%';
}
