/**
 * Plugin settings — validated, persisted, framework-free.
 *
 * The reference has no runtime configuration: its Prometheus namespace /
 * service / port, request timeout and rate window are compile-time constants
 * (SURVEY.md §5 "Config / flag system: absent"; reference
 * src/api/metrics.ts:61-65, IntelGpuDataContext.tsx:72). Here they are user
 * settings, stored in the browser (localStorage) and edited on Headlamp's
 * plugin settings page (src/components/SettingsPage.tsx).
 *
 * Every value read back is re-validated: a corrupted or hand-edited entry
 * falls back to the defaults field by field instead of breaking the plugin.
 */

import { PROMETHEUS_SERVICES } from './series.js';
import { isObject } from './k8sCore.js';

export const SETTINGS_KEY = 'headlamp-amd-gpu-plugin.settings';

export const REFRESH_CHOICES = [0, 15, 30, 60, 300];

export const DEFAULT_SETTINGS = Object.freeze({
  /** Explicit Prometheus service, tried before the built-in candidates. */
  prometheus: null,
  /** Auto-refresh period in seconds (0 = manual refresh only, like the reference). */
  refreshIntervalSec: 0,
  /** Per-request timeout for the CRD / pod / discovery requests. */
  requestTimeoutMs: 2000,
  /** Time-series window on the Metrics page. */
  seriesMinutes: 30,
});

const DNS_LABEL = /^[a-z0-9]([-a-z0-9]*[a-z0-9])?$/;

function clampInt(v, lo, hi, dflt) {
  const n = typeof v === 'number' ? v : parseInt(String(v), 10);
  if (!isFinite(n)) return dflt;
  return Math.min(hi, Math.max(lo, Math.round(n)));
}

/** Validate a {namespace, service, port} triple; null when incomplete or invalid. */
export function parsePrometheus(v) {
  if (!isObject(v)) return null;
  const ns = String(v.namespace || '').trim();
  const svc = String(v.service || '').trim();
  const port = String(v.port || '').trim();
  if (!DNS_LABEL.test(ns) || !DNS_LABEL.test(svc)) return null;
  if (!/^([0-9]{1,5}|[a-z][-a-z0-9]{0,14})$/.test(port)) return null;
  return { namespace: ns, service: svc, port: port };
}

/**
 * Unknown → settings, field by field, with defaults for anything invalid.
 * @returns {{prometheus: ({namespace: string, service: string, port: string}|null), refreshIntervalSec: number,
 *            requestTimeoutMs: number, seriesMinutes: number}}
 */
export function parseSettings(raw) {
  const o = isObject(raw) ? raw : {};
  const refresh = clampInt(o.refreshIntervalSec, 0, 3600, DEFAULT_SETTINGS.refreshIntervalSec);
  return {
    prometheus: parsePrometheus(o.prometheus),
    refreshIntervalSec: refresh > 0 && refresh < 5 ? 5 : refresh,
    requestTimeoutMs: clampInt(o.requestTimeoutMs, 250, 30000, DEFAULT_SETTINGS.requestTimeoutMs),
    seriesMinutes: clampInt(o.seriesMinutes, 5, 24 * 60, DEFAULT_SETTINGS.seriesMinutes),
  };
}

/** Prometheus candidates in priority order: the configured service first, then the defaults. */
export function prometheusCandidates(settings) {
  const out = [];
  const p = settings && settings.prometheus;
  if (p) out.push(p);
  for (let i = 0; i < PROMETHEUS_SERVICES.length; i++) {
    const d = PROMETHEUS_SERVICES[i];
    if (!p || d.namespace !== p.namespace || d.service !== p.service || d.port !== p.port) out.push(d);
  }
  return out;
}

/** Range-query step that keeps the series near 60 points. */
export function seriesStepSec(settings) {
  return Math.max(15, Math.round((settings.seriesMinutes * 60) / 60 / 15) * 15);
}

function defaultStorage() {
  try {
    if (typeof localStorage !== 'undefined' && localStorage && typeof localStorage.getItem === 'function') return localStorage;
  } catch (e) {
    // storage disabled (privacy mode): settings stay in memory
  }
  return null;
}

function readSettings(st) {
  if (!st) return parseSettings(null);
  try {
    const raw = st.getItem(SETTINGS_KEY);
    return parseSettings(raw ? JSON.parse(raw) : null);
  } catch (e) {
    return parseSettings(null);
  }
}

// Memo of the browser-storage read. Every hook of every render asks for the
// settings (providerCore.js); parsing localStorage JSON each time is wasted
// work, so the parsed value is kept until `saveSettings` writes a new one or
// another tab changes the key (the `storage` event).
let settingsVersion = 0;
let memo = null; // {version, value}
let storageListener = false;

/** `storage` event handler: another tab wrote the settings key (or cleared storage, key null). */
export function onStorageEvent(e) {
  if (!e || e.key === null || e.key === undefined || e.key === SETTINGS_KEY) invalidateSettings();
}

function listenForStorage() {
  if (storageListener) return;
  if (typeof window === 'undefined' || !window || typeof window.addEventListener !== 'function') return;
  storageListener = true;
  window.addEventListener('storage', onStorageEvent);
}

/** Drop the memoised settings; the next `loadSettings()` reads storage again. */
export function invalidateSettings() {
  settingsVersion++;
  memo = null;
}

/** Memo generation (tests): bumped by `saveSettings` and by `storage` events. */
export function settingsGeneration() {
  return settingsVersion;
}

/**
 * Read settings from storage (defaults when absent or unreadable). With the
 * default storage the parsed value is memoised (a frozen object, the same one
 * until invalidated); an explicit `storage` argument always reads it.
 */
export function loadSettings(storage) {
  if (storage !== undefined) return readSettings(storage);
  listenForStorage();
  if (memo && memo.version === settingsVersion) return memo.value;
  const value = Object.freeze(readSettings(defaultStorage()));
  if (value.prometheus) Object.freeze(value.prometheus);
  memo = { version: settingsVersion, value: value };
  return value;
}

/** Validate and persist; returns what was stored. */
export function saveSettings(value, storage) {
  const clean = parseSettings(value);
  const st = storage === undefined ? defaultStorage() : storage;
  if (st) {
    try {
      st.setItem(SETTINGS_KEY, JSON.stringify(clean));
    } catch (e) {
      // quota / disabled storage: keep the in-memory value
    }
  }
  if (storage === undefined) {
    invalidateSettings();
    // Storage refused the write (disabled / quota): the memo still serves the
    // value just saved, as the comment above promises.
    if (!st) memo = { version: settingsVersion, value: Object.freeze(Object.assign({}, clean)) };
  }
  return clean;
}

/** Key prefix of a page's view state (pager page / filter / order), per browser tab. */
export const VIEW_STATE_KEY = 'headlamp-amd-gpu-plugin.view.';

function defaultSessionStorage() {
  try {
    if (typeof sessionStorage !== 'undefined' && sessionStorage && typeof sessionStorage.getItem === 'function') return sessionStorage;
  } catch (e) {
    // storage disabled: the view state lives as long as the page
  }
  return null;
}

/**
 * A paged page's view state saved in this tab's session ({page, filter,
 * sort}), so leaving a page and coming back (Headlamp unmounts it) keeps the
 * reader's place; null when nothing (valid) is stored. `storage` defaults to
 * sessionStorage.
 */
export function loadViewState(key, storage) {
  const st = storage === undefined ? defaultSessionStorage() : storage;
  if (!st) return null;
  try {
    const v = JSON.parse(st.getItem(VIEW_STATE_KEY + key) || 'null');
    if (!v || typeof v !== 'object') return null;
    return {
      page: typeof v.page === 'number' && v.page >= 0 && Math.floor(v.page) === v.page ? v.page : 0,
      filter: typeof v.filter === 'string' ? v.filter.slice(0, 200) : '',
      sort: typeof v.sort === 'string' ? v.sort.slice(0, 40) : 'name',
    };
  } catch (e) {
    return null;
  }
}

/** Persist a page's view state for this tab (see loadViewState); write errors are ignored. */
export function saveViewState(key, value, storage) {
  const st = storage === undefined ? defaultSessionStorage() : storage;
  if (!st) return;
  try {
    st.setItem(VIEW_STATE_KEY + key, JSON.stringify({ page: value.page, filter: value.filter, sort: value.sort }));
  } catch (e) {
    // quota / disabled storage
  }
}

/**
 * Interval poller with an injectable clock. `start(fn)` calls fn every
 * `periodSec` seconds, skipping a tick while the previous call's promise is
 * still pending (no overlapping refreshes), and while the browser tab is
 * hidden (an auto-refreshing dashboard left in a background tab would keep
 * querying the apiserver and Prometheus for nobody). When the tab is shown
 * again after a skipped tick, the refresh runs at once instead of up to one
 * period later. When `fn` resolves to POLL_MISS (its target did not answer)
 * the poller backs off: it skips the next 1, 2, 4, then at most
 * MAX_MISS_SKIPS ticks, until a call succeeds again. Period 0 → never.
 */
export const POLL_MISS = 'miss';
export const MAX_MISS_SKIPS = 8;

export function createPoller(periodSec, clock) {
  const c = clock || { setInterval: setInterval, clearInterval: clearInterval };
  const hidden = typeof c.hidden === 'function' ? c.hidden : documentHidden;
  const onVisible = typeof c.onVisible === 'function' ? c.onVisible : documentOnVisible;
  let handle = null;
  let unsubscribe = null;
  let busy = false;
  let missed = false;
  let ticks = 0;
  let skipped = 0;
  let hiddenSkips = 0;
  let backoff = 0; // ticks to skip after each consecutive miss
  let skipLeft = 0;
  let missSkips = 0;
  function tick(fn) {
    if (busy) {
      skipped++;
      return;
    }
    if (skipLeft > 0) {
      skipLeft--;
      missSkips++;
      return;
    }
    if (hidden()) {
      hiddenSkips++;
      missed = true;
      return;
    }
    missed = false;
    busy = true;
    ticks++;
    Promise.resolve()
      .then(fn)
      .then(
        function (r) {
          busy = false;
          if (r === POLL_MISS) {
            backoff = backoff ? Math.min(backoff * 2, MAX_MISS_SKIPS) : 1;
            skipLeft = backoff;
          } else {
            backoff = 0;
            skipLeft = 0;
          }
        },
        function () { busy = false; }
      );
  }
  return {
    start: function (fn) {
      if (handle !== null || !(periodSec > 0)) return;
      handle = c.setInterval(function () { tick(fn); }, periodSec * 1000);
      unsubscribe = onVisible(function () {
        if (handle !== null && missed) tick(fn);
      });
    },
    stop: function () {
      if (handle !== null) c.clearInterval(handle);
      handle = null;
      if (unsubscribe) unsubscribe();
      unsubscribe = null;
    },
    stats: function () {
      return { ticks: ticks, skipped: skipped, hiddenSkips: hiddenSkips, missSkips: missSkips, running: handle !== null };
    },
  };
}

/** True in a browser tab that is not visible; false outside a browser (the terminal dashboard). */
function documentHidden() {
  return typeof document !== 'undefined' && !!document && document.visibilityState === 'hidden';
}

/** Calls `cb` when the tab becomes visible; returns the unsubscribe. A no-op outside a browser. */
function documentOnVisible(cb) {
  if (typeof document === 'undefined' || !document || typeof document.addEventListener !== 'function') {
    return function () {};
  }
  const listener = function () {
    if (document.visibilityState !== 'hidden') cb();
  };
  document.addEventListener('visibilitychange', listener);
  return function () { document.removeEventListener('visibilitychange', listener); };
}
