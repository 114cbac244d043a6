/**
 * Settings subsystem (src/api/settings.js) — new: the reference has no
 * runtime configuration (SURVEY.md §5).
 */
import {
  DEFAULT_SETTINGS,
  SETTINGS_KEY,
  MAX_MISS_SKIPS,
  POLL_MISS,
  createPoller,
  invalidateSettings,
  loadSettings,
  onStorageEvent,
  settingsGeneration,
  parsePrometheus,
  parseSettings,
  prometheusCandidates,
  saveSettings,
  seriesStepSec,
} from '../../src/api/settings.js';
import { PROMETHEUS_SERVICES } from '../../src/api/series.js';

function memStorage() {
  const m = new Map();
  return {
    getItem: (k) => (m.has(k) ? m.get(k) : null),
    setItem: (k, v) => m.set(k, String(v)),
    raw: m,
  };
}

describe('parseSettings', () => {
  it('returns the defaults for garbage', () => {
    expect(parseSettings(null)).toEqual(Object.assign({}, DEFAULT_SETTINGS));
    expect(parseSettings('x')).toEqual(Object.assign({}, DEFAULT_SETTINGS));
  });
  it('clamps numbers field by field', () => {
    const s = parseSettings({ refreshIntervalSec: 2, requestTimeoutMs: 10, seriesMinutes: 100000 });
    expect(s.refreshIntervalSec).toBe(5);
    expect(s.requestTimeoutMs).toBe(250);
    expect(s.seriesMinutes).toBe(1440);
  });
  it('keeps valid values and parses numeric strings', () => {
    const s = parseSettings({ refreshIntervalSec: '30', requestTimeoutMs: 5000, seriesMinutes: 60 });
    expect(s).toEqual({ prometheus: null, refreshIntervalSec: 30, requestTimeoutMs: 5000, seriesMinutes: 60 });
  });
  it('zero refresh interval means manual', () => {
    expect(parseSettings({ refreshIntervalSec: 0 }).refreshIntervalSec).toBe(0);
  });
});

describe('parsePrometheus', () => {
  it('accepts DNS-label names and numeric or named ports', () => {
    expect(parsePrometheus({ namespace: 'obs', service: 'vmsingle', port: '8429' })).toEqual({ namespace: 'obs', service: 'vmsingle', port: '8429' });
    expect(parsePrometheus({ namespace: 'obs', service: 'prom', port: 'web' })).not.toBeNull();
  });
  it('rejects path tricks and incomplete triples', () => {
    expect(parsePrometheus({ namespace: '../x', service: 'p', port: '9090' })).toBeNull();
    expect(parsePrometheus({ namespace: 'a', service: 'p/../q', port: '9090' })).toBeNull();
    expect(parsePrometheus({ namespace: 'a', service: 'p' })).toBeNull();
    expect(parsePrometheus(null)).toBeNull();
  });
});

describe('prometheusCandidates', () => {
  it('defaults to the built-in services', () => {
    expect(prometheusCandidates(parseSettings(null))).toEqual(PROMETHEUS_SERVICES);
  });
  it('puts the configured service first without duplicating it', () => {
    const own = { namespace: 'monitoring', service: 'prometheus-operated', port: '9090' };
    const c = prometheusCandidates(parseSettings({ prometheus: own }));
    expect(c[0]).toEqual(own);
    expect(c).toHaveLength(PROMETHEUS_SERVICES.length);
  });
});

describe('persistence', () => {
  it('round-trips through storage with validation', () => {
    const st = memStorage();
    saveSettings({ refreshIntervalSec: 60, prometheus: { namespace: 'o', service: 's', port: '1' } }, st);
    expect(JSON.parse(st.raw.get(SETTINGS_KEY)).refreshIntervalSec).toBe(60);
    expect(loadSettings(st).prometheus).toEqual({ namespace: 'o', service: 's', port: '1' });
  });
  it('survives corrupted storage', () => {
    const st = memStorage();
    st.setItem(SETTINGS_KEY, '{not json');
    expect(loadSettings(st)).toEqual(Object.assign({}, DEFAULT_SETTINGS));
  });
  it('works without storage', () => {
    expect(loadSettings(null).requestTimeoutMs).toBe(2000);
    expect(saveSettings({ seriesMinutes: 10 }, null).seriesMinutes).toBe(10);
  });
});

describe('loadSettings memo (browser storage)', () => {
  let saved;
  let reads;
  let listeners;
  beforeEach(() => {
    saved = { ls: global.localStorage, win: global.window };
    const st = memStorage();
    reads = 0;
    const get = st.getItem;
    st.getItem = (k) => {
      reads++;
      return get(k);
    };
    listeners = [];
    global.localStorage = st;
    if (!saved.win) global.window = { addEventListener: (type, fn) => listeners.push({ type: type, fn: fn }) };
    invalidateSettings();
  });
  afterEach(() => {
    if (saved.ls === undefined) delete global.localStorage;
    else global.localStorage = saved.ls;
    if (saved.win === undefined) delete global.window;
    invalidateSettings();
  });

  it('parses storage once and hands every caller the same frozen object', () => {
    const a = loadSettings();
    const b = loadSettings();
    expect(reads).toBe(1);
    expect(a).toBe(b);
    expect(Object.isFrozen(a)).toBe(true);
  });
  it('saveSettings invalidates the memo', () => {
    const before = loadSettings();
    const g = settingsGeneration();
    saveSettings({ refreshIntervalSec: 30 });
    expect(settingsGeneration()).toBeGreaterThan(g);
    const after = loadSettings();
    expect(after).not.toBe(before);
    expect(after.refreshIntervalSec).toBe(30);
    expect(reads).toBe(2);
  });
  it('a storage event for the settings key (or a clear) invalidates it; other keys do not', () => {
    loadSettings();
    onStorageEvent({ key: 'some-other-plugin' });
    loadSettings();
    expect(reads).toBe(1);
    global.localStorage.setItem(SETTINGS_KEY, JSON.stringify({ seriesMinutes: 60 }));
    onStorageEvent({ key: SETTINGS_KEY });
    expect(loadSettings().seriesMinutes).toBe(60);
    onStorageEvent({ key: null });
    loadSettings();
    expect(reads).toBe(3);
  });
  it('registers the storage listener on the window when one exists', () => {
    loadSettings();
    if (saved.win) return; // a real DOM window: registration happened on its own object
    // the module attaches once per process; a runner sharing modules across files may have attached earlier
    if (listeners.length) {
      expect(listeners[0].type).toBe('storage');
      expect(listeners[0].fn).toBe(onStorageEvent);
    }
  });
  it('explicit storage bypasses the memo', () => {
    const st = memStorage();
    st.setItem(SETTINGS_KEY, JSON.stringify({ requestTimeoutMs: 900 }));
    loadSettings();
    expect(loadSettings(st).requestTimeoutMs).toBe(900);
    expect(loadSettings().requestTimeoutMs).toBe(2000);
  });
});

describe('seriesStepSec', () => {
  it('keeps about 60 points on a 15 s grid', () => {
    expect(seriesStepSec(parseSettings({ seriesMinutes: 30 }))).toBe(30);
    expect(seriesStepSec(parseSettings({ seriesMinutes: 5 }))).toBe(15);
    expect(seriesStepSec(parseSettings({ seriesMinutes: 360 }))).toBe(360);
  });
});

describe('createPoller', () => {
  it('ticks every period and stops', async () => {
    vi.useFakeTimers();
    const fn = vi.fn(() => Promise.resolve());
    const p = createPoller(30);
    p.start(fn);
    await vi.advanceTimersByTimeAsync(95000);
    expect(fn).toHaveBeenCalledTimes(3);
    p.stop();
    await vi.advanceTimersByTimeAsync(60000);
    expect(fn).toHaveBeenCalledTimes(3);
    expect(p.stats().running).toBe(false);
    vi.useRealTimers();
  });
  it('skips ticks while a refresh is still running', async () => {
    vi.useFakeTimers();
    let release;
    const fn = vi.fn(() => new Promise((r) => { release = r; }));
    const p = createPoller(10);
    p.start(fn);
    await vi.advanceTimersByTimeAsync(35000);
    expect(fn).toHaveBeenCalledTimes(1);
    expect(p.stats().skipped).toBe(2);
    release();
    await vi.advanceTimersByTimeAsync(10000);
    expect(fn).toHaveBeenCalledTimes(2);
    p.stop();
    vi.useRealTimers();
  });
  it('skips ticks while the tab is hidden and resumes when it is shown', async () => {
    vi.useFakeTimers();
    let hidden = false;
    const fn = vi.fn(() => Promise.resolve());
    const p = createPoller(10, { setInterval, clearInterval, hidden: () => hidden });
    p.start(fn);
    await vi.advanceTimersByTimeAsync(10000);
    expect(fn).toHaveBeenCalledTimes(1);
    hidden = true;
    await vi.advanceTimersByTimeAsync(30000);
    expect(fn).toHaveBeenCalledTimes(1);
    expect(p.stats().hiddenSkips).toBe(3);
    hidden = false;
    await vi.advanceTimersByTimeAsync(10000);
    expect(fn).toHaveBeenCalledTimes(2);
    p.stop();
    vi.useRealTimers();
  });
  it('refreshes at once when the tab is shown after a skipped tick, and unsubscribes on stop', async () => {
    vi.useFakeTimers();
    let hidden = true;
    const listeners = new Set();
    const clock = {
      setInterval,
      clearInterval,
      hidden: () => hidden,
      onVisible: (cb) => {
        listeners.add(cb);
        return () => listeners.delete(cb);
      },
    };
    const fn = vi.fn(() => Promise.resolve());
    const p = createPoller(60, clock);
    p.start(fn);
    hidden = false;
    listeners.forEach((cb) => cb());
    expect(fn).not.toHaveBeenCalled(); // shown before any tick was missed: nothing is stale
    hidden = true;
    await vi.advanceTimersByTimeAsync(60000);
    expect(fn).not.toHaveBeenCalled();
    hidden = false;
    listeners.forEach((cb) => cb());
    await vi.advanceTimersByTimeAsync(0);
    expect(fn).toHaveBeenCalledTimes(1);
    listeners.forEach((cb) => cb()); // a second show without a missed tick does nothing
    await vi.advanceTimersByTimeAsync(0);
    expect(fn).toHaveBeenCalledTimes(1);
    p.stop();
    expect(listeners.size).toBe(0);
    vi.useRealTimers();
  });
  it('reads document.visibilityState by default', async () => {
    vi.useFakeTimers();
    const had = Object.prototype.hasOwnProperty.call(globalThis, 'document');
    const prev = globalThis.document;
    const listeners = new Set();
    globalThis.document = {
      visibilityState: 'hidden',
      addEventListener: (type, l) => type === 'visibilitychange' && listeners.add(l),
      removeEventListener: (type, l) => listeners.delete(l),
    };
    try {
      const fn = vi.fn(() => Promise.resolve());
      const p = createPoller(5);
      p.start(fn);
      expect(listeners.size).toBe(1);
      await vi.advanceTimersByTimeAsync(15000);
      expect(fn).not.toHaveBeenCalled();
      globalThis.document.visibilityState = 'visible';
      listeners.forEach((l) => l());
      await vi.advanceTimersByTimeAsync(0);
      expect(fn).toHaveBeenCalledTimes(1);
      p.stop();
      expect(listeners.size).toBe(0);
    } finally {
      if (had) globalThis.document = prev;
      else delete globalThis.document;
      vi.useRealTimers();
    }
  });
  it('backs off 1, 2, 4, 8, 8 ticks while calls miss and resets on the first success', async () => {
    vi.useFakeTimers();
    const at = [];
    let n = 0;
    const fn = vi.fn(() => {
      at.push(Date.now());
      n++;
      return Promise.resolve(n <= 5 ? POLL_MISS : undefined);
    });
    const t0 = Date.now();
    const p = createPoller(10, { setInterval, clearInterval, hidden: () => false, onVisible: () => () => {} });
    p.start(fn);
    await vi.advanceTimersByTimeAsync(300000);
    expect(at.map((t) => (t - t0) / 1000)).toEqual([10, 30, 60, 110, 200, 290, 300]);
    expect(p.stats().missSkips).toBe(1 + 2 + 4 + MAX_MISS_SKIPS + MAX_MISS_SKIPS);
    p.stop();
    vi.useRealTimers();
  });
  it('period 0 never polls', () => {
    const fn = vi.fn();
    const p = createPoller(0);
    p.start(fn);
    expect(p.stats().running).toBe(false);
  });
});
