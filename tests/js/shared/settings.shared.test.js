/**
 * The plugin's settings page (src/view/settingsPage.js, registered with
 * registerPluginSettings) driven like a user: pick an auto-refresh interval,
 * type into the number and Prometheus fields and leave them. On the harness
 * React and on real React 18.3.1 (form events go through react-dom's event
 * system there: change on the select, input + focusout on the fields).
 */
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import * as CC from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { createPlugin } from '../../../src/plugin.js';
import { DEFAULT_SETTINGS } from '../../../src/api/settings.js';

const h = React.createElement;

function memoryStorage(initial) {
  let v = initial || null;
  const saved = [];
  return {
    saved,
    load: () => v || Object.assign({}, DEFAULT_SETTINGS),
    save: (x) => {
      v = x;
      saved.push(x);
      return x;
    },
  };
}

function page(storage, props) {
  const p = createPlugin({ React, lib, CommonComponents: CC, settingsStorage: storage });
  return render(h(p.SettingsPage, props || {}));
}

describe('shared: settings page (' + tier + ')', () => {
  it('picking an auto-refresh interval saves it and tells Headlamp', () => {
    const storage = memoryStorage();
    const onDataChange = vi.fn();
    const r = page(storage, { onDataChange });
    expect(r.text()).toContain('AMD GPU plugin settings');
    const sel = r.byLabel('Auto-refresh interval');
    expect(r.value(sel)).toBe('0');
    r.change(sel, '30');
    expect(storage.saved).toHaveLength(1);
    expect(storage.saved[0].refreshIntervalSec).toBe(30);
    expect(onDataChange).toHaveBeenCalledTimes(1);
    expect(r.value(r.byLabel('Auto-refresh interval'))).toBe('30');
    r.unmount();
  });

  it('a number out of range is clamped when the field is left, and the field then shows the clamped value', () => {
    const storage = memoryStorage();
    const r = page(storage);
    expect(r.value(r.byLabel('Request timeout'))).toBe('2000');
    r.blur(r.byLabel('Request timeout'), '5');
    expect(storage.saved[0].requestTimeoutMs).toBe(250);
    expect(r.value(r.byLabel('Request timeout'))).toBe('250');
    r.blur(r.byLabel('Series window'), '100000');
    const last = storage.saved[storage.saved.length - 1];
    expect(last.requestTimeoutMs).toBe(250); // the earlier edit is kept
    expect(r.value(r.byLabel('Series window'))).toBe(String(last.seriesMinutes));
    expect(last.seriesMinutes).toBeLessThan(100000);
    r.unmount();
  });

  it('a Prometheus service is saved only once namespace, name and port are all there', () => {
    const storage = memoryStorage();
    const r = page(storage);
    r.change(r.byLabel('Prometheus namespace'), 'monitoring');
    r.blur(r.byLabel('Prometheus namespace'));
    expect(storage.saved[0].prometheus).toBeNull();
    expect(r.value(r.byLabel('Prometheus namespace'))).toBe('monitoring'); // the draft stays on screen
    r.change(r.byLabel('Prometheus service'), 'prom');
    r.change(r.byLabel('Prometheus port'), '9090');
    r.blur(r.byLabel('Prometheus port'));
    expect(storage.saved[storage.saved.length - 1].prometheus).toEqual({ namespace: 'monitoring', service: 'prom', port: '9090' });
    r.unmount();
  });

  it('opens on the stored settings', () => {
    const stored = Object.assign({}, DEFAULT_SETTINGS, { refreshIntervalSec: 60, requestTimeoutMs: 4000,
      prometheus: { namespace: 'obs', service: 'kps', port: '9090' } });
    const r = page(memoryStorage(stored));
    expect(r.value(r.byLabel('Auto-refresh interval'))).toBe('60');
    expect(r.value(r.byLabel('Request timeout'))).toBe('4000');
    expect(r.value(r.byLabel('Prometheus service'))).toBe('kps');
    r.unmount();
  });
});
