/**
 * SettingsPage — the plugin's entry on Headlamp's plugin settings screen.
 *
 * Edits the validated settings of src/api/settings.js: an explicit Prometheus
 * service (tried before the built-in candidates), auto-refresh period,
 * request timeout and the Metrics time-series window. Values are validated on
 * save; invalid input falls back to the defaults field by field.
 */
import { NameValueTable, SectionBox } from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import React, { useState } from 'react';
import { loadSettings, parseSettings, REFRESH_CHOICES, saveSettings } from '../api/settings.js';

interface Props {
  data?: Record<string, unknown>;
  onDataChange?: (data: Record<string, unknown>) => void;
}

const input: React.CSSProperties = { padding: '4px 6px', fontSize: '13px', minWidth: '180px' };

export default function SettingsPage({ onDataChange }: Props) {
  const [s, setS] = useState(() => loadSettings());
  const [prom, setProm] = useState(() => ({
    namespace: s.prometheus ? s.prometheus.namespace : '',
    service: s.prometheus ? s.prometheus.service : '',
    port: s.prometheus ? s.prometheus.port : '',
  }));

  function commit(next: ReturnType<typeof parseSettings>) {
    const saved = saveSettings(next);
    setS(saved);
    if (onDataChange) onDataChange(saved as unknown as Record<string, unknown>);
  }

  function commitProm(p: typeof prom) {
    setProm(p);
    const any = p.namespace || p.service || p.port;
    commit(parseSettings({ ...s, prometheus: any ? p : null }));
  }

  return (
    <SectionBox title="AMD GPU plugin settings">
      <NameValueTable
        rows={[
          {
            name: 'Prometheus service (namespace / name / port)',
            value: (
              <div style={{ display: 'flex', gap: '6px' }}>
                {(['namespace', 'service', 'port'] as const).map(k => (
                  <input
                    key={k}
                    aria-label={`Prometheus ${k}`}
                    placeholder={k === 'namespace' ? 'monitoring' : k === 'service' ? 'prometheus-operated' : '9090'}
                    style={input}
                    value={prom[k]}
                    onChange={e => setProm({ ...prom, [k]: e.target.value })}
                    onBlur={() => commitProm(prom)}
                  />
                ))}
              </div>
            ),
          },
          {
            name: 'Auto-refresh',
            value: (
              <select
                aria-label="Auto-refresh interval"
                style={input}
                value={s.refreshIntervalSec}
                onChange={e => commit(parseSettings({ ...s, refreshIntervalSec: Number(e.target.value) }))}
              >
                {REFRESH_CHOICES.map(v => (
                  <option key={v} value={v}>
                    {v === 0 ? 'Off (manual)' : v < 60 ? `${v} s` : `${v / 60} min`}
                  </option>
                ))}
              </select>
            ),
          },
          {
            name: 'Request timeout (ms)',
            value: (
              <input
                aria-label="Request timeout"
                type="number"
                style={input}
                defaultValue={s.requestTimeoutMs}
                onBlur={e => commit(parseSettings({ ...s, requestTimeoutMs: Number(e.target.value) }))}
              />
            ),
          },
          {
            name: 'Metrics time-series window (min)',
            value: (
              <input
                aria-label="Series window"
                type="number"
                style={input}
                defaultValue={s.seriesMinutes}
                onBlur={e => commit(parseSettings({ ...s, seriesMinutes: Number(e.target.value) }))}
              />
            ),
          },
        ]}
      />
    </SectionBox>
  );
}
