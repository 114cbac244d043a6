/**
 * Settings page — the plugin's entry on Headlamp's plugin settings screen,
 * written against an injected React and CommonComponents (no JSX) like the
 * rest of the presentation layer (./react.js).
 *
 * Edits the validated settings of src/api/settings.js: an explicit Prometheus
 * service (tried before the built-in candidates), auto-refresh period,
 * request timeout and the Metrics time-series window. Values are validated
 * on save; invalid input falls back to the defaults field by field. The
 * reference has no runtime settings at all (SURVEY.md §5 "Config / flag
 * system: absent").
 */

import { loadSettings as defaultLoad, parseSettings, REFRESH_CHOICES, saveSettings as defaultSave } from '../api/settings.js';

const INPUT = { padding: '4px 6px', fontSize: '13px', minWidth: '180px' };
const PROM_FIELDS = ['namespace', 'service', 'port'];
const PLACEHOLDER = { namespace: 'monitoring', service: 'prometheus-operated', port: '9090' };

/** Label of an auto-refresh choice in seconds. */
export function refreshChoiceLabel(v) {
  if (v === 0) return 'Off (manual)';
  return v < 60 ? v + ' s' : v / 60 + ' min';
}

/**
 * @param {any} React
 * @param {Record<string, Function>} CC  CommonComponents (SectionBox, NameValueTable)
 * @param {{load?: Function, save?: Function}} [storage]  settings persistence (tests inject memory storage)
 */
export function createSettingsPage(React, CC, storage) {
  const h = React.createElement;
  const load = (storage && storage.load) || function () { return defaultLoad(); };
  const save = (storage && storage.save) || function (v) { return defaultSave(v); };

  return function SettingsPage(props) {
    const st = React.useState(function () { return load(); });
    const s = st[0];
    const setS = st[1];
    const pr = React.useState(function () {
      return {
        namespace: s.prometheus ? s.prometheus.namespace : '',
        service: s.prometheus ? s.prometheus.service : '',
        port: s.prometheus ? s.prometheus.port : '',
      };
    });
    const prom = pr[0];
    const setProm = pr[1];
    // What the number fields show while being edited; on leaving a field the
    // validated (maybe clamped) value replaces the draft, so the screen never
    // shows a number that was not saved.
    const dr = React.useState(function () {
      return { requestTimeoutMs: String(s.requestTimeoutMs), seriesMinutes: String(s.seriesMinutes) };
    });
    const drafts = dr[0];
    const setDrafts = dr[1];

    function commit(next) {
      const saved = save(next);
      setS(saved);
      if (props && props.onDataChange) props.onDataChange(saved);
      return saved;
    }

    function commitProm(p) {
      const any = p.namespace || p.service || p.port;
      commit(parseSettings(Object.assign({}, s, { prometheus: any ? p : null })));
    }

    function numberField(label, key) {
      return h('input', {
        'aria-label': label,
        type: 'number',
        style: INPUT,
        value: drafts[key],
        onChange: function (e) {
          const next = Object.assign({}, drafts);
          next[key] = e.target.value;
          setDrafts(next);
        },
        onBlur: function (e) {
          const patch = {};
          patch[key] = Number(e.target.value);
          const saved = commit(parseSettings(Object.assign({}, s, patch)));
          const next = Object.assign({}, drafts);
          next[key] = String(saved[key]);
          setDrafts(next);
        },
      });
    }

    return h(
      CC.SectionBox,
      { title: 'AMD GPU plugin settings' },
      h(CC.NameValueTable, {
        rows: [
          {
            name: 'Prometheus service (namespace / name / port)',
            value: h(
              'div',
              { style: { display: 'flex', gap: '6px' } },
              PROM_FIELDS.map(function (k) {
                return h('input', {
                  key: k,
                  'aria-label': 'Prometheus ' + k,
                  placeholder: PLACEHOLDER[k],
                  style: INPUT,
                  value: prom[k],
                  onChange: function (e) {
                    const next = Object.assign({}, prom);
                    next[k] = e.target.value;
                    setProm(next);
                  },
                  onBlur: function () { commitProm(prom); },
                });
              })
            ),
          },
          {
            name: 'Auto-refresh',
            value: h(
              'select',
              {
                'aria-label': 'Auto-refresh interval',
                style: INPUT,
                value: s.refreshIntervalSec,
                onChange: function (e) {
                  commit(parseSettings(Object.assign({}, s, { refreshIntervalSec: Number(e.target.value) })));
                },
              },
              REFRESH_CHOICES.map(function (v) { return h('option', { key: v, value: v }, refreshChoiceLabel(v)); })
            ),
          },
          { name: 'Request timeout (ms)', value: numberField('Request timeout', 'requestTimeoutMs') },
          { name: 'Metrics time-series window (min)', value: numberField('Series window', 'seriesMinutes') },
        ],
      })
    );
  };
}
