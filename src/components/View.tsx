/**
 * View — renders the page IR (src/view/ir.js) with Headlamp CommonComponents.
 *
 * Every page/section of the plugin is computed by a pure view-model in
 * src/view/pages.js and drawn here, one IR node → one component:
 *   page     → SectionHeader + refresh <button> (+ aria-label) + items
 *   loader   → Loader
 *   section  → SectionBox
 *   kv       → NameValueTable
 *   table    → SimpleTable
 *   pctbar   → PercentageBar
 *   status   → StatusLabel
 *   bar      → inline allocation / power bar (reference NodesPage.tsx:35-63)
 *   slots    → per-GPU allocation strip (new)
 *   matrix   → xGMI neighbour matrix (new)
 *   series   → inline SVG sparklines of per-node power / HBM (new)
 * Only CommonComponents plus inline-styled elements are used (reference
 * CLAUDE.md conventions: no extra UI libraries).
 */

import {
  Loader,
  NameValueTable,
  PercentageBar,
  SectionBox,
  SectionHeader,
  SimpleTable,
  StatusLabel,
} from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import React from 'react';
import { BAR_COLORS } from '../api/amdgpu.js';

/* eslint-disable @typescript-eslint/no-explicit-any */
type IR = any;

export function Value({ v }: { v: IR }): JSX.Element {
  if (v === null || v === undefined) return <></>;
  if (typeof v === 'string' || typeof v === 'number') return <>{String(v)}</>;
  switch (v.t) {
    case 'status':
      return <StatusLabel status={v.status}>{v.text}</StatusLabel>;
    case 'bar':
      return <InlineBar pct={v.pct} color={v.color} text={v.text} />;
    case 'lines':
      return (
        <>
          {v.lines.map((l: { label: string; text: string }, i: number) => (
            <div key={i} style={{ marginBottom: '2px', fontSize: '13px' }}>
              {l.label ? <strong>{l.label}</strong> : null}
              {l.label ? ': ' : null}
              {l.text}
            </div>
          ))}
        </>
      );
    default:
      return <></>;
  }
}

function InlineBar({ pct, color, text }: { pct: number | null; color: string; text: string }) {
  return (
    <div style={{ display: 'flex', alignItems: 'center', gap: '8px' }}>
      {pct !== null && (
        <div
          style={{
            width: '100px',
            height: '8px',
            backgroundColor: BAR_COLORS.track,
            borderRadius: '4px',
            overflow: 'hidden',
            flexShrink: 0,
          }}
        >
          <div
            style={{
              width: `${pct}%`,
              height: '100%',
              backgroundColor: color,
              borderRadius: '4px',
              transition: 'width 0.4s ease',
            }}
          />
        </div>
      )}
      <span style={{ fontSize: '12px', fontVariantNumeric: 'tabular-nums' }}>{text}</span>
    </div>
  );
}

function Slots({ b }: { b: IR }) {
  return (
    <div style={{ marginTop: '12px' }}>
      <div style={{ fontSize: '13px', marginBottom: '6px', color: 'var(--mui-palette-text-secondary)' }}>
        Per-GPU allocation{b.exact ? '' : ' (inferred from pod order — exporter pod labels unavailable)'}
      </div>
      <div
        style={{
          display: 'grid',
          // one row per board on partitioned nodes (up to 8 partitions each)
          gridTemplateColumns: `repeat(${Math.min(8, b.partitionsPerGpu > 1 ? b.partitionsPerGpu : 8)}, minmax(0, 1fr))`,
          gap: '4px',
        }}
      >
        {b.slots.map((s: IR) => (
          <div
            key={s.index}
            title={s.pod ? `${s.namespace ? s.namespace + '/' : ''}${s.pod}` : 'free'}
            style={{
              padding: '6px 4px',
              borderRadius: '4px',
              fontSize: '11px',
              textAlign: 'center',
              overflow: 'hidden',
              textOverflow: 'ellipsis',
              whiteSpace: 'nowrap',
              color: s.pod ? '#fff' : 'inherit',
              backgroundColor: s.pod ? BAR_COLORS.ok : BAR_COLORS.track,
              opacity: s.inferred ? 0.8 : 1,
            }}
          >
            {s.partition === null || s.partition === undefined ? `GPU ${s.index}` : `GPU ${s.board}·${s.partition}`}
            <br />
            {s.pod || 'free'}
          </div>
        ))}
      </div>
    </div>
  );
}

function Matrix({ b }: { b: IR }) {
  const m = b.matrix;
  return (
    <div style={{ marginTop: '12px', overflowX: 'auto' }}>
      <div style={{ fontSize: '13px', marginBottom: '6px', color: 'var(--mui-palette-text-secondary)' }}>
        xGMI topology ({b.measuredTopology ? 'measured' : 'MI355X platform model'}) —{' '}
        {b.fullMesh ? `full mesh, ${m.linksPerGpu} links/GPU` : 'partial'} · {m.linksPerGpu}×
        {m.size > 1 ? ` ${m.cells[0][1].peakGBs}` : ''} GB/s per GPU · ring collectives bound at {m.ringBusGBs} GB/s per link
      </div>
      <table style={{ borderCollapse: 'collapse', fontSize: '11px' }}>
        <thead>
          <tr>
            <th />
            {m.cells.map((_: IR, j: number) => (
              <th key={j} style={{ padding: '2px 6px' }}>
                GPU {j}
              </th>
            ))}
          </tr>
        </thead>
        <tbody>
          {m.cells.map((row: IR[], i: number) => (
            <tr key={i}>
              <th style={{ padding: '2px 6px', textAlign: 'right' }}>GPU {i}</th>
              {row.map((c: IR, j: number) => {
                const util = c.measuredGBs !== null && c.peakGBs > 0 ? c.measuredGBs / c.peakGBs : null;
                return (
                  <td
                    key={j}
                    title={c.kind === 'xgmi' ? `${c.hops} hop · ${c.peakGBs} GB/s peak` : c.kind}
                    style={{
                      padding: '2px 6px',
                      textAlign: 'center',
                      border: '1px solid var(--mui-palette-divider, #e0e0e0)',
                      backgroundColor:
                        c.kind === 'self'
                          ? 'transparent'
                          : util !== null
                          ? `rgba(237, 28, 36, ${0.15 + 0.85 * Math.min(1, util)})`
                          : c.kind === 'xgmi'
                          ? 'rgba(237, 28, 36, 0.08)'
                          : BAR_COLORS.track,
                    }}
                  >
                    {c.kind === 'self' ? '—' : c.measuredGBs !== null ? c.measuredGBs.toFixed(0) : c.kind === 'xgmi' ? '•' : c.kind}
                  </td>
                );
              })}
            </tr>
          ))}
        </tbody>
      </table>
    </div>
  );
}

function Sparkline({ points, color }: { points: Array<[number, number]>; color: string }) {
  if (points.length < 2) return <span>—</span>;
  const w = 240;
  const h = 36;
  const t0 = points[0][0];
  const t1 = points[points.length - 1][0];
  let lo = Infinity;
  let hi = -Infinity;
  for (const [, v] of points) {
    lo = Math.min(lo, v);
    hi = Math.max(hi, v);
  }
  const span = hi - lo || 1;
  const d = points
    .map(([t, v], i) => `${i ? 'L' : 'M'}${(((t - t0) / (t1 - t0 || 1)) * w).toFixed(1)},${(h - ((v - lo) / span) * h).toFixed(1)}`)
    .join(' ');
  return (
    <svg width={w} height={h} viewBox={`0 0 ${w} ${h}`} role="img" aria-label="time series">
      <path d={d} fill="none" stroke={color} strokeWidth={1.5} />
    </svg>
  );
}

function Series({ b }: { b: IR }) {
  const nodes = Object.keys(b.power || {});
  return (
    <SimpleTable
      columns={[
        { label: 'Node', getter: (n: string) => n },
        { label: 'Power (W)', getter: (n: string) => <Sparkline points={b.power[n] || []} color={BAR_COLORS.ok} /> },
        {
          label: 'HBM in use',
          getter: (n: string) => <Sparkline points={(b.vram && b.vram[n]) || []} color="#6a1b9a" />,
        },
      ]}
      data={nodes}
    />
  );
}

export function Block({ b }: { b: IR }): JSX.Element | null {
  switch (b.t) {
    case 'kv':
      return <NameValueTable rows={b.rows.map((r: IR) => ({ name: r.name, value: <Value v={r.value} /> }))} />;
    case 'table':
      return (
        <SimpleTable
          columns={b.columns.map((label: string, i: number) => ({
            label,
            getter: (row: IR[]) => <Value v={row[i]} />,
          }))}
          data={b.rows}
        />
      );
    case 'pctbar':
      return (
        <div style={{ marginBottom: '16px' }}>
          <div style={{ marginBottom: '8px', fontSize: '14px', color: 'var(--mui-palette-text-secondary)' }}>
            {b.label}
          </div>
          <PercentageBar data={b.data} total={b.total} />
        </div>
      );
    case 'slots':
      return <Slots b={b} />;
    case 'matrix':
      return <Matrix b={b} />;
    case 'series':
      return <Series b={b} />;
    default:
      return null;
  }
}

function SectionImpl({ s }: { s: IR }): JSX.Element | null {
  if (!s) return null;
  return (
    <SectionBox title={s.title}>
      {s.blocks.map((b: IR, i: number) => (
        <Block key={i} b={b} />
      ))}
    </SectionBox>
  );
}

/**
 * View-models return the same section object while its inputs are unchanged
 * (src/view/pages.js memo + the store's structural sharing), so a memoised
 * Section skips re-rendering unchanged parts of a page on refresh.
 */
export const Section = React.memo(SectionImpl);

const buttonStyle = (disabled: boolean): React.CSSProperties => ({
  padding: '6px 16px',
  backgroundColor: 'transparent',
  color: 'var(--mui-palette-primary-main, #ed1c24)',
  border: '1px solid var(--mui-palette-primary-main, #ed1c24)',
  borderRadius: '4px',
  cursor: disabled ? 'not-allowed' : 'pointer',
  fontSize: '13px',
  fontWeight: 500,
  opacity: disabled ? 0.6 : 1,
});

export function Page({ vm, onRefresh }: { vm: IR; onRefresh?: () => void }): JSX.Element {
  return (
    <>
      {vm.title && (
        <div style={{ display: 'flex', justifyContent: 'space-between', alignItems: 'center', marginBottom: '20px' }}>
          <SectionHeader title={vm.title} />
          {vm.refresh && (
            <button
              onClick={() => onRefresh && onRefresh()}
              disabled={vm.refresh.disabled}
              aria-label={vm.refresh.ariaLabel}
              style={buttonStyle(vm.refresh.disabled)}
            >
              {vm.refresh.label}
            </button>
          )}
        </div>
      )}
      {vm.items.map((it: IR, i: number) =>
        it.t === 'loader' ? <Loader key={`loader-${i}`} title={it.title} /> : <Section key={it.key || i} s={it} />
      )}
    </>
  );
}
