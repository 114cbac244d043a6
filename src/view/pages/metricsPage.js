/**
 * Metrics page view-model (reference src/components/MetricsPage.tsx:191-355,
 * SURVEY C9): cluster totals, power / HBM history, one card per GPU node of
 * the page with a per-GPU table.
 */

import { formatWatts, MI355X } from '../../api/k8sCore.js';
import { PROMETHEUS_SERVICES } from '../../api/series.js';
import { clusterPowerStats, summarizeMetrics } from '../../api/telemetry.js';
import { kv, lines, loader, page, pager, row, section, status, table } from '../ir.js';
import {
  BRAND,
  eccCell,
  formatWindow,
  hbmBar,
  localTimeText,
  memo,
  nowOf,
  pctText,
  powerBar,
  refreshButton,
  seriesMeans,
  tempCell,
  nodesPending,
} from './common.js';
import { nodePage, nodeSortOf, RANKED_NODE_SORTS, rankedPage } from './paging.js';

/** "k / n GPU nodes": nodes with telemetry out of the cluster's GPU nodes (reference mock-up "Nodes Reporting"). */
export function nodesReporting(m, ctx) {
  const seen = {};
  let k = 0;
  for (let i = 0; i < m.gpus.length; i++) {
    if (!seen[m.gpus[i].nodeName]) {
      seen[m.gpus[i].nodeName] = true;
      k++;
    }
  }
  const n = ctx && ctx.gpuNodes ? ctx.gpuNodes.length : 0;
  if (!n) return String(k);
  let missing = 0;
  for (let i = 0; i < ctx.gpuNodes.length; i++) if (!seen[ctx.gpuNodes[i].metadata.name]) missing++;
  const text = k + ' / ' + n + ' GPU nodes';
  return missing > 0 ? status('warning', text + ' (' + missing + ' without telemetry)') : text;
}

/** "k / n GPU nodes" from an aggregate count of nodes reporting (paged snapshot totals). */
export function nodesReportingCount(k, ctx) {
  const n = ctx && ctx.gpuNodes ? ctx.gpuNodes.length : 0;
  if (!n) return String(k);
  const text = k + ' / ' + n + ' GPU nodes';
  return k < n ? status('warning', text + ' (' + (n - k) + ' without telemetry)') : text;
}

/** The "GPU Nodes" row of the empty state: names, capped (a 1,000-node list is no help in one cell). */
function gpuNodeNamesText(ctx) {
  const ns = ctx.gpuNodes || [];
  if (!ns.length) return 'None detected';
  const shown = ns.slice(0, 20).map(function (n) { return n.metadata.name; }).join(', ');
  return ns.length > 20 ? shown + ' … (' + ns.length + ' GPU nodes)' : shown;
}

/** Label of the cluster-wide line in the series table. */
export const ALL_NODES_SERIES = 'All GPU nodes';

function withTotal(pts) {
  const o = {};
  if (pts && pts.length) o[ALL_NODES_SERIES] = pts;
  return o;
}

/** The entries of `byNode` for `names`, in that order. */
function pick(byNode, names) {
  const out = {};
  for (let i = 0; i < names.length; i++) if (byNode[names[i]]) out[names[i]] = byNode[names[i]];
  return out;
}

/** Per-step sum over every node of a cluster-wide series window (memoised per window). */
function seriesTotal(sr) {
  return memo('series-total', [sr], function () {
    function sum(byNode) {
      const total = {};
      for (const n in byNode || {}) {
        const pts = byNode[n] || [];
        for (let i = 0; i < pts.length; i++) {
          if (typeof pts[i][1] === 'number' && isFinite(pts[i][1])) total[pts[i][0]] = (total[pts[i][0]] || 0) + pts[i][1];
        }
      }
      return Object.keys(total).map(Number).sort(function (a, b) { return a - b; }).map(function (t) { return [t, total[t]]; });
    }
    return { power: sum(sr.power), vram: sum(sr.vram) };
  });
}

function noTelemetrySection(name) {
  return section(name + ' — no telemetry', [
    kv([row('Status', status('warning', 'No exporter series for this node (exporter not scheduled here, or not scraped yet)'))]),
  ], name);
}

/**
 * What each telemetry source provides: [row, field of a joined GPU (null: the snapshot's xGMI map), exporter
 * series, node-exporter series (null: the exporter alone has it)].
 */
const AVAILABILITY = [
  ['Power (W)', 'powerWatts', 'gpu_power_usage', 'node_hwmon_power_average_watt / power_input_watt (amdgpu hwmon)'],
  ['HBM used / total', 'vramUsedBytes', 'gpu_used_vram / gpu_total_vram', 'node_drm_memory_vram_used_bytes / size_bytes (--collector.drm)'],
  ['GFX activity (%)', 'gfxActivityPct', 'gpu_gfx_activity', 'node_drm_gpu_busy_percent (--collector.drm)'],
  ['HBM controller activity (%)', 'memActivityPct', 'gpu_umc_activity', null],
  ['Junction temperature', 'tempC', 'gpu_junction_temperature', 'node_hwmon_temp_celsius, the sensor labelled "junction" (amdgpu hwmon)'],
  ['xGMI link throughput', null, 'xgmi_neighbor_N_tx_throughput (7 links per GPU; per link where gpu_xgmi_link_hops gives the neighbour order, else per GPU)', null],
  ['Per-GPU pod owner', 'pod', 'pod / namespace labels (exporter pod association)', null],
];

/**
 * The reference's MetricRequirements box (MetricsPage.tsx:125-185), said of
 * the source that answered: each figure is "Reporting" when a GPU of the
 * page carries it, else why not and what would provide it. Before any
 * answer (or with no GPU series) the static list of what each source offers.
 * @param {any} [m]  the page's telemetry snapshot
 */
export function metricAvailabilitySection(m) {
  if (m && m.gpus && m.gpus.length && (m.source === 'amd-exporter' || m.source === 'node-exporter')) {
    const ne = m.source === 'node-exporter';
    const rows = [];
    for (let i = 0; i < AVAILABILITY.length; i++) {
      const a = AVAILABILITY[i];
      const series = ne ? a[3] : a[2];
      // This page's snapshot ('gauges') does not ask for link throughput: GPU Nodes draws it.
      if (a[1] === null && !ne && m.view === 'gauges') {
        rows.push(row(a[0], lines([{ label: '', text: 'On GPU Nodes (xGMI matrix) — ' + series }])));
        continue;
      }
      let seen = a[1] === null && Object.keys(m.xgmi || {}).length > 0;
      for (let k = 0; a[1] !== null && k < m.gpus.length && !seen; k++) seen = m.gpus[k][a[1]] !== null && m.gpus[k][a[1]] !== undefined;
      rows.push(row(a[0], seen
        ? status('success', 'Reporting — ' + series)
        : ne && series === null
          ? status('warning', 'Not available from node-exporter — the AMD Device Metrics Exporter reports ' + a[2])
          : status('warning', 'Not reported on this page — ' + series)));
    }
    return section('Metric Availability', [kv(rows)]);
  }
  return section('Metric Availability', [
    kv([
      row('Power (W)', lines([
        { label: '', text: 'Available — gpu_power_usage (AMD Device Metrics Exporter) or amdgpu hwmon power via node-exporter (power1_input on MI355X, which has no power1_average)' },
      ])),
      row('HBM used / total', lines([
        { label: '', text: 'Available — gpu_used_vram / gpu_total_vram, or node-exporter --collector.drm node_drm_memory_vram_* (288 GB HBM3E per MI355X)' },
      ])),
      row('GFX activity (%)', lines([{ label: '', text: 'Available — gpu_gfx_activity, or node_drm_gpu_busy_percent' }])),
      row('HBM controller activity (%)', lines([{ label: '', text: 'Available — gpu_umc_activity (exporter only)' }])),
      row('xGMI link throughput', lines([{ label: '', text: 'Available — xgmi_neighbor_N_tx_throughput (exporter only; 7 links per GPU). ' +
        'Drawn per link where gpu_xgmi_link_hops gives the neighbour order (this repo\'s amdgpu-exporter), else as each GPU\'s total' }])),
      row('Per-GPU pod owner', lines([{ label: '', text: 'Available when the exporter runs with pod association (pod / namespace labels)' }])),
    ]),
  ]);
}

/**
 * @param {{gpuNodes: any[], loading: boolean}} ctx
 * @param {{ metrics: any|null, fetchError: string|null, fetching: boolean, series?: any }} mstate
 *
 * Differences: one card per NODE with a per-GPU table (the reference renders
 * one card per chip — 64 cards at 8 nodes); HBM, activity and temperature
 * columns; per-node power/HBM series when range data is present.
 */
export function metricsView(ctx, mstate, opts) {
  const now = nowOf(opts);
  const items = [];
  // Only the node list matters here (nodes reporting, the per-node cards in
  // name order); the pod list and the DeviceConfigs are not drawn on this
  // page, so it never waits for them (reference: the fetch waits for the
  // whole context, MetricsPage.tsx:203-205).
  const nodesPend = nodesPending(ctx);
  if (nodesPend) items.push(loader('Loading ' + BRAND + ' data...'));
  const m = mstate.metrics;
  // The sections below that read the snapshot alone are memoised on it: a
  // watch event (a new store snapshot, same telemetry) re-renders none of them.
  items.push(memo('metrics-availability', [m], function () { return metricAvailabilitySection(m); }));
  if (mstate.fetching && !m) items.push(loader('Querying Prometheus for GPU metrics...'));

  if (mstate.fetchError) {
    // RBAC (HTTP 403 from the service proxy) is not an outage: say which permission is missing.
    const denied = /denied \(HTTP 403\)/.test(String(mstate.fetchError));
    items.push(
      section(denied ? 'Prometheus Access Denied' : 'Prometheus Unreachable', [
        kv([
          row('Error', status('error', mstate.fetchError)),
          row(
            'Checked services',
            PROMETHEUS_SERVICES.map(function (s) { return s.service + ':' + s.port; }).join(', ') + ' (monitoring namespace)'
          ),
        ]),
      ])
    );
  }

  const tot = m && m.totals ? m.totals : null;
  if (m && m.gpus.length === 0 && !(tot && tot.gpus > 0) && !(m.scope && !tot)) {
    items.push(
      section('No AMD GPU Metrics in Prometheus', [
        kv([
          row('Status', status('warning', 'Prometheus reachable — no gpu_power_usage or amdgpu hwmon series found')),
          row('GPU Nodes', gpuNodeNamesText(ctx)),
          row(
            'Likely cause',
            'The AMD Device Metrics Exporter is not deployed (DeviceConfig spec.metricsExporter.enable) or not scraped, and node-exporter is not running on the GPU nodes.'
          ),
        ]),
      ])
    );
  }

  if (m && (m.gpus.length > 0 || (tot && tot.gpus > 0))) {
    // Cluster totals: server-side aggregates on a paged (scoped) snapshot,
    // else summed here from every GPU of the snapshot.
    const sum = tot || memo('metrics-sum', [m], function () { return summarizeMetrics(m); });
    items.push(memo('metrics-summary', [m, sum, ctx.gpuNodes], function () {
      return section('GPU Power Summary', [
        kv([
          row('GPUs Monitored', String(sum.gpus)),
          row('Nodes Reporting', tot ? nodesReportingCount(tot.nodes, ctx) : nodesReporting(m, ctx)),
          row('Total Power', powerBar(sum.powerWatts, sum.powerCapWatts > 0 ? sum.powerCapWatts : null)),
          row('HBM In Use', hbmBar(sum.vramUsedBytes, sum.vramTotalBytes > 0 ? sum.vramTotalBytes : null)),
          row('Avg GFX Activity', pctText(sum.avgGfxActivityPct)),
        ].concat(sum.eccUncorrectable === null ? [] : [row('RAS Errors', eccCell(sum))], [
          row('Source', m.source === 'node-exporter' ? 'node-exporter (amdgpu hwmon + DRM)' : 'AMD Device Metrics Exporter'),
        ], limitsRows(sum), [
          // Browser-local time, as the reference shows it (MetricsPage.tsx:336-338).
          row(
            'Last Fetched',
            m.stale
              ? status('warning', localTimeText(m.fetchedAt) + ' (stale: the latest refresh failed)')
              : localTimeText(m.fetchedAt)
          ),
        ], m.query ? [row('Query', m.query)] : [])),
      ]);
    }));

    const grouped = memo('metrics-by-node', [m], function () { return gpusByNode(m.gpus); });
    const byNode = grouped.byNode;
    const order = grouped.order;
    // One page of per-node cards. A paged snapshot covers the GPU nodes of
    // the page (m.scope); a cluster-wide one is paged over the nodes reporting.
    const scoped = Array.isArray(m.scope);
    const k8s = scoped && !nodesPend && ctx.gpuNodes && ctx.gpuNodes.length > 0;
    // Power order: Prometheus picked and ranked the page (metrics.js rankedSnapshot).
    const pagerState = opts && opts.pager;
    const rankedView = !!m.rank && nodeSortOf(pagerState, RANKED_NODE_SORTS) === 'power';
    const pg = rankedView ? rankedPage(m, pagerState)
      : k8s ? nodePage(ctx.gpuNodes, pagerState, ctx.index) : nodePage(scoped ? m.scope : order, pagerState);

    const sr = mstate.series;
    if (sr && sr.power) {
      const cap = sum.powerCapWatts > 0 ? sum.powerCapWatts : null;
      items.push(memo('metrics-series', [sr, cap].concat(pg.names), function () { return seriesSection(sr, cap, pg.names); }));
    }

    items.push(rankedView ? pager(pg, 'GPU nodes reporting', { sort: 'power', sorts: RANKED_NODE_SORTS, label: 'GPU nodes' })
      : k8s ? pager(pg, 'GPU nodes', { sort: nodeSortOf(pagerState, RANKED_NODE_SORTS), sorts: RANKED_NODE_SORTS })
        : pager(pg, scoped ? 'GPU nodes' : 'GPU nodes reporting', { label: 'GPU nodes' }));
    const covered = {};
    if (scoped) for (let i = 0; i < m.scope.length; i++) covered[m.scope[i]] = true;
    let matched = 0;
    for (let i = 0; i < pg.names.length; i++) {
      const name = pg.names[i];
      const gs = byNode[name];
      if (gs) {
        matched++;
        // Deps are the node's GPU objects, which the metrics client reuses while unchanged.
        items.push(memo('metrics-node:' + name, gs, function () { return metricsNodeSection(name, gs); }));
      } else if (!scoped || covered[name]) {
        items.push(memo('metrics-none:' + name, [], function () { return noTelemetrySection(name); }));
      } else {
        items.push(section(name + ' — fetching telemetry…', [], name));
      }
    }
    if (scoped && tot && tot.gpus > 0 && matched === 0 && pg.names.length > 0 && pg.names.every(function (n) { return covered[n]; })) {
      items.push(section('Telemetry Not Matched To Nodes', [
        kv([
          row('Status', status('warning', 'Prometheus reports ' + tot.gpus + ' GPUs on ' + tot.nodes + ' nodes, none under the names of the nodes on this page')),
          row('Likely cause', 'The exporter\'s hostname label is not the Kubernetes node name (Device Metrics Exporter: set the node name as hostname).'),
        ]),
      ]));
    }
  }

  void now;
  return page(BRAND + ' — Metrics', refreshButton('Refresh metrics', mstate.fetching || nodesPend), items);
}

/** The snapshot's GPUs grouped by node, nodes in order of first appearance. */
function gpusByNode(gpus) {
  const byNode = {};
  const order = [];
  for (let i = 0; i < gpus.length; i++) {
    const g = gpus[i];
    if (!byNode[g.nodeName]) {
      byNode[g.nodeName] = [];
      order.push(g.nodeName);
    }
    byNode[g.nodeName].push(g);
  }
  return { byNode: byNode, order: order };
}

/** The power / HBM history of the cluster line and the nodes of the page (`names`). */
function seriesSection(sr, cap, names) {
  const win = formatWindow(sr.rangeSec || 1800);
  // A paged snapshot's series carry the cluster line apart (series.total);
  // a cluster-wide one is summed here. Peak / average are the cluster's;
  // the table shows the cluster line and the nodes of the page.
  const total = sr.total || seriesTotal(sr);
  const ps = clusterPowerStats({ cluster: total.power || [] });
  const statRows = ps
    ? [kv([
      row('Peak Power (' + win + ')', powerBar(ps.peakWatts, cap)),
      row('Average Power (' + win + ')', powerBar(ps.avgWatts, cap)),
    ])]
    : [];
  const power = Object.assign(withTotal(total.power), pick(sr.power, names));
  const vram = Object.assign(withTotal(total.vram), pick(sr.vram || {}, names));
  return section('Power & HBM (last ' + win + ')', statRows.concat([
    { t: 'series', power: power, vram: vram, avgPower: seriesMeans(power) },
  ]));
}

/** Says which limits are MI355X platform values because the source reports none. */
function limitsRows(sum) {
  const parts = [];
  if (sum.powerCapAssumed > 0) {
    parts.push('power cap ' + formatWatts(MI355X.tdpWatts) + ' (MI355X board limit; no gpu_power_cap series for ' +
      sum.powerCapAssumed + ' of ' + sum.gpus + ' GPUs)');
  }
  if (sum.tempLimitAssumed > 0) {
    parts.push('throttle threshold ' + MI355X.junctionSlowdownC + ' °C (MI355X; no gpu_junction_temperature_slowdown series for ' +
      sum.tempLimitAssumed + ' of ' + sum.gpus + ' GPUs)');
  }
  return parts.length ? [row('Assumed Limits', status('warning', parts.join('; ')))] : [];
}

/** One node's GPUs as a table: power against cap, HBM, activity, junction temperature, ECC, owning pod. */
export function gpuTelemetryTable(gs) {
  return table(
    ['GPU', 'Power', 'HBM Used', 'GFX', 'HBM Activity', 'Temp', 'ECC', 'Pod'],
    gs.map(function (g) {
      return [
        'GPU ' + g.gpu,
        g.powerWatts !== null ? powerBar(g.powerWatts, g.powerCapWatts) : status('warning', 'No data'),
        hbmBar(g.vramUsedBytes, g.vramTotalBytes),
        pctText(g.gfxActivityPct),
        pctText(g.memActivityPct),
        tempCell(g),
        eccCell(g),
        g.pod ? (g.namespace ? g.namespace + '/' : '') + g.pod : '—',
      ];
    }),
    gs.map(function (g) { return g.nodeName + '-' + g.gpu; })
  );
}

function metricsNodeSection(name, gs) {
  return section(name + ' — ' + gs.length + ' × ' + MI355X.shortName, [gpuTelemetryTable(gs)], name);
}
