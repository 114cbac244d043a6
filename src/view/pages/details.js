/**
 * Native-view integrations (SURVEY C10-C12): the section on Headlamp's Node
 * detail page (reference src/components/NodeDetailSection.tsx:36-138), the one
 * on its Pod detail page (PodDetailSection.tsx:25-114) and the columns of its
 * Nodes table (integrations/NodeColumns.tsx:17-48).
 */

import {
  formatGpuModel,
  getGpuResources,
  getNodeGpuCount,
  getNodeGpuModel,
  getNodePhysicalGpuCount,
  isAmdGpuNode,
} from '../../api/amdNodes.js';
import {
  containerGpuEntries,
  getPodGpuCount,
  getPodGpuDemand,
  gpuContainers,
  gpuInitContainers,
  isGpuRequestingPod,
  podPhase,
} from '../../api/amdPods.js';
import {
  AMD_GPU_RESOURCE,
  formatBytes,
  formatGpuResourceName,
  formatWatts,
  get,
  MI355X,
  pct,
  pctToStatus,
  unwrapKubeObject,
} from '../../api/k8sCore.js';
import { clusterPowerStats } from '../../api/telemetry.js';
import { kv, row, section, status } from '../ir.js';
import { formatWindow, memo, podDetailCache, podName, podsPending, seriesMeans } from './common.js';
import { gpuTelemetryTable } from './metricsPage.js';
import { matrixBlock, ownersByNode, slotsBlock } from './nodes.js';
import { assignedLines, podGpuAssignments } from './pods.js';

/**
 * @param {any} resource  Headlamp KubeObject or raw Node
 * @param {{gpuPods: any[], loading: boolean, index?: any}} ctx
 * @returns {any|null}  a section, or null for non-GPU nodes
 *
 * Differences: in-use counts GPUs of every bound non-terminated pod
 * including init containers (reference: running pods' regular containers
 * only, quirk Q3); adds HBM, slots and the xGMI matrix.
 */
export function nodeDetailView(resource, ctx, opts) {
  const raw = unwrapKubeObject(resource);
  if (!isAmdGpuNode(raw)) return null;
  const cap = getGpuResources(get(raw, ['status', 'capacity'], null));
  const alloc = getGpuResources(get(raw, ['status', 'allocatable'], null));
  if (Object.keys(cap).length === 0 && Object.keys(alloc).length === 0) return null;
  const name = raw.metadata.name;
  let podsOnNode;
  const podsPend = podsPending(ctx);
  if (podsPend) podsOnNode = [];
  else if (ctx.index && ctx.index.podsByNode && ctx.index.podsByNode.get(name)) podsOnNode = ctx.index.podsByNode.get(name);
  else podsOnNode = ctx.gpuPods.filter(function (p) { return get(p, ['spec', 'nodeName'], null) === name; });
  const metrics = opts && opts.metrics ? opts.metrics : null;
  const own = ownersByNode(metrics)[name];
  const xg = metrics && metrics.xgmi ? metrics.xgmi[name] : undefined;
  const lk = metrics && metrics.links ? metrics.links[name] : undefined;
  const podsUnreadable = ctx.podsState === 'error';
  // Pods from the store's last list while the node's own list is on its way (nodePodHooks.js useNodePods).
  const seeded = !!ctx.podsSeeded && !podsPend;
  const series = opts && opts.series && opts.series.power && opts.series.power.length ? opts.series : null;
  // This node's GPUs from the node-scoped snapshot (metrics.js fetchNodeMetrics): the live telemetry table.
  const gs = metrics && metrics.gpus ? metrics.gpus.filter(function (g) { return g.nodeName === name; }) : [];
  const deps = [raw, podsOnNode, podsPend, podsUnreadable, seeded, own, xg, lk, series].concat(gs);
  return memo('node-detail:' + name, deps, function () {
    return nodeDetailSection(raw, name, cap, alloc, podsOnNode, podsPend, own, xg, lk, podsUnreadable, series, gs, seeded);
  });
}

const SEEDED_NOTE = ' (from an earlier pod list; refreshing…)';

function nodeDetailSection(raw, name, cap, alloc, podsOnNode, loading, own, xg, lk, podsUnreadable, series, gs, seeded) {
  const allocatable = parseInt(alloc[AMD_GPU_RESOURCE] || '0', 10) || 0;
  let inUse = 0;
  for (let i = 0; i < podsOnNode.length; i++) {
    const ph = podPhase(podsOnNode[i]);
    if (ph !== 'Succeeded' && ph !== 'Failed') inUse += getPodGpuCount(podsOnNode[i]);
  }
  const p = pct(inUse, allocatable);
  const model = getNodeGpuModel(raw);
  const rows = [row('GPU Model', model.product)];
  for (const k in cap) rows.push(row(formatGpuResourceName(k) + ' (capacity)', cap[k]));
  for (const k in alloc) rows.push(row(formatGpuResourceName(k) + ' (allocatable)', alloc[k]));
  const count = getNodeGpuCount(raw);
  const phys = getNodePhysicalGpuCount(raw);
  if (count > 0) rows.push(row('HBM', formatBytes(phys * MI355X.hbmBytes)));
  if (allocatable > 0 && !podsUnreadable) {
    rows.push(row('GPU Allocation', status(pctToStatus(p), inUse + '/' + allocatable + ' (' + p + '%)' + (seeded ? SEEDED_NOTE : ''))));
  }
  // With the pod list unreadable (RBAC) the node's pods are unknown, not
  // absent: say so rather than "None" or an endless "Loading…".
  rows.push(
    row(
      'GPU Workload Pods',
      podsOnNode.length > 0
        ? podsOnNode.map(podName).join(', ') + (seeded ? SEEDED_NOTE : '')
        : podsUnreadable
          ? status('warning', 'Unavailable — the pod list could not be read')
          : loading ? 'Loading…' : seeded ? 'None' + SEEDED_NOTE : 'None'
    )
  );
  let blocks = [kv(rows)];
  if (count > 0) {
    blocks.push(slotsBlock(raw, podsOnNode, own));
    if (gs.length) blocks.push(gpuTelemetryTable(gs));
    // xGMI links join the GPUs of a node: a single-GPU node has no matrix to show.
    if (phys > 1) blocks.push(matrixBlock(phys, xg, lk));
  }
  if (series) blocks = blocks.concat(powerHistoryBlocks(name, 'Node', series));
  return section('AMD GPU', blocks);
}

/**
 * Self-contained (no store). Differences: init containers are listed too, so
 * an init-only GPU pod renders (reference quirk Q3), and the effective GPU
 * demand the scheduler uses is shown.
 */
export function podDetailView(resource, opts) {
  const raw = unwrapKubeObject(resource);
  const metrics = opts && opts.metrics ? opts.metrics : null;
  const series = opts && opts.series && opts.series.power && opts.series.power.length ? opts.series : null;
  if ((metrics || series) && raw && typeof raw === 'object' && raw.metadata) {
    // Live telemetry of the GPUs this pod holds (exporter pod labels), and
    // their power over the series window.
    const gs = metrics ? podGpuAssignments(metrics)[(raw.metadata.namespace || '') + '/' + raw.metadata.name] : undefined;
    if (gs || series) {
      return memo('pod-detail:' + (raw.metadata.uid || raw.metadata.namespace + '/' + raw.metadata.name), [raw, gs, series], function () {
        return podDetailSection(raw, gs, series);
      });
    }
  }
  if (podDetailCache && raw && typeof raw === 'object') {
    if (podDetailCache.has(raw)) return podDetailCache.get(raw);
    const s = podDetailSection(raw);
    podDetailCache.set(raw, s);
    return s;
  }
  return podDetailSection(raw);
}

/**
 * Blocks of a node's or pod's GPU power history: peak / average / energy over
 * the window and the sparkline row (`label` heads its first column).
 */
function powerHistoryBlocks(name, label, series) {
  const win = formatWindow(series.rangeSec || 1800);
  const byPod = {};
  byPod[name] = series.power;
  const st = clusterPowerStats(byPod);
  if (!st) return []; // no numeric sample in the window
  return [
    kv([
      row('Peak GPU Power (' + win + ')', formatWatts(st.peakWatts)),
      row('Average GPU Power (' + win + ')', formatWatts(st.avgWatts)),
      // Σ samples × query step: the energy the GPUs drew while observed.
      row('GPU Energy (' + win + ')', formatEnergy(seriesEnergyJoules(series.power, series.stepSec))),
    ]),
    { t: 'series', label: label, power: byPod, vram: {}, avgPower: seriesMeans(byPod) },
  ];
}

/**
 * Energy (J) of a power series [[t s, W]]; null with fewer than 2 samples.
 * With the range query's `stepSec` each sample holds for one step, so a gap
 * Prometheus left (an exporter restart) adds nothing instead of stretching
 * the step guessed from the first and last timestamps. Without it the
 * trapezoid rule runs over the real timestamps.
 */
export function seriesEnergyJoules(pts, stepSec) {
  if (!pts || pts.length < 2) return null;
  let sum = 0;
  if (stepSec > 0) {
    for (let i = 0; i < pts.length; i++) sum += pts[i][1];
    return sum * stepSec;
  }
  for (let i = 1; i < pts.length; i++) sum += ((pts[i][1] + pts[i - 1][1]) / 2) * (pts[i][0] - pts[i - 1][0]);
  return sum;
}

/** Joules → "x Wh" / "x kWh"; "—" when unknown. */
export function formatEnergy(joules) {
  if (joules === null || joules === undefined || !isFinite(joules)) return '—';
  const wh = joules / 3600;
  return wh >= 1000 ? (wh / 1000).toFixed(2) + ' kWh' : wh.toFixed(1) + ' Wh';
}

function podDetailSection(raw, assigned, series) {
  if (!isGpuRequestingPod(raw)) return null;
  const ics = gpuInitContainers(raw);
  const cs = gpuContainers(raw);
  const all = ics.map(function (c) { return [c, true]; }).concat(cs.map(function (c) { return [c, false]; }));
  if (all.length === 0) return null;
  const rows = [];
  for (let i = 0; i < all.length; i++) {
    const c = all[i][0];
    const cname = c.name + (all[i][1] ? ' (init)' : '');
    const es = containerGpuEntries(c);
    for (let j = 0; j < es.length; j++) {
      const res = formatGpuResourceName(es[j].key);
      rows.push(row(cname + ' → ' + res + ' request', es[j].request === null ? '—' : es[j].request));
      if (es[j].limit !== null && es[j].limit !== es[j].request) rows.push(row(cname + ' → ' + res + ' limit', es[j].limit));
    }
  }
  const phase = get(raw, ['status', 'phase'], null);
  const phaseStatus = phase === 'Running' || phase === 'Succeeded' ? 'success' : phase === 'Pending' ? 'warning' : 'error';
  const gpus = getPodGpuCount(raw);
  const whole = getPodGpuDemand(raw)[AMD_GPU_RESOURCE] === gpus;
  return section('AMD GPU Resources', [
    kv(
      [
        row('Phase', status(phaseStatus, phase || 'Unknown')),
        row('Scheduled Node', get(raw, ['spec', 'nodeName'], '—')),
        row('GPU Containers', String(all.length)),
        row(
          'GPUs (effective)',
          gpus === 0 ? '—'
            : whole ? gpus + ' × ' + MI355X.shortName + ' (' + formatBytes(gpus * MI355X.hbmBytes) + ' HBM)'
              : gpus + ' GPU device' + (gpus === 1 ? '' : 's') + ' (partitions)'
        ),
      ].concat(assigned ? [row('Assigned GPUs', assignedLines(assigned))] : []).concat(rows)
    ),
  ].concat(series ? powerHistoryBlocks(raw.metadata.name, 'Pod', series) : []));
}

/**
 * Column descriptors for the native `headlamp-nodes` table. Getters return
 * IR cells; the TSX wrapper turns status cells into StatusLabels.
 * Each getter unwraps and classifies the row once via a WeakMap cache, so
 * N columns cost one `isAmdGpuNode` per row (reference re-ran it per column).
 */
export function nodeColumns() {
  const cache = typeof WeakMap === 'function' ? new WeakMap() : null;
  function info(resource) {
    const key = resource && typeof resource === 'object' ? resource : null;
    if (cache && key && cache.has(key)) return cache.get(key);
    const raw = unwrapKubeObject(resource);
    const v = isAmdGpuNode(raw)
      ? { raw: raw, count: getNodeGpuCount(raw), physical: getNodePhysicalGpuCount(raw), model: getNodeGpuModel(raw) }
      : null;
    if (cache && key) cache.set(key, v);
    return v;
  }
  return [
    {
      label: 'GPU Model',
      getter: function (resource) {
        const i = info(resource);
        return i ? status('success', formatGpuModel(i.model)) : '—';
      },
    },
    {
      label: 'GPU Devices',
      getter: function (resource) {
        const i = info(resource);
        return i && i.count > 0 ? String(i.count) : '—';
      },
    },
    {
      label: 'GPU HBM',
      getter: function (resource) {
        const i = info(resource);
        return i && i.count > 0 ? formatBytes(i.physical * MI355X.hbmBytes) : '—';
      },
    },
  ];
}
