/**
 * GPU Pods page view-model (reference src/components/PodsPage.tsx:94-270,
 * SURVEY C8): one page of GPU pods, the pending pods, and which physical
 * GPUs each pod holds when the exporter attributes them (ownersScope).
 */

import {
  formatPodGpuRequests,
  phaseToStatus,
  podPhase,
  podWaitingMessage,
  podWaitingReason,
} from '../../api/amdPods.js';
import { podContainerLines, podFacts } from '../../api/clusterIndex.js';
import { assignmentTexts, podGpuAssignments, podPowerText } from '../../api/nodeSummaries.js';
import { formatBytes, formatWatts } from '../../api/k8sCore.js';
import { SMALL_CLUSTER_PODS } from '../../api/series.js';
import { kv, lines, loader, page, pager, row, section, status, table } from '../ir.js';
import {
  ageText,
  BRAND,
  chunkedFilter,
  chunkedRows,
  errorSection,
  memo,
  nowOf,
  pendingRows,
  podName,
  podNode,
  podNs,
  podRows,
  refreshButton,
  restartsCell,
  nodesPending,
  podsPending,
} from './common.js';
import { podKeyOf, podPage, PODS_PER_PAGE, podSortOf, RANKED_POD_SORTS, rankedSlice } from './paging.js';

/** The rank of a power-ordered owners answer as a pager page: its pods, in rank order, out of the pods ranked. */
function rankedPodPage(ctx, m, state) {
  const byKey = memo('pods-by-key', [ctx.gpuPods], function () {
    const out = new Map();
    for (let i = 0; i < ctx.gpuPods.length; i++) out.set(podKeyOf(ctx.gpuPods[i]), ctx.gpuPods[i]);
    return out;
  });
  return memo('pods-ranked-page', [m, byKey], function () {
    const r = m.rank;
    const pods = [];
    for (let i = 0; i < r.order.length; i++) if (byKey.has(r.order[i])) pods.push(byKey.get(r.order[i]));
    return Object.assign(rankedSlice(r, pods.length, state), { nodes: pods, names: pods.map(podKeyOf), ranked: true });
  });
}

// podGpuAssignments: "namespace/pod" → the GPUs the exporter attributes to
// the pod, derived when a telemetry snapshot arrives (api/nodeSummaries.js).
export { podGpuAssignments, podPowerText };

export function assignedLines(gs) {
  return lines(
    gs.map(function (g) {
      const parts = [];
      if (g.powerWatts !== null && g.powerWatts !== undefined) parts.push(formatWatts(g.powerWatts));
      if (g.gfxActivityPct !== null && g.gfxActivityPct !== undefined) parts.push(Math.round(g.gfxActivityPct) + '% GFX');
      if (g.vramUsedBytes !== null && g.vramUsedBytes !== undefined) parts.push(formatBytes(g.vramUsedBytes) + ' HBM');
      if (g.tempC !== null && g.tempC !== undefined) parts.push(Math.round(g.tempC) + ' °C');
      return { label: g.nodeName + ' GPU ' + g.gpu, text: parts.length ? parts.join(', ') : 'no telemetry' };
    })
  );
}

/**
 * The Pods page's owner query: `small` (every owner when at most
 * SMALL_CLUSTER_PODS pods hold a GPU, else the page's pods) while the pod
 * list loads or is that short; the pods of its page (namespace/name keys)
 * once a longer list is in; cluster-wide when the pod list failed.
 * @returns {{enabled: boolean, pods: (string[]|undefined), small?: boolean, preview?: number}}
 */
export function ownersScope(ctx, state) {
  if (!ctx) return { enabled: false, pods: [] };
  // Power order: Prometheus picks the page — no pod list needed.
  if (podSortOf(state, RANKED_POD_SORTS) === 'power') {
    const st = state || {};
    return {
      enabled: true,
      rank: { by: 'power', page: Math.max(0, Math.floor(st.page) || 0), per: PODS_PER_PAGE, filter: (st.filter || '').trim().toLowerCase() },
    };
  }
  if (ctx.podsState === 'error') return { enabled: true, pods: undefined };
  // As telemetryScope: every owner of a small cluster in the first wave; on a
  // larger one the PODS_PER_PAGE pods drawing the most power, so the page has
  // rows before the pod list is in (podsPreview).
  if (ctx.podsState !== 'ready' && podsPending(ctx)) return { enabled: true, pods: [], small: true, preview: PODS_PER_PAGE };
  if (ctx.error && (!ctx.gpuPods || ctx.gpuPods.length === 0)) return { enabled: true, pods: undefined };
  const pods = podPage(ctx.gpuPods, state).names;
  return ctx.gpuPods.length <= SMALL_CLUSTER_PODS ? { enabled: true, pods: pods, small: true } : { enabled: true, pods: pods };
}

/**
 * Per-container GPU lines (reference GpuContainerList, PodsPage.tsx:49-88),
 * init containers included — derived once per pod object, the first time a
 * page shows the pod (clusterIndex.js podContainerLines). One container is
 * plain text.
 */
export function gpuContainerLines(pod) {
  const cs = podContainerLines(pod);
  if (!cs.length) return '—';
  return cs.length === 1 ? cs[0].label + ': ' + cs[0].text : lines(cs);
}

export function podsView(ctx, opts) {
  const now = nowOf(opts);
  // The page draws the pod list (and the index, built from the nodes too); it
  // does not wait for the DeviceConfigs. Until the lists are in, the
  // exporter's owner answer (when it came first) is shown as a partial page.
  if (podsPending(ctx) || nodesPending(ctx)) {
    const pv = podsPreview(opts && opts.metrics);
    if (!pv) return page(null, null, [loader('Loading GPU pod data...')]);
    return page(BRAND + ' — Pods', refreshButton('Refresh pod data', !!(opts && opts.fetching)), pv);
  }
  const assign = opts && opts.metrics ? podGpuAssignments(opts.metrics) : null;
  // One page of the GPU pod table (PODS_PER_PAGE, filter on namespace/name
  // and node): the reference lists every GPU pod (PodsPage.tsx:201-236).
  const sort = podSortOf(opts && opts.pager, RANKED_POD_SORTS);
  const m = opts && opts.metrics;
  const ranked = sort === 'power' && m && m.rank && Array.isArray(m.rank.order);
  const pg = ranked ? rankedPodPage(ctx, m, opts.pager) : podPage(ctx.gpuPods, opts && opts.pager);
  const items = memo('pods', [pg, ctx.index, ctx.error, assign, sort], function () {
    return podsItems(ctx, now, assign, pg, sort);
  }, now);
  return page(BRAND + ' — Pods', refreshButton('Refresh pod data', !!(opts && opts.fetching)), items);
}

function podsItems(ctx, now, assign, pg, sort) {
  const items = [];
  if (ctx.error) items.push(errorSection(ctx.error));
  const pods = ctx.gpuPods;

  if (pods.length === 0) {
    items.push(
      section('No GPU Pods Found', [
        kv([
          row('Status', status('warning', 'No pods requesting AMD GPU resources were found')),
          row('Note', 'Pods appear here when they request resources like amd.com/gpu.'),
        ]),
      ])
    );
  }

  const ph = ctx.index.phases;
  const pending = ph.Pending > 0 ? chunkedFilter('pending-pods', pods, function (p) { return podFacts(p).phase === 'Pending'; }) : [];
  if (pods.length > 0) {
    const rows = [row('Total GPU Pods', String(pods.length))];
    if (ph.Running > 0) rows.push(row('Running', status('success', ph.Running)));
    if (ph.Pending > 0) rows.push(row('Pending', status('warning', ph.Pending)));
    if (ph.Failed > 0) rows.push(row('Failed', status('error', ph.Failed)));
    rows.push(row('GPUs Held', String(ctx.index.totals.heldGpus)));
    items.push(section('Summary', [kv(rows)]));

    // With exporter pod labels, show which physical GPUs each pod holds.
    const exact = assign && Object.keys(assign).length > 0;
    const cols = ['Name', 'Namespace', 'Node', 'Phase', 'GPU Resources', 'Restarts', 'Age'];
    if (exact) cols.splice(5, 0, 'Assigned GPUs', 'GPU Power');
    items.push(pager(pg, pg.ranked ? 'GPU pods drawing power' : 'GPU pods', { sort: sort, sorts: RANKED_POD_SORTS, label: 'GPU pods' }));
    items.push(
      section('All GPU Pods', [
        table(
          cols,
          chunkedRows('pod-rows', pg.nodes, [exact, assign], function (p) {
            // A pod's assignment keeps its identity while its GPUs are unchanged (podGpuAssignments).
            const gs = exact ? assign[(p.metadata.namespace || '') + '/' + p.metadata.name] : undefined;
            return podRows(p, [exact, gs], function () {
              const phase = podPhase(p);
              const r = [
                podName(p), podNs(p), podNode(p), status(phaseToStatus(phase), phase), gpuContainerLines(p),
                restartsCell(p), ageText(p.metadata.creationTimestamp, now),
              ];
              if (exact) {
                const t = assignmentTexts(gs);
                r.splice(5, 0, t.assigned, t.power);
              }
              return r;
            }, now);
          }, now),
          pg.nodes.map(function (p) { return p.metadata.uid || (p.metadata.namespace + '/' + p.metadata.name); })
        ),
      ])
    );
  }

  if (pending.length > 0) {
    // The oldest PODS_PER_PAGE pending pods (a scheduler backlog can be
    // thousands deep); the rest are counted, and found with the filter.
    const shown = pending.length > PODS_PER_PAGE ? pending.slice(0, PODS_PER_PAGE) : pending;
    const blocks = [
      table(
        // "Message" (beyond the reference): why the scheduler cannot place the pod.
        ['Name', 'Namespace', 'GPU Resources', 'Waiting Reason', 'Message', 'Age'],
        shown.map(function (p) {
          return pendingRows(p, [], function () {
            return [podName(p), podNs(p), formatPodGpuRequests(p), podWaitingReason(p) || '—', podWaitingMessage(p) || '—',
              ageText(p.metadata.creationTimestamp, now)];
          }, now);
        })
      ),
    ];
    if (shown.length < pending.length) {
      blocks.push(kv([row('Not shown', (pending.length - shown.length) + ' more pending GPU pods (filter the table above by name)')]));
    }
    items.push(section('Attention: Pending GPU Pods', blocks));
  }

  return items;
}

/**
 * The GPU Pods page while the pod list is on its way (ADR 013): rows for the
 * pods the exporter attributes GPUs to — on a small cluster every owner in
 * namespace / name order, on a larger one the PODS_PER_PAGE pods drawing the
 * most power (ownersScope `preview`) — marked partial. Kubernetes facts the
 * exporter does not carry (requests, restarts, age, pending pods) follow with
 * the list, which then replaces these rows. Null when the answer names no
 * owner (or has not come).
 */
const HOLDS_GPUS = 'Holds GPUs';

export function podsPreview(metrics) {
  if (!metrics || !metrics.gpus) return null;
  const assign = podGpuAssignments(metrics);
  const pv = metrics.preview;
  return memo('pods-preview', [assign, pv], function () {
    const keys = pv && Array.isArray(pv.order) ? pv.order.filter(function (k) { return assign[k]; })
      : Object.keys(assign).sort().slice(0, PODS_PER_PAGE);
    if (!keys.length) return null;
    const total = pv ? pv.count : Object.keys(assign).length;
    const held = pv ? null : metrics.gpus.filter(function (g) { return !!g.pod; }).length;
    const sum = [
      row('Status', status('warning', 'Partial — the pod list is loading; these rows come from the GPU exporter')),
      row('Pods Holding GPUs', String(total)),
    ];
    if (held !== null) sum.push(row('GPUs Held', String(held)));
    const rows = keys.map(function (k) {
      const gs = assign[k];
      const slash = k.indexOf('/');
      const nodes = [];
      for (let i = 0; i < gs.length; i++) if (nodes.indexOf(gs[i].nodeName) < 0) nodes.push(gs[i].nodeName);
      // The exporter says the pod holds GPUs, not its phase: devices are bound at
      // admission, so a pod still in ContainerCreating (Pending) is attributed too.
      return [k.slice(slash + 1), k.slice(0, slash), nodes.join(', '), HOLDS_GPUS,
        gs.length + ' GPU' + (gs.length === 1 ? '' : 's') + ' held', assignmentTexts(gs).assigned, assignmentTexts(gs).power, '—', '—'];
    });
    return [
      section('Summary (partial)', [kv(sum)]),
      section(pv ? 'GPU Pods Drawing the Most Power (partial)' : 'GPU Pods (partial)', [
        table(['Name', 'Namespace', 'Node', 'Phase', 'GPU Resources', 'Assigned GPUs', 'GPU Power', 'Restarts', 'Age'], rows, keys),
      ]),
    ];
  });
}

/** Live power of the GPUs a pod holds (exporter pod labels), summed; "—" without a reading. */
