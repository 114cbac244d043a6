/**
 * Replay of the REFERENCE plugin's request schedule against the same fake
 * cluster, for the measured baseline (BASELINE.md "How the comparison will
 * be made"; SURVEY.md §6). Paths are the AMD equivalents so both schedules
 * fetch the same data from the same server; only ordering, concurrency,
 * caching and timeouts follow the reference:
 *
 *   provider refresh      src/api/IntelGpuDataContext.tsx:113-190
 *     CRD list (2 s timeout)                                  :122-138
 *     then 3 plugin-pod requests, one after another (2 s each) :142-165
 *     dedupe by uid, uid-less pods dropped                     :168-174
 *   metrics fetch         src/api/metrics.ts:96-155, re-run by
 *                         MetricsPage.tsx:203-231 once ctx loading ends
 *     serial discovery probes, no timeout, no cache            :77-90
 *     then 4 instant queries in parallel                       :101-116
 *     power / cap joined by chip only                          :127-138
 *   cold route mount      src/index.tsx:87-145 (one provider per route)
 *     node + pod list (Headlamp useList) alongside the chain   :98-99
 *
 * This file is original code that reproduces the schedule; it contains no
 * reference source.
 */

import { filterAmdGpuNodes, isDeviceConfig } from '../src/api/amdNodes.js';
import { filterAmdGpuPluginPods, filterGpuRequestingPods } from '../src/api/amdPods.js';
import { buildClusterIndex } from '../src/api/clusterIndex.js';
import { AMD_GPU_OPERATOR_NAMESPACE, DEVICE_CONFIG_LIST_PATH, isKubeList } from '../src/api/k8sCore.js';
import { withTimeout } from '../src/api/clusterStore.js';
import { PROMETHEUS_SERVICES, servicePath } from '../src/api/series.js';

export const REF_TIMEOUT_MS = 2000;

/** The reference's three selector requests, with AMD labels. */
export const REF_SELECTORS = [
  '/api/v1/pods?labelSelector=' + encodeURIComponent('name=amdgpu-dp-ds'),
  '/api/v1/pods?labelSelector=' + encodeURIComponent('name=amdgpu-labeller-ds'),
  '/api/v1/namespaces/' + AMD_GPU_OPERATOR_NAMESPACE + '/pods',
];

/** The reference's four PromQL queries, on amdgpu hwmon instead of i915. */
export const REF_QUERIES = [
  'node_hwmon_chip_names{chip_name="amdgpu"}',
  'node_hwmon_power_average_watt * on(chip,instance) group_left(chip_name) node_hwmon_chip_names{chip_name="amdgpu"}',
  'node_hwmon_power_cap_watt * on(chip,instance) group_left(chip_name) node_hwmon_chip_names{chip_name="amdgpu"}',
  'node_uname_info',
];

export function createReferenceSchedule(request) {
  const state = {
    nodes: null,
    pods: null,
    deviceConfigs: [],
    crdAvailable: false,
    pluginPods: [],
    metrics: null,
  };

  async function providerRefresh() {
    try {
      const list = await withTimeout(request(DEVICE_CONFIG_LIST_PATH), REF_TIMEOUT_MS);
      if (isKubeList(list)) {
        state.crdAvailable = true;
        state.deviceConfigs = list.items.filter(isDeviceConfig);
      }
    } catch (e) {
      state.crdAvailable = false;
      state.deviceConfigs = [];
    }
    const found = [];
    for (let i = 0; i < REF_SELECTORS.length; i++) {
      try {
        const list = await withTimeout(request(REF_SELECTORS[i]), REF_TIMEOUT_MS);
        if (isKubeList(list)) found.push.apply(found, filterAmdGpuPluginPods(list.items));
      } catch (e) {
        // ignored, as in the reference
      }
    }
    const seen = {};
    state.pluginPods = found.filter(function (p) {
      const uid = p.metadata.uid;
      if (!uid || seen[uid]) return false;
      seen[uid] = true;
      return true;
    });
  }

  async function findPrometheusPath() {
    for (let i = 0; i < PROMETHEUS_SERVICES.length; i++) {
      const base = servicePath(PROMETHEUS_SERVICES[i]);
      try {
        const raw = await request(base + '/api/v1/query?query=1');
        if (raw && raw.status === 'success') return base;
      } catch (e) {
        // try next
      }
    }
    return null;
  }

  async function fetchMetrics() {
    const base = await findPrometheusPath();
    if (!base) {
      state.metrics = null;
      return;
    }
    const res = await Promise.all(
      REF_QUERIES.map(function (q) {
        return request(base + '/api/v1/query?query=' + encodeURIComponent(q)).then(function (raw) {
          return raw && raw.status === 'success' && raw.data ? raw.data.result : [];
        });
      })
    );
    const chips = res[0];
    const instToNode = {};
    res[3].forEach(function (r) {
      if (r.metric.instance) instToNode[r.metric.instance] = r.metric.nodename || r.metric.node || r.metric.instance;
    });
    // Keyed by chip only, exactly as the reference (quirk Q1).
    const power = {};
    res[1].forEach(function (r) { if (r.metric.chip) power[r.metric.chip] = parseFloat(r.value[1]); });
    const cap = {};
    res[2].forEach(function (r) { if (r.metric.chip) cap[r.metric.chip] = parseFloat(r.value[1]); });
    const gpus = chips.map(function (r, i) {
      const chip = r.metric.chip || '';
      return {
        nodeName: instToNode[r.metric.instance] || r.metric.instance,
        gpu: String(i),
        instance: r.metric.instance,
        powerWatts: chip in power ? power[chip] : null,
        powerCapWatts: chip in cap ? cap[chip] : null,
        vramUsedBytes: null, vramTotalBytes: null, gfxActivityPct: null, memActivityPct: null, tempC: null,
        pod: null, namespace: null,
      };
    });
    state.metrics = { source: 'node-exporter', gpus: gpus, xgmi: {}, fetchedAt: new Date().toISOString(), prometheusPath: base };
  }

  async function loadLists() {
    const r = await Promise.all([request('/api/v1/nodes'), request('/api/v1/pods')]);
    state.nodes = r[0].items;
    state.pods = r[1].items;
  }

  /**
   * Composite refresh: provider chain, then the Metrics page's re-fetch. No
   * single reference button does this (kept as a secondary figure); a click
   * runs ONE of the two, see refreshPage.
   */
  async function refresh() {
    await providerRefresh();
    await fetchMetrics();
  }

  /**
   * One page's Refresh button, as the reference wires it:
   *   Overview / Device Plugins / GPU Nodes / GPU Pods → the provider's
   *   `refresh` (OverviewPage.tsx:143-158, DevicePluginsPage.tsx:39,
   *   NodesPage.tsx:203, PodsPage.tsx:118 → IntelGpuDataContext.tsx:122-165);
   *   Metrics → `fetchGpuMetrics` only (MetricsPage.tsx:198-200,238-258).
   */
  function refreshPage(page) {
    return page === 'metrics' ? fetchMetrics() : providerRefresh();
  }

  /** Cold route mount: lists alongside the chain, then metrics. */
  async function coldOpen() {
    await Promise.all([loadLists(), providerRefresh()]);
    await fetchMetrics();
  }

  /**
   * One page mounted cold, as the reference wires it: every route mounts a
   * fresh provider (lists alongside the serial CRD + selector chain,
   * src/index.tsx:87-145); the Metrics page then waits for the provider to
   * finish loading before it fetches (MetricsPage.tsx:203-205).
   */
  async function coldOpenPage(page) {
    await Promise.all([loadLists(), providerRefresh()]);
    if (page === 'metrics') await fetchMetrics();
  }

  /** Snapshot in the shape the view-models take. */
  function snapshot() {
    const gpuNodes = filterAmdGpuNodes(state.nodes || []);
    const gpuPods = filterGpuRequestingPods(state.pods || []);
    return {
      deviceConfigs: state.deviceConfigs,
      pluginInstalled: state.deviceConfigs.length > 0 || state.pluginPods.length > 0,
      gpuNodes: gpuNodes,
      gpuPods: gpuPods,
      pluginPods: state.pluginPods,
      crdAvailable: state.crdAvailable,
      loading: false,
      refreshing: false,
      error: null,
      index: buildClusterIndex(gpuNodes, gpuPods),
      lastUpdated: Date.now(),
    };
  }

  return { refresh: refresh, refreshPage: refreshPage, coldOpen: coldOpen, coldOpenPage: coldOpenPage, snapshot: snapshot, metrics: function () { return state.metrics; } };
}
