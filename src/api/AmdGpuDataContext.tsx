/**
 * AmdGpuDataContext — React binding of the shared ClusterStore.
 *
 * Reference analog: src/api/IntelGpuDataContext.tsx (SURVEY.md C3). Same
 * public contract — `useAmdGpuContext()` returns {deviceConfigs,
 * pluginInstalled, gpuNodes, gpuPods, pluginPods, crdAvailable, loading,
 * error, refresh} and throws outside a provider — but the provider is a thin
 * view onto one store per cluster (src/api/clusterStore.js):
 *
 *   * Headlamp's reactive `useList()` hooks feed nodes and pods into the
 *     store (two-track design of reference ADR 002);
 *   * the imperative track (DeviceConfig CRD + operator pods) runs in
 *     parallel inside the store, with timeouts and a sequence guard;
 *   * a mounting provider calls `revalidate(STALE_MS)`: if another view
 *     fetched moments ago (route switch, Node detail section next to a page)
 *     nothing is re-fetched and the cached snapshot renders immediately.
 */

import { ApiProxy, K8s } from '@kinvolk/headlamp-plugin/lib';
import React, { createContext, useContext, useEffect, useMemo, useState, useSyncExternalStore } from 'react';
import type { ClusterSnapshot } from './clusterStore.js';
import { createClusterStore, getSharedStore } from './clusterStore.js';
import { createMetricsSource } from './metrics.js';
import type { GpuMetrics } from './metrics.js';
import { clusterKey } from './cluster.js';
import { createPoller, loadSettings, prometheusCandidates, seriesStepSec } from './settings.js';

/** Data younger than this is served from the shared store on mount without re-fetching. */
export const STALE_MS = 5000;

export type AmdGpuContextValue = ClusterSnapshot & { refresh: () => void };

const AmdGpuContext = createContext<AmdGpuContextValue | null>(null);

export function useAmdGpuContext(): AmdGpuContextValue {
  const ctx = useContext(AmdGpuContext);
  if (!ctx) {
    throw new Error('useAmdGpuContext must be used within an AmdGpuDataProvider');
  }
  return ctx;
}

function request(path: string): Promise<unknown> {
  return ApiProxy.request(path);
}

/** The shared store of the current cluster (created on first use). */
export function storeFor(cluster: string) {
  const settings = loadSettings();
  return getSharedStore(`${cluster}|${settings.requestTimeoutMs}`, () =>
    createClusterStore({ request, timeoutMs: settings.requestTimeoutMs })
  );
}

const metricsSources: Record<string, ReturnType<typeof createMetricsSource>> = {};

/**
 * The shared Prometheus client of the current cluster (its discovery cache
 * lives here). Keyed by the settings that shape it, so saving new settings
 * takes effect on the next mount.
 */
export function metricsSourceFor(cluster: string) {
  const settings = loadSettings();
  const key = `${cluster}|${JSON.stringify(settings.prometheus)}|${settings.requestTimeoutMs}`;
  if (!metricsSources[key]) {
    metricsSources[key] = createMetricsSource({
      request,
      services: prometheusCandidates(settings),
      timeoutMs: settings.requestTimeoutMs,
    });
  }
  return metricsSources[key];
}

export function AmdGpuDataProvider({ children }: { children: React.ReactNode }) {
  const store = storeFor(clusterKey());

  // Track 1 — reactive lists from Headlamp (all namespaces for pods).
  const [allNodes, nodeError] = K8s.ResourceClasses.Node.useList();
  const [allPods, podError] = K8s.ResourceClasses.Pod.useList({ namespace: '' });

  useEffect(() => {
    store.setNodes((allNodes as unknown[] | null) ?? null, nodeError ? String(nodeError) : null);
  }, [store, allNodes, nodeError]);
  useEffect(() => {
    store.setPods((allPods as unknown[] | null) ?? null, podError ? String(podError) : null);
  }, [store, allPods, podError]);

  // Track 2 — imperative CRD / operator-pod fetch, shared and deduplicated.
  useEffect(() => {
    void store.revalidate(STALE_MS);
  }, [store]);

  // Optional auto-refresh (settings; the reference only refreshes on click).
  const refreshIntervalSec = loadSettings().refreshIntervalSec;
  useEffect(() => {
    const poller = createPoller(refreshIntervalSec);
    poller.start(() => store.revalidate(STALE_MS));
    return () => poller.stop();
  }, [store, refreshIntervalSec]);

  const snapshot = useSyncExternalStore(store.subscribe, store.getSnapshot);
  const value = useMemo<AmdGpuContextValue>(
    () => ({
      ...snapshot,
      refresh: () => {
        void store.refresh();
      },
    }),
    [snapshot, store]
  );

  return <AmdGpuContext.Provider value={value}>{children}</AmdGpuContext.Provider>;
}

// ---------------------------------------------------------------------------
// Metrics hook (reference: MetricsPage.tsx:191-231 state + effect)
// ---------------------------------------------------------------------------

export interface GpuMetricsState {
  metrics: GpuMetrics | null;
  series: {
    rangeSec: number;
    power: Record<string, Array<[number, number]>>;
    vram: Record<string, Array<[number, number]>>;
  } | null;
  fetchError: string | null;
  fetching: boolean;
  refresh: () => void;
}

export const PROMETHEUS_UNREACHABLE =
  'Could not reach Prometheus. Ensure kube-prometheus-stack is installed in the monitoring namespace.';

/**
 * Fetch GPU telemetry + power/HBM series. Unlike the reference it does not
 * wait for the cluster context to finish loading: the two are independent
 * and fetched in parallel. Stale responses are dropped on unmount / re-run.
 */
export function useGpuMetrics(enabled = true, withSeries = true): GpuMetricsState {
  const source = metricsSourceFor(clusterKey());
  const settings = loadSettings();
  const [state, setState] = useState<Omit<GpuMetricsState, 'refresh'>>({
    metrics: null,
    series: null,
    fetchError: null,
    fetching: false,
  });
  const [seq, setSeq] = useState(0);

  useEffect(() => {
    if (!enabled) return;
    let cancelled = false;
    setState(s => ({ ...s, fetching: true, fetchError: null }));
    Promise.all([
      source.fetchGpuMetrics(),
      withSeries ? source.fetchSeries(settings.seriesMinutes * 60, seriesStepSec(settings)) : Promise.resolve(null),
    ])
      .then(([metrics, series]) => {
        if (cancelled) return;
        setState({ metrics, series, fetching: false, fetchError: metrics ? null : PROMETHEUS_UNREACHABLE });
      })
      .catch((e: unknown) => {
        if (cancelled) return;
        setState(s => ({ ...s, fetching: false, fetchError: e instanceof Error ? e.message : String(e) }));
      });
    return () => {
      cancelled = true;
    };
  }, [enabled, withSeries, seq, source, settings.seriesMinutes]);

  useEffect(() => {
    if (!enabled) return;
    const poller = createPoller(settings.refreshIntervalSec);
    poller.start(() => setSeq(s => s + 1));
    return () => poller.stop();
  }, [enabled, settings.refreshIntervalSec]);

  return useMemo(() => ({ ...state, refresh: () => setSeq(s => s + 1) }), [state]);
}

/**
 * A metrics fetch narrower than the cluster-wide snapshot, re-run by the
 * auto-refresh poller and by `refresh()`. `key` null fetches nothing; a new
 * key drops the previous key's in-flight answer.
 */
function useScopedMetrics(key: string | null, fetch: () => Promise<GpuMetrics | null>): GpuMetricsState {
  const refreshIntervalSec = loadSettings().refreshIntervalSec;
  const [state, setState] = useState<Omit<GpuMetricsState, 'refresh'>>({
    metrics: null,
    series: null,
    fetchError: null,
    fetching: false,
  });
  const [seq, setSeq] = useState(0);

  useEffect(() => {
    if (key === null) return;
    let cancelled = false;
    setState(s => ({ ...s, fetching: true, fetchError: null }));
    fetch()
      .then(metrics => {
        if (cancelled) return;
        setState({ metrics, series: null, fetching: false, fetchError: metrics ? null : PROMETHEUS_UNREACHABLE });
      })
      .catch((e: unknown) => {
        if (cancelled) return;
        setState(s => ({ ...s, fetching: false, fetchError: e instanceof Error ? e.message : String(e) }));
      });
    return () => {
      cancelled = true;
    };
    // `fetch` is rebuilt every render; `key` names what it fetches.
    // eslint-disable-next-line react-hooks/exhaustive-deps
  }, [key, seq]);

  useEffect(() => {
    if (key === null) return;
    const poller = createPoller(refreshIntervalSec);
    poller.start(() => setSeq(s => s + 1));
    return () => poller.stop();
  }, [key, refreshIntervalSec]);

  return useMemo(() => ({ ...state, refresh: () => setSeq(s => s + 1) }), [state]);
}

/**
 * Telemetry of one node's GPUs for the native Node / Pod detail pages: a
 * `hostname`-scoped query through the shared client (metrics.js
 * fetchNodeMetrics), so a detail page costs the same few KB on a 500-node
 * cluster as on one node. `nodeName` null (or `enabled` false) fetches
 * nothing.
 */
export function useNodeGpuMetrics(nodeName: string | null, enabled = true): GpuMetricsState {
  const source = metricsSourceFor(clusterKey());
  const active = enabled && !!nodeName;
  return useScopedMetrics(active ? `node|${clusterKey()}|${nodeName}` : null, () =>
    source.fetchNodeMetrics(nodeName as string)
  );
}

/**
 * Pod → GPU attribution for the Pods page (metrics.js fetchGpuOwners): one
 * series per allocated GPU instead of the whole cluster's telemetry.
 */
export function useGpuOwners(enabled = true): GpuMetricsState {
  const source = metricsSourceFor(clusterKey());
  return useScopedMetrics(enabled ? `owners|${clusterKey()}` : null, () => source.fetchGpuOwners());
}
