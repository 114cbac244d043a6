/** Types of the provider core (./providerCore.js). */
import type { ComponentType, Context, ReactNode } from 'react';
import type { AmdGpuContextValue, GpuMetrics, GpuMetricsState } from './types';

export const STALE_MS: number;
export const PROMETHEUS_UNREACHABLE: string;
export const PROMETHEUS_FORBIDDEN: string;
export const OUTSIDE_PROVIDER: string;
/** Needs of a provider that reads the store and mounts nothing. */
export const READ_ONLY_NEEDS: { nodes: false; pods: false; crd: false; operatorPods: false };
/** Re-read period (s) of a scoped request standing in for an unscoped watch, when auto-refresh is off. */
export const SCOPED_POLL_SEC: number;

/** List options of a scoped list + watch (the apiserver applies them; ADR 012 checks the host passed them on). */
export interface ListOptions {
  namespace?: string;
  labelSelector?: string;
  fieldSelector?: string;
}

export interface HeadlampLibLike {
  K8s: {
    ResourceClasses: {
      Node: { useList: (opts?: ListOptions) => [unknown[] | null, unknown, ...unknown[]] };
      Pod: { useList: (opts?: ListOptions) => [unknown[] | null, unknown, ...unknown[]] };
    };
  };
  ApiProxy: { request: (path: string) => Promise<unknown> };
}

export interface ProviderDeps {
  request?: (path: string) => Promise<unknown>;
  clusterKey?: () => string;
  loadSettings?: () => { prometheus: { namespace: string; service: string; port: string } | null; refreshIntervalSec: number; requestTimeoutMs: number; seriesMinutes: number };
}

/** The shared data store (./clusterStore.js createClusterStore). */
export interface ClusterStore {
  subscribe(fn: () => void): () => void;
  getSnapshot(): Omit<AmdGpuContextValue, 'refresh'>;
  setNodes(items: unknown[] | null, error: string | null): void;
  setPods(items: unknown[] | null, error: string | null): void;
  /** A pod list feed mounted; returns its detach (operator pods come from the plugin-pod requests once none is). */
  attachPodFeed(): () => void;
  /** An operator pod feed mounted (its own scoped lists + watches); returns its detach. */
  attachOperatorFeed(): () => void;
  /** Feed the operator pods of the scoped lists (null while in flight). */
  setOperatorPods(items: unknown[] | null, error: string | null): void;
  /** The operator pods by the plugin-pod requests (a client without list hooks, or a host ignoring list options). */
  loadOperatorPods(): Promise<void>;
  refresh(): Promise<void>;
  revalidate(maxAgeMs?: number): Promise<void>;
  loadLists(which?: { nodes?: boolean; pods?: boolean }): Promise<void>;
  settled(): Promise<void>;
  hasLoaded(): boolean;
  /** A pod list feed is mounted right now. */
  podFeedMounted(): boolean;
  /** A scoped list of `kind` delivered `n` objects outside its selection (the host ignored the options). */
  noteSelectorIgnored(kind: 'nodePods' | 'operatorPods', n: number, delivery?: object): void;
  selectorsIgnored(kind: 'nodePods' | 'operatorPods'): boolean;
  counters(): {
    indexBuilds: number;
    indexPatches: number;
    subscribers: number;
    podFeeds: number;
    operatorFeeds: number;
    selectorIgnored: { nodePods: number; operatorPods: number } | null;
    [k: string]: unknown;
  };
}

export interface MetricsSource {
  /**
   * `scope`: node names of a paged view (hostname=~); `summary`: also the cluster totals (GpuMetrics.totals);
   * `small`: every GPU when the cluster has at most SMALL_CLUSTER_NODES GPU nodes, else `scope`'s (one request)
   */
  fetchGpuMetrics(
    view?: 'all' | 'gauges' | 'topology',
    opts?: { scope?: string[]; summary?: boolean; small?: boolean; rank?: { by: 'power'; page: number; per: number; filter: string } }
  ): Promise<GpuMetrics | null>;
  fetchNodeMetrics(nodeName: string): Promise<GpuMetrics | null>;
  /** `pods`: "namespace/name" keys of one page of the Pods table; `small` as in fetchGpuMetrics */
  fetchGpuOwners(
    opts?: { pods?: string[]; small?: boolean; preview?: number; rank?: { by: 'power'; page: number; per: number; filter: string } }
  ): Promise<GpuMetrics | null>;
  failureReason(): 'forbidden' | 'unreachable';
  fetchPodSeries(namespace: string, pod: string, rangeSec: number, stepSec: number): Promise<{ rangeSec: number; stepSec: number; power: Array<[number, number]> } | null>;
  fetchNodeSeries(nodeName: string, rangeSec: number, stepSec: number): Promise<{ rangeSec: number; stepSec: number; power: Array<[number, number]> } | null>;
  fetchSeries(rangeSec: number, stepSec: number, scope?: string[], small?: boolean): Promise<GpuMetricsState['series']>;
}

export interface ProviderCore {
  Context: Context<AmdGpuContextValue | null>;
  /** `needs`: what the page draws — only those lists / requests are mounted (default: all) */
  AmdGpuDataProvider: ComponentType<{ children?: ReactNode; needs?: { nodes?: boolean; pods?: boolean; crd?: boolean; operatorPods?: boolean } }>;
  /** Mounts the pod list + watch into the current cluster's store (a page whose provider does not feed pods) */
  PodListHere: ComponentType<Record<string, never>>;
  useAmdGpuContext(): AmdGpuContextValue;
  useGpuMetrics(
    enabled?: boolean,
    withSeries?: boolean,
    view?: 'all' | 'gauges' | 'topology',
    scope?: string[],
    small?: boolean,
    rank?: { by: 'power'; page: number; per: number; filter: string }
  ): GpuMetricsState;
  useNodeGpuMetrics(nodeName: string | null, enabled?: boolean): GpuMetricsState;
  useGpuOwners(
    enabled?: boolean,
    pods?: string[],
    small?: boolean,
    rank?: { by: 'power'; page: number; per: number; filter: string },
    /** with `small` and no page yet: the pods drawing the most power on a larger cluster (a partial page) */
    preview?: number
  ): GpuMetricsState;
  usePodGpuSeries(namespace: string | null, pod: string | null, enabled?: boolean): GpuMetricsState;
  useNodeGpuSeries(nodeName: string | null, enabled?: boolean): GpuMetricsState;
  /**
   * One node's pods for a Node detail section no page feeds: the host's list + watch scoped by `spec.nodeName`
   * (or, on a host ignoring list options, the field-selected request re-read), seeded by the store's last list.
   * Returns [what nodeDetailView reads, the feed element the caller must render].
   */
  useNodePods(
    nodeName: string
  ): [{ loading: boolean; gpuPods: unknown[]; podsState: 'pending' | 'ready' | 'error'; error: string | null }, ReactNode];
  /** A mounted pod feed keeps the shared store current (re-renders the caller when that flips). */
  usePodsLive(): boolean;
  storeFor(cluster: string): ClusterStore;
  metricsSourceFor(cluster: string): MetricsSource;
  /** The current cluster's key (per-cluster state: stores, view state). */
  clusterKey(): string;
}

export function createProviderCore(React: unknown, lib: HeadlampLibLike, deps?: ProviderDeps): ProviderCore;

/** [items, error] from a Headlamp list hook: the `[items, error]` tuple or a `{items, error | errors, isLoading}` object. */
export function listResult(res: unknown): [unknown[] | null, unknown];
