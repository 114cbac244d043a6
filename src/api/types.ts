/**
 * Typed shapes of the Kubernetes / AMD objects the plugin reads — the fields
 * it actually uses, nothing more. Runtime narrowing from `unknown` happens in
 * the `is*` guards of ./k8sCore.js, ./amdNodes.js and ./amdPods.js; these interfaces describe what a value is
 * once a guard has accepted it.
 *
 * Reference analog: src/api/k8s.ts:37-50 (KubeObjectMeta, KubeObject),
 * :56-80 (CRD), :92-122 (Node), :209-247 (Pod), :315-318 (KubeList)
 * — SURVEY.md C2.2, C2.3, C2.4, C2.8, C2.12.
 */

// ---------------------------------------------------------------------------
// Generic
// ---------------------------------------------------------------------------

export interface KubeObjectMeta {
  name: string;
  namespace?: string;
  uid?: string;
  resourceVersion?: string;
  creationTimestamp?: string;
  labels?: Record<string, string>;
  annotations?: Record<string, string>;
}

export interface KubeObject {
  apiVersion?: string;
  kind?: string;
  metadata: KubeObjectMeta;
}

export interface KubeList<T> {
  items: T[];
  metadata?: { resourceVersion?: string };
}

/** Headlamp `useList()` returns class instances that keep the raw JSON here. */
export interface KubeObjectWrapper<T> {
  jsonData: T;
}

export type Status = 'success' | 'warning' | 'error';

// ---------------------------------------------------------------------------
// AMD GPU Operator DeviceConfig (amd.com/v1alpha1) — fields used, verify per release
// ---------------------------------------------------------------------------

export interface OperandStatus {
  nodesMatchingSelectorNumber?: number;
  desiredNumber?: number;
  availableNumber?: number;
}

export interface DeviceConfigSpec {
  driver?: { enable?: boolean; version?: string; image?: string };
  devicePlugin?: { devicePluginImage?: string; nodeLabellerImage?: string; enableNodeLabeller?: boolean };
  metricsExporter?: { enable?: boolean; port?: number; image?: string; serviceType?: string; nodePort?: number };
  testRunner?: { enable?: boolean };
  selector?: Record<string, string>;
}

export interface DeviceConfigStatus {
  devicePlugin?: OperandStatus;
  nodeLabeller?: OperandStatus;
  metricsExporter?: OperandStatus;
  driver?: OperandStatus;
}

export interface DeviceConfig extends KubeObject {
  kind: 'DeviceConfig';
  spec?: DeviceConfigSpec;
  status?: DeviceConfigStatus;
}

// ---------------------------------------------------------------------------
// Node
// ---------------------------------------------------------------------------

export type NodeResources = Record<string, string | undefined>;

export interface NodeCondition {
  type: string;
  status: string;
  reason?: string;
  message?: string;
  lastHeartbeatTime?: string;
}

export interface NodeStatus {
  capacity?: NodeResources;
  allocatable?: NodeResources;
  conditions?: NodeCondition[];
  nodeInfo?: {
    kernelVersion?: string;
    osImage?: string;
    architecture?: string;
    kubeletVersion?: string;
    containerRuntimeVersion?: string;
  };
}

export interface NodeSpec {
  taints?: Array<{ key: string; effect: string; value?: string }>;
  unschedulable?: boolean;
}

export interface AmdGpuNode extends KubeObject {
  spec?: NodeSpec;
  status?: NodeStatus;
}

/** Result of getNodeGpuModel(). */
export interface GpuModel {
  product: string;
  shortName: string;
  fromLabels: boolean;
  computePartition: string | null;
  memoryPartition: string | null;
  vram: string;
  cuCount: number;
}

// ---------------------------------------------------------------------------
// Pod
// ---------------------------------------------------------------------------

export interface ResourceRequirements {
  requests?: Record<string, string>;
  limits?: Record<string, string>;
}

export interface ContainerSpec {
  name: string;
  image?: string;
  resources?: ResourceRequirements;
  /** `Always` marks a restartable (sidecar) init container. */
  restartPolicy?: string;
}

export interface ContainerStatus {
  name: string;
  ready: boolean;
  restartCount: number;
  image?: string;
  state?: {
    running?: { startedAt?: string };
    waiting?: { reason?: string; message?: string };
    terminated?: { exitCode?: number; reason?: string };
  };
}

export interface PodSpec {
  nodeName?: string;
  containers?: ContainerSpec[];
  initContainers?: ContainerSpec[];
}

export interface PodStatus {
  phase?: string;
  conditions?: Array<{ type: string; status: string; reason?: string }>;
  containerStatuses?: ContainerStatus[];
  initContainerStatuses?: ContainerStatus[];
}

export interface AmdGpuPod extends KubeObject {
  spec?: PodSpec;
  status?: PodStatus;
}

/** One AMD resource entry of a container (containerGpuEntries()). */
export interface ContainerGpuEntry {
  key: string;
  request: string | null;
  limit: string | null;
  effective: number;
}

// ---------------------------------------------------------------------------
// Cluster index (buildClusterIndex())
// ---------------------------------------------------------------------------

export interface NodeStats {
  capacity: number;
  allocatable: number;
  inUse: number;
  pods: number;
  ready: boolean;
  physicalGpus: number;
  partitionsPerGpu: number;
}

export interface ClusterIndex {
  podsByNode: Map<string, AmdGpuPod[]>;
  nodeStats: Map<string, NodeStats>;
  totals: {
    nodes: number;
    readyNodes: number;
    capacity: number;
    allocatable: number;
    inUse: number;
    free: number;
    partitions: number;
    physicalGpus: number;
    hbmBytes: number;
    hbmAllocatedBytes: number;
    utilizationPct: number;
  };
  phases: { Running: number; Pending: number; Succeeded: number; Failed: number; Other: number };
}

// ---------------------------------------------------------------------------
// Store snapshot (clusterStore.js getSnapshot()) — the context value minus `refresh`
// ---------------------------------------------------------------------------

export type ListState = 'unknown' | 'pending' | 'ready' | 'error';

export interface ClusterSnapshot {
  deviceConfigs: DeviceConfig[];
  pluginInstalled: boolean;
  gpuNodes: AmdGpuNode[];
  gpuPods: AmdGpuPod[];
  pluginPods: AmdGpuPod[];
  crdAvailable: boolean;
  /** The DeviceConfig list was refused (401 / 403) rather than absent (404). */
  crdForbidden: boolean;
  /** true until the node and pod lists settled (arrived or failed) and the first CRD fetch is in */
  loading: boolean;
  /** the node list has not settled yet (pages that draw nodes show their loader) */
  nodesLoading: boolean;
  /** the pod list has not settled yet (pod-derived sections show a loader; the rest renders) */
  podsLoading: boolean;
  /** the first DeviceConfig / operator-pod fetch is not in yet */
  crdLoading: boolean;
  /** the operator pods are not known yet (from the watched pod list, else from the plugin-pod requests) */
  pluginPodsLoading: boolean;
  nodesState: ListState;
  podsState: ListState;
  /** a refresh is in flight; the data above is still valid */
  refreshing: boolean;
  error: string | null;
  index: ClusterIndex;
  lastUpdated: number | null;
  version: number;
}

/** The provider's context value (reference IntelGpuContextValue, IntelGpuDataContext.tsx:28-52). */
export interface AmdGpuContextValue extends ClusterSnapshot {
  refresh: () => void;
}

// ---------------------------------------------------------------------------
// Telemetry (metrics.js)
// ---------------------------------------------------------------------------

export interface GpuTelemetry {
  nodeName: string;
  /** device index on the node ("0".."7") */
  gpu: string;
  instance: string;
  powerWatts: number | null;
  powerCapWatts: number | null;
  vramUsedBytes: number | null;
  vramTotalBytes: number | null;
  gfxActivityPct: number | null;
  memActivityPct: number | null;
  tempC: number | null;
  tempSlowdownC: number | null;
  eccCorrectable: number | null;
  eccUncorrectable: number | null;
  pod: string | null;
  namespace: string | null;
  /** `powerCapWatts` is the MI355X board limit because the source reported no cap */
  powerCapAssumed: boolean;
}

export interface GpuMetrics {
  source: 'amd-exporter' | 'node-exporter' | null;
  gpus: GpuTelemetry[];
  /** node → "src-dst" → GB/s */
  xgmi: Record<string, Record<string, number>>;
  /** node → "src-dst" → link type / hops (measured topology) */
  links: Record<string, Record<string, { type: string; hops: number }>>;
  fetchedAt: string;
  stale?: boolean;
  prometheusPath: string;
  /** PromQL the snapshot came from (Metrics page "Query" row). */
  query?: string;
  /** the series set the answer carries (metrics.js METRIC_VIEWS): every series, the Metrics page's, or GPU Nodes' */
  view?: 'all' | 'gauges' | 'topology';
  /** node names a paged snapshot covers (gpus holds only theirs); 'owners' on a pod → GPU attribution answer */
  scope?: string[] | 'owners';
  /** cluster totals of a paged snapshot, from server-side aggregates */
  totals?: GpuTotals;
  /** a size-guarded (small-cluster) snapshot: GPU nodes (pods) reporting, and whether that was more than a page */
  small?: { count: number; limit: number; exceeded: boolean };
  /**
   * an owners answer asked before the pod list (ownersScope `preview`) on a cluster of more than one page of owners:
   * the `per` pods drawing the most power, "namespace/pod" keys highest first, out of `count` pods holding GPUs
   */
  preview?: { per: number; count: number; order: string[]; watts: Record<string, number | null> };
  /** a power-ranked page (metrics.js rankedSnapshot): `scope` is in rank order */
  /** power order: the page Prometheus ranked; `order` ("namespace/pod" keys, highest first) on an owners answer */
  rank?: {
    by: 'power';
    page: number;
    per: number;
    filter: string;
    count: number;
    watts: Record<string, number | null>;
    order?: string[];
  };
}

/** Cluster totals (metrics.js totalsFromRows / summarizeMetrics + nodes reporting). */
export interface GpuTotals {
  gpus: number;
  withPower: number;
  nodes?: number;
  powerWatts: number;
  powerCapWatts: number;
  vramUsedBytes: number;
  vramTotalBytes: number;
  avgGfxActivityPct: number | null;
  eccCorrectable: number | null;
  eccUncorrectable: number | null;
  powerCapAssumed: number;
  tempLimitAssumed: number;
}

export interface GpuSeries {
  rangeSec: number;
  /** step of the range query (s): each sample stands for one step */
  stepSec?: number;
  power: Record<string, Array<[number, number]>>;
  vram: Record<string, Array<[number, number]>>;
  /** node names of a paged window (power / vram hold only theirs) */
  scope?: string[];
  /** the cluster-wide line of a paged window */
  total?: { power: Array<[number, number]>; vram: Array<[number, number]> };
}

export interface GpuMetricsState {
  metrics: GpuMetrics | null;
  series: GpuSeries | null;
  fetchError: string | null;
  fetching: boolean;
  refresh: () => void;
}
