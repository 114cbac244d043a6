/**
 * AMD Instinct MI355X domain model — pure, I/O-free.
 *
 * Everything the plugin knows about AMD GPUs in Kubernetes lives here:
 * resource names, the AMD GPU Operator `DeviceConfig` CRD, node-labeller /
 * NFD labels, pod accounting, xGMI platform facts, formatters and status
 * mappers. All inputs arriving from the API server are `unknown` and are
 * narrowed with `is*` guards at this boundary.
 *
 * Parity map (reference = privilegedescalation/headlamp-intel-gpu-plugin):
 *   constants            src/api/k8s.ts:13-31      (C2.1)
 *   CRD model + guard    src/api/k8s.ts:56-86      (C2.3)
 *   node detection       src/api/k8s.ts:125-156    (C2.5)
 *   resource extraction  src/api/k8s.ts:159-180    (C2.6)
 *   GPU "type"           src/api/k8s.ts:183-203    (C2.7) → product model
 *   pod detection        src/api/k8s.ts:250-268    (C2.9)
 *   plugin-pod detection src/api/k8s.ts:271-286    (C2.10)
 *   pod aggregation      src/api/k8s.ts:289-309    (C2.11)
 *   list envelope        src/api/k8s.ts:315-323    (C2.12)
 *   readiness            src/api/k8s.ts:329-331    (C2.13)
 *   formatters           src/api/k8s.ts:337-364    (C2.14)
 *   status mapping       src/api/k8s.ts:370-386    (C2.15)
 *
 * Deliberate departures from the reference (SURVEY.md §7.3, Appendix A):
 *   - Pod GPU demand follows the Kubernetes effective-request rule
 *     (max(Σ app + Σ sidecar, max init)) and falls back to limits for
 *     extended resources (Q3, Q4).
 *   - Node allocation counts GPUs, not pods (Q2); "free" is clamped (Q10).
 *
 * Written as ES2019 (no `?.` / `??`) so it runs unchanged under the Node 12
 * test runner in this repo and under Headlamp's vite build.
 *
 * Label / CRD names marked (verify) come from the AMD GPU Operator and
 * k8s-device-plugin manifests and must be re-checked against the deployed
 * operator version; they are centralised (./k8sCore.js) so that is a one-line change.
 *
 * The model is split by subject and re-exported here, so callers import it
 * from one module:
 *   ./k8sCore.js       constants, generic helpers, list envelope, formatters
 *   ./amdNodes.js      DeviceConfig CRD, GPU nodes, GPU model
 *   ./amdPods.js       GPU pods, demand accounting, operator pods
 *   ./clusterIndex.js  per-node / cluster aggregates, patched per watch event
 */

export {
  AMD_DEVICE_PLUGIN_POD_LABEL,
  AMD_GPU_OPERATOR_API_GROUP,
  AMD_GPU_OPERATOR_API_VERSION,
  AMD_GPU_OPERATOR_NAMESPACE,
  AMD_GPU_RESOURCE,
  AMD_LABELLER_LEGACY_PREFIX,
  AMD_LABELLER_PREFIX,
  AMD_NFD_GPU_LABEL,
  AMD_NODE_LABELLER_POD_LABEL,
  AMD_PARTITION_RESOURCE_RE,
  AMD_RESOURCE_PREFIX,
  BAR_COLORS,
  DEVICE_CONFIG_KIND,
  DEVICE_CONFIG_LIST_PATH,
  DEVICE_CONFIG_PLURAL,
  ERROR_PCT,
  formatAge,
  formatBytes,
  formatGpuResourceName,
  formatPercent,
  formatWatts,
  get,
  isKubeList,
  isNamedObject,
  isObject,
  LABEL_COMPUTE_PARTITION,
  LABEL_CU_COUNT,
  LABEL_DEVICE_ID,
  LABEL_DRIVER_VERSION,
  LABEL_FAMILY,
  LABEL_MEMORY_PARTITION,
  LABEL_PRODUCT_NAME,
  LABEL_VRAM,
  MI355X,
  nextAgeChange,
  parseCount,
  parseTime,
  pct,
  pctToColor,
  pctToStatus,
  OPERATOR_POD_LISTS,
  PLUGIN_POD_QUERIES,
  unwrapAll,
  unwrapKubeObject,
  WARN_PCT,
} from './k8sCore.js';
export {
  COMPUTE_PARTITIONS,
  countsToStatus,
  countsToText,
  deviceConfigStatus,
  deviceConfigStatusText,
  filterAmdGpuNodes,
  formatGpuModel,
  formatSelector,
  getGpuResources,
  getNodeGpuAllocatable,
  getNodeGpuCount,
  getNodeGpuModel,
  getNodePartitionCount,
  getNodePhysicalGpuCount,
  GPU_DEVICE_IDS,
  isAmdGpuNode,
  isDeviceConfig,
  isDeviceResource,
  isNodeReady,
  labellerValue,
  operandEnabled,
  OPERANDS,
  operandStatus,
  partitionsPerGpu,
  shortProductName,
} from './amdNodes.js';
export {
  containerGpuEntries,
  dedupePods,
  filterAmdGpuPluginPods,
  filterGpuRequestingPods,
  formatComponent,
  formatPodGpuRequests,
  getPodGpuCount,
  getPodGpuDemand,
  getPodGpuRequests,
  getPodRestarts,
  gpuContainers,
  gpuInitContainers,
  isAmdGpuPluginPod,
  isGpuRequestingPod,
  isPodReady,
  phaseToStatus,
  pluginPodComponent,
  podPhase,
  podWaitingMessage,
  podWaitingReason,
} from './amdPods.js';
export {
  buildClusterIndex,
  patchClusterIndex,
  podFacts,
} from './clusterIndex.js';
