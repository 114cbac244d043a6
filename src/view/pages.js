/**
 * Page view-models: snapshot → View IR. Pure functions, no React, no I/O.
 *
 * One module per reference page / integration (SURVEY.md C5–C12):
 *   overviewView        ./pages/overview.js       ← src/components/OverviewPage.tsx
 *   devicePluginsView   ./pages/devicePlugins.js  ← src/components/DevicePluginsPage.tsx
 *   nodesView           ./pages/nodes.js          ← src/components/NodesPage.tsx
 *   podsView            ./pages/pods.js           ← src/components/PodsPage.tsx
 *   metricsView         ./pages/metricsPage.js    ← src/components/MetricsPage.tsx
 *   nodeDetailView      ./pages/details.js        ← src/components/NodeDetailSection.tsx
 *   podDetailView       ./pages/details.js        ← src/components/PodDetailSection.tsx
 *   nodeColumns         ./pages/details.js        ← src/components/integrations/NodeColumns.tsx
 * with the shared memo, caches and cells in ./pages/common.js and the pager
 * in ./pages/paging.js.
 *
 * Section titles, loader texts, empty states and refresh aria-labels keep
 * the reference's wording with AMD vocabulary, so the reference's component
 * assertions translate one-for-one. Behavioural differences are listed in
 * each function's comment.
 *
 * `opts.now` (ms epoch) makes ages deterministic in tests.
 */

export {
  allocationBar,
  BRAND,
  clearViewMemo,
  eccCell,
  formatWindow,
  hbmBar,
  powerBar,
  seriesMeans,
  tempCell,
} from './pages/common.js';
export {
  NODE_SORTS,
  nodePage,
  NODES_PER_PAGE,
  nodeSortOf,
  POD_SORTS,
  podPage,
  PODS_PER_PAGE,
  podSortOf,
  RANKED_NODE_SORTS,
  RANKED_POD_SORTS,
} from './pages/paging.js';
export {
  ACTIVE_PODS_LIMIT,
  HELM_INSTALL,
  OPERATOR_DOCS,
  OVERVIEW_PLUGIN_PODS,
  overviewView,
  partitionModeDistribution,
} from './pages/overview.js';
export {
  devicePluginsView,
} from './pages/devicePlugins.js';
export {
  formatTaints,
  matrixBlock,
  nodePowerKeys,
  nodeTempKeys,
  nodeReadyCell,
  nodesView,
  slotsBlock,
  telemetryScope,
  visibleNodeNames,
} from './pages/nodes.js';
export {
  gpuContainerLines,
  ownersScope,
  podGpuAssignments,
  podPowerText,
  podsView,
} from './pages/pods.js';
export {
  ALL_NODES_SERIES,
  metricAvailabilitySection,
  metricsView,
  nodesReporting,
  nodesReportingCount,
} from './pages/metricsPage.js';
export {
  formatEnergy,
  nodeColumns,
  nodeDetailView,
  podDetailView,
  seriesEnergyJoules,
} from './pages/details.js';
