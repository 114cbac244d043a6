/**
 * Sidebar entries and routes as data, so registration is testable without
 * Headlamp (the reference's registration is untested, SURVEY.md §4 gaps).
 * Reference: src/index.tsx:35-81 (sidebar), :87-145 (routes).
 *
 * The root label is the product name, not the URL slug (reference quirk Q13).
 */

export const ROOT = 'amd-gpu';
export const BASE_URL = '/amd-gpu';

/** @type {Array<{parent: string|null, name: string, label: string, url: string, icon: string}>} */
export const SIDEBAR = [
  { parent: null, name: ROOT, label: 'AMD GPU', url: BASE_URL, icon: 'mdi:expansion-card' },
  { parent: ROOT, name: ROOT + '-overview', label: 'Overview', url: BASE_URL, icon: 'mdi:view-dashboard' },
  { parent: ROOT, name: ROOT + '-device-plugins', label: 'Device Plugins', url: BASE_URL + '/device-plugins', icon: 'mdi:chip' },
  { parent: ROOT, name: ROOT + '-nodes', label: 'GPU Nodes', url: BASE_URL + '/nodes', icon: 'mdi:server' },
  { parent: ROOT, name: ROOT + '-pods', label: 'GPU Pods', url: BASE_URL + '/pods', icon: 'mdi:cube-outline' },
  { parent: ROOT, name: ROOT + '-metrics', label: 'Metrics', url: BASE_URL + '/metrics', icon: 'mdi:chart-line' },
];

/** @type {Array<{path: string, sidebar: string, name: string, page: string}>} */
export const ROUTES = [
  { path: BASE_URL, sidebar: ROOT + '-overview', name: ROOT + '-overview', page: 'overview' },
  { path: BASE_URL + '/device-plugins', sidebar: ROOT + '-device-plugins', name: ROOT + '-device-plugins', page: 'device-plugins' },
  { path: BASE_URL + '/nodes', sidebar: ROOT + '-nodes', name: ROOT + '-nodes', page: 'nodes' },
  { path: BASE_URL + '/pods', sidebar: ROOT + '-pods', name: ROOT + '-pods', page: 'pods' },
  { path: BASE_URL + '/metrics', sidebar: ROOT + '-metrics', name: ROOT + '-metrics', page: 'metrics' },
];

/** Headlamp table id the GPU columns are appended to. */
export const NODES_TABLE_ID = 'headlamp-nodes';

/**
 * Apply a columns-processor call the way Headlamp does: append our columns
 * to the native Nodes table only.
 */
export function processColumns(args, buildColumns) {
  if (args && args.id === NODES_TABLE_ID) return args.columns.concat(buildColumns());
  return args.columns;
}
