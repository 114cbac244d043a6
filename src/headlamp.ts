/**
 * The plugin bound to the real React and the Headlamp plugin library — the
 * one place the host runtime meets the plugin's code (src/plugin.js), and its
 * one TypeScript surface besides the entry (src/index.tsx). Types come from
 * src/plugin.d.ts.
 *
 * The reference spreads this surface over one module per component
 * (src/components/*.tsx, src/components/integrations/NodeColumns.tsx,
 * src/api/IntelGpuDataContext.tsx). Here they are named exports of the
 * binding: the pages and detail sections, the Nodes-table columns, the
 * provider and its hooks, and the IR renderer (src/view/react.js).
 */
import * as lib from '@kinvolk/headlamp-plugin/lib';
import * as CommonComponents from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import React from 'react';
import { createPlugin } from './plugin.js';

export const plugin = createPlugin({ React, lib, CommonComponents });

export const {
  OverviewPage,
  DevicePluginsPage,
  NodesPage,
  PodsPage,
  MetricsPage,
  NodeDetailSection,
  PodDetailSection,
  SettingsPage,
  buildNodeGpuColumns,
  AmdGpuDataProvider,
  useAmdGpuContext,
} = plugin;
export const { useGpuMetrics, useNodeGpuMetrics, useGpuOwners, storeFor, metricsSourceFor } = plugin.core;
export const { Page, Section, Value, Block } = plugin.view;
export { STALE_MS, PROMETHEUS_UNREACHABLE, PROMETHEUS_FORBIDDEN } from './api/providerCore.js';
