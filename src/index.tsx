/**
 * amd-gpu — Headlamp plugin entry point (AMD Instinct MI355X).
 *
 * Registers every extension point at module load, like the reference
 * (src/index.tsx:35-182, SURVEY.md C1):
 *   - sidebar root "AMD GPU" + 5 children (C1.a)
 *   - 5 exact routes: Overview / Device Plugins / GPU Nodes / GPU Pods / Metrics (C1.b)
 *   - Node detail section (C1.c) and Pod detail section (C1.d)
 *   - GPU columns on the native `headlamp-nodes` table (C1.e)
 *
 * Unlike the reference, routes do not each mount a cold provider: the
 * provider is a view onto one shared per-cluster store, so switching pages
 * or opening a Node detail view renders cached data immediately and
 * revalidates in the background (reference quirk Q7).
 */

import * as pluginLib from '@kinvolk/headlamp-plugin/lib';
import {
  registerDetailsViewSection,
  registerResourceTableColumnsProcessor,
  registerRoute,
  registerSidebarEntry,
} from '@kinvolk/headlamp-plugin/lib';
import React from 'react';
import { AmdGpuDataProvider } from './api/AmdGpuDataContext';
import DevicePluginsPage from './components/DevicePluginsPage';
import { buildNodeGpuColumns } from './components/integrations/NodeColumns';
import MetricsPage from './components/MetricsPage';
import NodeDetailSection from './components/NodeDetailSection';
import NodesPage from './components/NodesPage';
import OverviewPage from './components/OverviewPage';
import PodDetailSection from './components/PodDetailSection';
import PodsPage from './components/PodsPage';
import SettingsPage from './components/SettingsPage';
import { processColumns, ROUTES, SIDEBAR } from './routes.js';

// ---------------------------------------------------------------------------
// Sidebar
// ---------------------------------------------------------------------------

for (const entry of SIDEBAR) {
  registerSidebarEntry(entry);
}

// ---------------------------------------------------------------------------
// Routes
// ---------------------------------------------------------------------------

const PAGES: Record<string, React.ComponentType> = {
  overview: OverviewPage,
  'device-plugins': DevicePluginsPage,
  nodes: NodesPage,
  pods: PodsPage,
  metrics: MetricsPage,
};

for (const route of ROUTES) {
  const Page = PAGES[route.page];
  registerRoute({
    path: route.path,
    sidebar: route.sidebar,
    name: route.name,
    exact: true,
    component: () => (
      <AmdGpuDataProvider>
        <Page />
      </AmdGpuDataProvider>
    ),
  });
}

// ---------------------------------------------------------------------------
// Native Node / Pod detail pages
// ---------------------------------------------------------------------------

registerDetailsViewSection(({ resource }: { resource?: { kind?: string } }) => {
  if (!resource || resource.kind !== 'Node') return null;
  return (
    <AmdGpuDataProvider>
      <NodeDetailSection resource={resource} />
    </AmdGpuDataProvider>
  );
});

registerDetailsViewSection(({ resource }: { resource?: { kind?: string } }) => {
  if (!resource || resource.kind !== 'Pod') return null;
  return <PodDetailSection resource={resource} />;
});

// ---------------------------------------------------------------------------
// Native Nodes table
// ---------------------------------------------------------------------------

registerResourceTableColumnsProcessor((args: { id: string; columns: unknown[] }) =>
  processColumns(args, buildNodeGpuColumns)
);

// ---------------------------------------------------------------------------
// Plugin settings (Headlamp >= 0.22 exposes registerPluginSettings; older
// hosts simply run with the defaults of src/api/settings.js)
// ---------------------------------------------------------------------------

const registerPluginSettings = (pluginLib as unknown as Record<string, unknown>)['registerPluginSettings'];
if (typeof registerPluginSettings === 'function') {
  (registerPluginSettings as (name: string, c: React.ComponentType<any>, save: boolean) => void)(
    'amd-gpu',
    SettingsPage,
    false
  );
}
