/** Types of the assembled plugin (./plugin.js). */
import type { ComponentType, ReactElement } from 'react';
import type { HeadlampLibLike, ProviderCore, ProviderDeps } from './api/providerCore';
import type { AmdGpuContextValue } from './api/types';
import type { Renderer } from './view/react';

export const PLUGIN_NAME: string;

/** What each page draws, hence what its route mounts (lists, DeviceConfig request). */
export const PAGE_NEEDS: Readonly<Record<'overview' | 'device-plugins' | 'nodes' | 'pods' | 'metrics', Readonly<{ nodes: boolean; pods: boolean; crd: boolean; operatorPods?: boolean }>>>;

export interface PluginEnv {
  React: unknown;
  lib: HeadlampLibLike;
  CommonComponents: unknown;
  deps?: ProviderDeps;
  settingsStorage?: { load: () => unknown; save: (v: unknown) => unknown };
  /** Where the pages keep their pager state (default: sessionStorage). */
  viewStorage?: { getItem: (k: string) => string | null; setItem: (k: string, v: string) => void } | null;
}

export interface NodeColumn {
  label: string;
  getter: (resource: unknown) => ReactElement;
}

export interface Plugin {
  core: ProviderCore;
  view: Renderer;
  AmdGpuDataProvider: ProviderCore['AmdGpuDataProvider'];
  useAmdGpuContext(): AmdGpuContextValue;
  OverviewPage: ComponentType;
  DevicePluginsPage: ComponentType;
  NodesPage: ComponentType;
  PodsPage: ComponentType;
  MetricsPage: ComponentType;
  NodeDetailSection: ComponentType<{ resource: unknown }>;
  /** Node detail on a cold store: the node's own pods by one field-selected request */
  NodeDetailCold: ComponentType<{ resource: unknown }>;
  PodDetailSection: ComponentType<{ resource: unknown }>;
  SettingsPage: ComponentType<{ data?: Record<string, unknown>; onDataChange?: (data: Record<string, unknown>) => void }>;
  buildNodeGpuColumns(): NodeColumn[];
  pages: Record<'overview' | 'device-plugins' | 'nodes' | 'pods' | 'metrics', ComponentType>;
  routeComponent(page: string): ComponentType;
  nodeDetailSectionFor(args: { resource?: { kind?: string } }): ReactElement | null;
  podDetailSectionFor(args: { resource?: { kind?: string } }): ReactElement | null;
}

export interface HeadlampRegistry extends HeadlampLibLike {
  registerSidebarEntry(e: { parent: string | null; name: string; label: string; url: string; icon: string }): void;
  registerRoute(r: { path: string; sidebar: string; name: string; exact: boolean; component: ComponentType }): void;
  registerDetailsViewSection(f: (args: { resource?: { kind?: string } }) => ReactElement | null): void;
  registerResourceTableColumnsProcessor(f: (args: { id: string; columns: unknown[] }) => unknown[]): void;
  registerPluginSettings?: (name: string, c: ComponentType, displaySaveButton: boolean) => void;
}

export function createPlugin(env: PluginEnv): Plugin;

export function registerPlugin(
  lib: HeadlampRegistry,
  plugin: Plugin
): { sidebar: number; routes: number; detailSections: number; columnProcessors: number; settings: boolean };
