/**
 * AmdGpuDataContext — the provider and hooks (reference
 * src/api/IntelGpuDataContext.tsx, SURVEY.md C3), bound to React. The
 * implementation is src/api/providerCore.js.
 */
import { plugin } from '../headlamp';

export const { AmdGpuDataProvider, useAmdGpuContext } = plugin;
export const { useGpuMetrics, useNodeGpuMetrics, useGpuOwners, storeFor, metricsSourceFor } = plugin.core;
export { STALE_MS, PROMETHEUS_UNREACHABLE, PROMETHEUS_FORBIDDEN } from './providerCore.js';
