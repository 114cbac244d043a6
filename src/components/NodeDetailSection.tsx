/**
 * NodeDetailSection — injected into Headlamp's native Node detail page
 * (reference NodeDetailSection.tsx, SURVEY.md C10). Renders nothing for
 * non-AMD nodes. Reads the shared store, so it costs no extra fetch when a
 * plugin page already loaded the cluster; the node's own telemetry (exact
 * GPU owners, measured xGMI links and throughput) comes from one
 * `hostname`-scoped query.
 */
import React from 'react';
import { useAmdGpuContext, useNodeGpuMetrics } from '../api/AmdGpuDataContext';
import { isAmdGpuNode, unwrapKubeObject } from '../api/amdgpu.js';
import { nodeDetailView } from '../view/pages.js';
import { Section } from './View';

export default function NodeDetailSection({ resource }: { resource: unknown }) {
  const ctx = useAmdGpuContext();
  const raw = unwrapKubeObject(resource);
  const gpuNode = isAmdGpuNode(raw);
  const m = useNodeGpuMetrics(gpuNode ? (raw as { metadata: { name: string } }).metadata.name : null, gpuNode);
  const section = nodeDetailView(resource, ctx, { metrics: m.metrics });
  return section ? <Section s={section} /> : null;
}
