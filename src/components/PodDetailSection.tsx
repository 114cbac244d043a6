/**
 * PodDetailSection — injected into Headlamp's native Pod detail page
 * (reference PodDetailSection.tsx, SURVEY.md C11). Needs no cluster data, so
 * it mounts no provider; for a scheduled GPU pod it reads the shared
 * Prometheus client (cached discovery) for the telemetry of the pod's node
 * only — a `hostname`-scoped query, a few KB whatever the cluster size — and
 * shows the live power / GFX / HBM of the GPUs the pod holds.
 */
import React from 'react';
import { useNodeGpuMetrics } from '../api/AmdGpuDataContext';
import { get, isGpuRequestingPod, unwrapKubeObject } from '../api/amdgpu.js';
import { podDetailView } from '../view/pages.js';
import { Section } from './View';

export default function PodDetailSection({ resource }: { resource: unknown }) {
  const raw = unwrapKubeObject(resource);
  const gpuPod = isGpuRequestingPod(raw);
  const nodeName = gpuPod ? (get(raw, ['spec', 'nodeName'], null) as string | null) : null;
  const m = useNodeGpuMetrics(nodeName, gpuPod);
  const section = podDetailView(resource, { metrics: m.metrics });
  return section ? <Section s={section} /> : null;
}
