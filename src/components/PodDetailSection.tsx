/**
 * PodDetailSection — injected into Headlamp's native Pod detail page
 * (reference PodDetailSection.tsx, SURVEY.md C11). Needs no cluster data, so
 * it mounts no provider; for GPU pods it reads the shared Prometheus client
 * (cached discovery, one query) to show live telemetry of the GPUs the pod
 * holds.
 */
import React from 'react';
import { useGpuMetrics } from '../api/AmdGpuDataContext';
import { isGpuRequestingPod, unwrapKubeObject } from '../api/amdgpu.js';
import { podDetailView } from '../view/pages.js';
import { Section } from './View';

export default function PodDetailSection({ resource }: { resource: unknown }) {
  const gpuPod = isGpuRequestingPod(unwrapKubeObject(resource));
  const m = useGpuMetrics(gpuPod, false);
  const section = podDetailView(resource, { metrics: m.metrics });
  return section ? <Section s={section} /> : null;
}
