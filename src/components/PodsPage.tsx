/**
 * PodsPage — pods requesting amd.com/* resources (reference PodsPage.tsx, SURVEY.md C8).
 * With exporter telemetry the pod table also names the physical GPUs each
 * pod holds (exporter pod labels).
 */
import React from 'react';
import { useAmdGpuContext, useGpuMetrics } from '../api/AmdGpuDataContext';
import { podsView } from '../view/pages.js';
import { Page } from './View';

export default function PodsPage() {
  const ctx = useAmdGpuContext();
  const m = useGpuMetrics(true, false);
  const refresh = () => {
    ctx.refresh();
    m.refresh();
  };
  return <Page vm={podsView(ctx, { metrics: m.metrics })} onRefresh={refresh} />;
}
