/**
 * PodsPage — pods requesting amd.com/* resources (reference PodsPage.tsx, SURVEY.md C8).
 * With exporter telemetry the pod table also names the physical GPUs each
 * pod holds (exporter pod labels) — fetched as attribution only, one series
 * per allocated GPU, not the whole cluster's telemetry.
 */
import React from 'react';
import { useAmdGpuContext, useGpuOwners } from '../api/AmdGpuDataContext';
import { podsView } from '../view/pages.js';
import { Page } from './View';

export default function PodsPage() {
  const ctx = useAmdGpuContext();
  const m = useGpuOwners();
  const refresh = () => {
    ctx.refresh();
    m.refresh();
  };
  return <Page vm={podsView(ctx, { metrics: m.metrics })} onRefresh={refresh} />;
}
