/**
 * NodesPage — MI355X nodes: summary table, per-node cards with per-GPU
 * allocation and the xGMI neighbour matrix (reference NodesPage.tsx, SURVEY.md C7).
 * Exporter telemetry, when reachable, upgrades the slots to exact pod→GPU
 * ownership and overlays measured xGMI throughput.
 */
import React from 'react';
import { useAmdGpuContext, useGpuMetrics } from '../api/AmdGpuDataContext';
import { nodesView } from '../view/pages.js';
import { Page } from './View';

export default function NodesPage() {
  const ctx = useAmdGpuContext();
  // Telemetry only (owners, xGMI): this page draws no time series.
  const m = useGpuMetrics(true, false);
  const refresh = () => {
    ctx.refresh();
    m.refresh();
  };
  return <Page vm={nodesView(ctx, { metrics: m.metrics })} onRefresh={refresh} />;
}
