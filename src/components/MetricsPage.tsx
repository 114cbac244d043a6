/**
 * MetricsPage — MI355X power, HBM, activity, temperature and xGMI telemetry
 * from Prometheus (reference MetricsPage.tsx, SURVEY.md C9).
 *
 * METRIC AVAILABILITY on AMD (the reference's i915 page lists most of these
 * as unavailable; amdgpu exposes all of them):
 *   Power (W)            gpu_power_usage (AMD Device Metrics Exporter) or
 *                        amdgpu hwmon power (power1_input on MI355X) via node-exporter
 *   HBM used / total     gpu_used_vram / gpu_total_vram, or node-exporter
 *                        --collector.drm node_drm_memory_vram_{used,size}_bytes
 *   GFX activity (%)     gpu_gfx_activity, or node_drm_gpu_busy_percent
 *   HBM activity (%)     gpu_umc_activity
 *   xGMI throughput      xgmi_neighbor_N_tx_throughput (7 links per GPU)
 *   Pod → GPU mapping    exporter pod / namespace labels
 */
import React from 'react';
import { useAmdGpuContext, useGpuMetrics } from '../api/AmdGpuDataContext';
import { metricsView } from '../view/pages.js';
import { Page } from './View';

export default function MetricsPage() {
  const ctx = useAmdGpuContext();
  const m = useGpuMetrics(true);
  return <Page vm={metricsView(ctx, m)} onRefresh={m.refresh} />;
}
