/**
 * DevicePluginsPage — AMD GPU Operator DeviceConfigs and operand pods
 * (reference DevicePluginsPage.tsx, SURVEY.md C6).
 */
import React from 'react';
import { useAmdGpuContext } from '../api/AmdGpuDataContext';
import { devicePluginsView } from '../view/pages.js';
import { Page } from './View';

export default function DevicePluginsPage() {
  const ctx = useAmdGpuContext();
  return <Page vm={devicePluginsView(ctx)} onRefresh={ctx.refresh} />;
}
