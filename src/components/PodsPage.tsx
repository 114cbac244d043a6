/**
 * PodsPage — pods requesting amd.com/* resources (reference PodsPage.tsx, SURVEY.md C8).
 */
import React from 'react';
import { useAmdGpuContext } from '../api/AmdGpuDataContext';
import { podsView } from '../view/pages.js';
import { Page } from './View';

export default function PodsPage() {
  const ctx = useAmdGpuContext();
  return <Page vm={podsView(ctx)} onRefresh={ctx.refresh} />;
}
