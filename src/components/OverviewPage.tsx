/**
 * OverviewPage — cluster-level MI355X dashboard (reference OverviewPage.tsx, SURVEY.md C5).
 * All content comes from `overviewView` (src/view/pages.js); this file only binds data.
 */
import React from 'react';
import { useAmdGpuContext } from '../api/AmdGpuDataContext';
import { overviewView } from '../view/pages.js';
import { Page } from './View';

export default function OverviewPage() {
  const ctx = useAmdGpuContext();
  return <Page vm={overviewView(ctx)} onRefresh={ctx.refresh} />;
}
