/**
 * NodeDetailSection — injected into Headlamp's native Node detail page
 * (reference NodeDetailSection.tsx, SURVEY.md C10). Renders nothing for
 * non-AMD nodes. Reads the shared store, so it costs no extra fetch when a
 * plugin page already loaded the cluster.
 */
import React from 'react';
import { useAmdGpuContext } from '../api/AmdGpuDataContext';
import { nodeDetailView } from '../view/pages.js';
import { Section } from './View';

export default function NodeDetailSection({ resource }: { resource: unknown }) {
  const ctx = useAmdGpuContext();
  const section = nodeDetailView(resource, ctx);
  return section ? <Section s={section} /> : null;
}
