/**
 * PodDetailSection — injected into Headlamp's native Pod detail page
 * (reference PodDetailSection.tsx, SURVEY.md C11). Self-contained: needs no
 * cluster data, so it mounts no provider.
 */
import React from 'react';
import { podDetailView } from '../view/pages.js';
import { Section } from './View';

export default function PodDetailSection({ resource }: { resource: unknown }) {
  const section = podDetailView(resource);
  return section ? <Section s={section} /> : null;
}
