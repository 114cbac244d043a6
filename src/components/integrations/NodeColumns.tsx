/**
 * NodeColumns — GPU columns appended to Headlamp's native Nodes table
 * (reference integrations/NodeColumns.tsx, SURVEY.md C12): GPU Model,
 * GPU Devices and GPU HBM. Each row is classified once for all columns.
 */
import React from 'react';
import { nodeColumns } from '../../view/pages.js';
import { Value } from '../View';

export function buildNodeGpuColumns() {
  return nodeColumns().map((c: { label: string; getter: (r: unknown) => unknown }) => ({
    label: c.label,
    getter: (resource: unknown) => <Value v={c.getter(resource)} />,
  }));
}
