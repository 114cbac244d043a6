/**
 * NodeColumns — GPU Model / GPU Devices / GPU HBM columns appended to the
 * native Nodes table (reference integrations/NodeColumns.tsx, SURVEY.md C12).
 * Implementation: src/plugin.js (`buildNodeGpuColumns`) over
 * src/view/pages/details.js (`nodeColumns`).
 */
import { plugin } from '../../headlamp';

export const buildNodeGpuColumns = plugin.buildNodeGpuColumns;
