/**
 * NodeDetailSection — Section on the native Node detail page (reference NodeDetailSection.tsx, C10).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.NodeDetailSection;
