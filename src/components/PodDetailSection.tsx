/**
 * PodDetailSection — Section on the native Pod detail page (reference PodDetailSection.tsx, C11).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.PodDetailSection;
