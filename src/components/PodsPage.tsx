/**
 * PodsPage — Pods requesting amd.com/* resources (reference PodsPage.tsx, C8).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.PodsPage;
