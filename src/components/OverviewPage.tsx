/**
 * OverviewPage — Cluster-level MI355X dashboard (reference OverviewPage.tsx, SURVEY.md C5).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.OverviewPage;
