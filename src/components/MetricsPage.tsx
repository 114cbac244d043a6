/**
 * MetricsPage — MI355X power, HBM, activity, temperature, RAS and xGMI telemetry (reference MetricsPage.tsx, C9).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.MetricsPage;
