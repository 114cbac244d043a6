/**
 * NodesPage — MI355X nodes with per-GPU allocation and the xGMI matrix (reference NodesPage.tsx, C7).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.NodesPage;
