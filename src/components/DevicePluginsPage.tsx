/**
 * DevicePluginsPage — AMD GPU Operator DeviceConfigs and operand pods (reference DevicePluginsPage.tsx, C6).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.DevicePluginsPage;
