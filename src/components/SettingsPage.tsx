/**
 * SettingsPage — Plugin settings (no reference analog: its settings are compile-time constants).
 * Implementation: src/plugin.js (`createPlugin`).
 */
import { plugin } from '../headlamp';

export default plugin.SettingsPage;
