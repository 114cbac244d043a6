/**
 * amd-gpu — Headlamp plugin entry point (AMD Instinct MI355X).
 *
 * Registers every extension point at module load, like the reference
 * (src/index.tsx:35-182, SURVEY.md C1): sidebar root "AMD GPU" + 5 children,
 * 5 exact routes (Overview / Device Plugins / GPU Nodes / GPU Pods /
 * Metrics), the Node and Pod detail sections, the GPU columns of the native
 * `headlamp-nodes` table and the plugin settings page. The work is done by
 * `registerPlugin` (src/plugin.js); this file only binds it to Headlamp.
 */
import * as lib from '@kinvolk/headlamp-plugin/lib';
import { plugin } from './headlamp';
import { registerPlugin } from './plugin.js';

export const registered = registerPlugin(lib, plugin);
