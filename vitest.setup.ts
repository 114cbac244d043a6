import { afterEach } from 'vitest';
import { resetSharedStores } from './src/api/clusterStore.js';

// Provider instances share one module-level store per cluster (ADR 001), so a
// snapshot cached by one spec would otherwise be served to the next one.
// Settings need no storage shim: src/api/settings.js falls back to defaults
// when `localStorage` is missing or is Node's method-less global.
afterEach(() => {
  resetSharedStores();
});
