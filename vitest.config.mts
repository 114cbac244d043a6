import { defineConfig } from 'vitest/config';

export default defineConfig({
  test: {
    globals: true,
    environment: 'jsdom',
    setupFiles: ['./vitest.setup.ts'],
    // tests/js/*.test.js are the framework-free specs of the plugin logic; they
    // also run on bare Node via tools/minitest.js (see package.json test:node12).
    include: ['src/**/*.test.{ts,tsx}', 'tests/js/**/*.test.js'],
    exclude: ['node_modules/**'],
    env: { NODE_ENV: 'test' },
  },
});
