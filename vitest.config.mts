import { defineConfig } from 'vitest/config';

// Two spec families share one runner:
//  - src/**/*.test.tsx: React bindings and renderers (jsdom, CommonComponents mocked);
//  - tests/js/*.test.js: the framework-free plugin logic, also run on bare Node
//    by tools/minitest.js (`npm run test:node12`), so they use only vitest globals.
const specs = ['src/**/*.test.{ts,tsx}', 'tests/js/**/*.test.js'];

export default defineConfig({
  test: {
    include: specs,
    exclude: ['node_modules/**', 'dist/**', 'gpurun_out/**'],
    environment: 'jsdom',
    globals: true,
    setupFiles: ['./vitest.setup.ts'],
    testTimeout: 20000,
    env: { NODE_ENV: 'test' },
    coverage: { provider: 'v8', include: ['src/**'], reporter: ['text', 'lcov'] },
  },
});
