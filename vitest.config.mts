import path from 'path';
import { defineConfig } from 'vitest/config';

// The harness tier: tests/js/*.test.js and tests/js/shared/*.test.js, written
// against the vitest globals API
// so that they also run on bare Node via tools/minitest.js
// (`npm run test:node12`). The React layer is exercised against the same
// stand-ins under both runners: 'react' and the Headlamp library resolve to
// tests/js/stubs/ (tools/plugin-loader.js does the same under Node), so a
// spec asserts the same markup and props whichever runner executes it.
const stubs = path.resolve(__dirname, 'tests/js/stubs');

export default defineConfig({
  resolve: {
    alias: [
      { find: /^@kinvolk\/headlamp-plugin\/lib\/CommonComponents$/, replacement: path.join(stubs, 'CommonComponents.js') },
      { find: /^@kinvolk\/headlamp-plugin\/lib$/, replacement: path.join(stubs, 'headlamp-lib.js') },
      { find: /^react$/, replacement: path.join(stubs, 'react.js') },
      { find: /^amd-test-harness$/, replacement: path.resolve(__dirname, 'tests/js/harness/stub.js') },
    ],
  },
  test: {
    include: ['tests/js/**/*.test.js'],
    exclude: ['node_modules/**', 'dist/**', 'gpurun_out/**'],
    environment: 'node',
    globals: true,
    setupFiles: ['./vitest.setup.ts'],
    testTimeout: 20000,
    env: { NODE_ENV: 'test' },
    coverage: { provider: 'v8', include: ['src/**'], reporter: ['text', 'lcov'] },
  },
});
