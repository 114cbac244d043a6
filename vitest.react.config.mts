import path from 'path';
import { defineConfig } from 'vitest/config';

// The real-React tier: the runner-agnostic specs (tests/js/shared/) on React
// 18.3 + react-dom in jsdom, rendered with @testing-library/react — the tier
// the reference's component tests run in (reference vitest.config.mts:4-6).
// Nothing aliases 'react': the real package renders. Only the Headlamp
// library is replaced, by the same stand-ins the reference mocks it with
// (reference src/components/OverviewPage.test.tsx:8-61): the registry /
// useList / ApiProxy stub and CommonComponents built on the real React.
// Needs `npm ci` (networked); offline, the same specs run on the harness
// React through vitest.config.mts and tools/minitest.js.
const js = path.resolve(__dirname, 'tests/js');

export default defineConfig({
  resolve: {
    alias: [
      { find: /^@kinvolk\/headlamp-plugin\/lib\/CommonComponents$/, replacement: path.join(js, 'harness', 'cc-dom.js') },
      { find: /^@kinvolk\/headlamp-plugin\/lib$/, replacement: path.join(js, 'stubs', 'headlamp-lib.js') },
      { find: /^amd-test-harness$/, replacement: path.join(js, 'harness', 'dom.js') },
    ],
  },
  test: {
    include: ['tests/js/shared/**/*.test.js'],
    environment: 'jsdom',
    globals: true,
    setupFiles: ['./vitest.setup.ts'],
    testTimeout: 20000,
    env: { NODE_ENV: 'test' },
  },
});
