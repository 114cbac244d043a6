module.exports = {
  extends: ['@headlamp-k8s/eslint-config'],
  rules: {
    // Prettier owns formatting.
    indent: 'off',
  },
  overrides: [
    {
      // Plain ES2019 modules shared with the Node 12 test runner.
      files: ['src/**/*.js', 'tests/js/**/*.js', 'bench/**/*.js', 'tools/**/*.js'],
      env: { node: true, browser: true, es2019: true },
      globals: { describe: 'readonly', it: 'readonly', expect: 'readonly', vi: 'readonly', beforeEach: 'readonly', afterEach: 'readonly' },
    },
  ],
};
