/**
 * tools/lint_js.js — the offline stand-in for ESLint's no-unused-vars on
 * imports and top-level declarations, plus the module-size budget.
 */
import { MAX_LINES, lintSource } from '../../tools/lint_js.js';

describe('lint_js', () => {
  it('flags an import the file never uses, and keeps one used in a template literal', () => {
    const src = "import { a, b as c } from './x.js';\nimport * as ns from './y.js';\nexport const s = `${c}`;\n";
    expect(lintSource('f.js', src)).toEqual(['f.js: import a is never used', 'f.js: import ns is never used']);
  });

  it('flags a top-level declaration neither exported nor used; exported ones are fine', () => {
    const src = 'function dead() {}\nconst used = 1;\nexport function live() { return used; }\nconst viaList = 2;\nexport { viaList };\n';
    expect(lintSource('f.js', src)).toEqual(['f.js: dead is declared but never used']);
  });

  it('holds every module to the size budget', () => {
    const src = 'export const x = 1;\n'.repeat(MAX_LINES + 1);
    expect(lintSource('big.js', src)).toEqual(['big.js: ' + (MAX_LINES + 1) + ' lines (budget ' + MAX_LINES + ')']);
  });
});
