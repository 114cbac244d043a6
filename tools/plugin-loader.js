/**
 * ESM loader that lets Node execute the plugin's TypeScript entry shims
 * (src/index.tsx, src/headlamp.ts) against the
 * harness stand-ins, so the files Headlamp bundles are the files the specs
 * run:
 *
 *   react                                   → tests/js/stubs/react.js
 *   @kinvolk/headlamp-plugin/lib            → tests/js/stubs/headlamp-lib.js
 *   @kinvolk/headlamp-plugin/lib/CommonComponents → tests/js/stubs/CommonComponents.js
 *   amd-test-harness                        → tests/js/harness/stub.js (shared specs' render API)
 *   (with AMD_TEST_TIER=react-umd: react → tests/js/harness/umd-react.js, the REAL React 18.3.1 UMD
 *    builds over a minimal DOM; CommonComponents → harness/cc-dom.js; amd-test-harness → harness/umd.js)
 *   './x' (no extension)                    → ./x.tsx | ./x.ts | ./x.js | ./x/index.tsx
 *   *.ts / *.tsx                            → ES module; `import type` lines removed
 *
 * The shims are written in the JavaScript subset of TypeScript (all types
 * come from the .d.ts files next to the JS modules), so nothing else needs
 * transpiling; any other TypeScript syntax fails to parse here, which keeps
 * the shims honest.
 *
 * Usage: node --experimental-loader ./tools/plugin-loader.js tools/minitest.js …
 * Hooks for both loader APIs: Node 12–16.11 (resolve/getFormat/getSource/
 * transformSource) and Node >= 16.12 (resolve/load).
 */
import fs from 'fs';
import path from 'path';
import { fileURLToPath, pathToFileURL } from 'url';

const ROOT = path.resolve(path.dirname(fileURLToPath(import.meta.url)), '..');
const STUBS = path.join(ROOT, 'tests', 'js', 'stubs');

const HARNESS = path.join(ROOT, 'tests', 'js', 'harness');

// AMD_TEST_TIER=react-umd: the REAL React 18.3.1 + react-dom (UMD builds,
// AMD_REACT_UMD_DIR) over a minimal DOM — the offline real-React tier
// (tests/test_js_real_react.py); otherwise the harness React.
const REAL = process.env.AMD_TEST_TIER === 'react-umd';

const ALIASES = {
  react: REAL ? path.join(HARNESS, 'umd-react.js') : path.join(STUBS, 'react.js'),
  '@kinvolk/headlamp-plugin/lib': path.join(STUBS, 'headlamp-lib.js'),
  '@kinvolk/headlamp-plugin/lib/CommonComponents': REAL ? path.join(HARNESS, 'cc-dom.js') : path.join(STUBS, 'CommonComponents.js'),
  'amd-test-harness': REAL ? path.join(HARNESS, 'umd.js') : path.join(HARNESS, 'stub.js'),
};

const TRY = ['.tsx', '.ts', '.js', '/index.tsx', '/index.ts', '/index.js'];

function isTs(url) {
  return /\.tsx?$/.test(url);
}

export function resolve(specifier, context, defaultResolve) {
  if (Object.prototype.hasOwnProperty.call(ALIASES, specifier)) {
    return { url: pathToFileURL(ALIASES[specifier]).href };
  }
  if ((specifier.startsWith('./') || specifier.startsWith('../')) && context.parentURL && !path.extname(specifier)) {
    const base = path.resolve(path.dirname(fileURLToPath(context.parentURL)), specifier);
    for (let i = 0; i < TRY.length; i++) {
      if (fs.existsSync(base + TRY[i])) return { url: pathToFileURL(base + TRY[i]).href };
    }
  }
  if (specifier.startsWith('file:') && isTs(specifier)) return { url: specifier };
  return defaultResolve(specifier, context, defaultResolve);
}

/** TypeScript → JavaScript for the shims: only `import type` statements are removed. */
export function stripTypes(source) {
  return String(source).replace(/^import type [^;]*;[ \t]*$/gm, '');
}

// Node 12 – 16.11
export function getFormat(url, context, defaultGetFormat) {
  if (isTs(url)) return { format: 'module' };
  return defaultGetFormat(url, context, defaultGetFormat);
}

export function transformSource(source, context, defaultTransformSource) {
  if (isTs(context.url)) return { source: stripTypes(source) };
  return defaultTransformSource(source, context, defaultTransformSource);
}

// Node >= 16.12
export function load(url, context, defaultLoad) {
  if (isTs(url)) {
    return { format: 'module', source: stripTypes(fs.readFileSync(fileURLToPath(url), 'utf8')), shortCircuit: true };
  }
  return defaultLoad(url, context, defaultLoad);
}
