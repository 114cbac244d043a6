/**
 * What the reference's realm gets of the test harness (bench/refWorker.cjs):
 * the minimal DOM and the CommonComponents stand-ins, bundled by
 * tools/bundle.js into one script evaluated inside the realm, so the
 * reference's pages render on the same DOM and stand-ins as this plugin's.
 */
export { createWindow } from '../tests/js/harness/minidom.js';
export { makeCommonComponents } from '../tests/js/harness/commonComponents.js';
