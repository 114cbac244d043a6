/**
 * Headlamp CommonComponents stand-ins for the Node-12 harness, built on the
 * React stand-in. Each renders the semantic element the reference's component
 * tests mock it with (reference src/components/OverviewPage.test.tsx:8-61) —
 * and that src/view/html.js emits for the same IR node — so specs assert on
 * one markup whichever renderer produced it:
 *   SectionBox → <section><h2>title</h2>…</section>, SectionHeader → <h1>,
 *   NameValueTable → <dl><div><dt>name</dt><dd>value</dd></div>…</dl>,
 *   SimpleTable → <table><thead>…</thead><tbody>…</tbody></table>,
 *   StatusLabel → <span data-status>, Loader → data-testid="loader",
 *   PercentageBar → data-testid="percentage-bar".
 * Component instances keep their props, so specs can also check what a page
 * handed each component (SimpleTable columns / getters / data, …).
 */
import { createElement as h } from './react.js';
import { makeCommonComponents } from '../harness/commonComponents.js';

const CC = makeCommonComponents(h);

export const SectionBox = CC.SectionBox;
export const SectionHeader = CC.SectionHeader;
export const NameValueTable = CC.NameValueTable;
export const SimpleTable = CC.SimpleTable;
export const StatusLabel = CC.StatusLabel;
export const Loader = CC.Loader;
export const PercentageBar = CC.PercentageBar;
