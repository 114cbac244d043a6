/**
 * View — the page IR (src/view/ir.js) rendered with Headlamp
 * CommonComponents. Implementation: src/view/react.js (typed in react.d.ts).
 */
import { plugin } from '../headlamp';

export const { Page, Section, Value, Block } = plugin.view;
