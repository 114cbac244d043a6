/** CommonComponents stand-ins on the real React (vitest.react.config.mts aliases the Headlamp path here). */
import * as ReactNS from 'react';
import { makeCommonComponents } from './commonComponents.js';

const React = ReactNS.default || ReactNS;
const CC = makeCommonComponents(React.createElement);

export const SectionBox = CC.SectionBox;
export const SectionHeader = CC.SectionHeader;
export const NameValueTable = CC.NameValueTable;
export const SimpleTable = CC.SimpleTable;
export const StatusLabel = CC.StatusLabel;
export const Loader = CC.Loader;
export const PercentageBar = CC.PercentageBar;
