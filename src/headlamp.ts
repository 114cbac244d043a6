/**
 * The plugin bound to the real React and the Headlamp plugin library — the
 * one place the host runtime meets the plugin's code (src/plugin.js). Every
 * other TypeScript file is a re-export shim of this binding. Types come from
 * src/plugin.d.ts.
 */
import * as lib from '@kinvolk/headlamp-plugin/lib';
import * as CommonComponents from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import React from 'react';
import { createPlugin } from './plugin.js';

export const plugin = createPlugin({ React, lib, CommonComponents });
