/** Types of the settings page (./settingsPage.js). */
import type { ComponentType } from 'react';

export function refreshChoiceLabel(v: number): string;

export function createSettingsPage(
  React: unknown,
  CC: unknown,
  storage?: { load: () => unknown; save: (v: unknown) => unknown }
): ComponentType<{ data?: Record<string, unknown>; onDataChange?: (data: Record<string, unknown>) => void }>;
