/**
 * Types of the IR renderer (./react.js). `ReactLike` is the slice of React
 * the renderer needs, so the real React and the harness stand-in
 * (tests/js/stubs/react.js) both satisfy it.
 */
import type { ComponentType, CSSProperties, ReactElement, ReactNode } from 'react';
import type { Block as IRBlock, Cell, GpuSlot, MatrixBlock, PageVM, PagerItem, Section as IRSection, SeriesPoint } from './ir';

export interface ReactLike {
  createElement: (...args: never[]) => ReactElement;
  memo: <P>(c: ComponentType<P>) => ComponentType<P>;
  Fragment: unknown;
}

/** The Headlamp CommonComponents the renderer draws with. */
export interface CommonComponentsLike {
  Loader: ComponentType<{ title: string }>;
  NameValueTable: ComponentType<{ rows: Array<{ name: string; value: ReactNode }> }>;
  PercentageBar: ComponentType<{ data: Array<{ name: string; value: number; fill: string }>; total: number }>;
  SectionBox: ComponentType<{ title: string; children?: ReactNode }>;
  SectionHeader: ComponentType<{ title: string }>;
  SimpleTable: ComponentType<{ columns: Array<{ label: string; getter: (row: never) => ReactNode }>; data: unknown[] }>;
  StatusLabel: ComponentType<{ status: 'success' | 'warning' | 'error'; children?: ReactNode }>;
}

export const REQUIRED_COMPONENTS: ReadonlyArray<keyof CommonComponentsLike>;

/** The renderer's stylesheet (classes amdgpu-*), added to the document once by ensureStyles. */
export const PLUGIN_CSS: string;
export const BUTTON_CLASS: string;
export function ensureStyles(doc?: Document | null): boolean;
export function barStyle(pct: number, color: string): CSSProperties;
export function slotsGradient(slots: GpuSlot[]): string;
export function sparklinePath(points: SeriesPoint[] | null | undefined, w: number, h: number): string | null;
export function matrixCellColor(c: MatrixBlock['matrix']['cells'][number][number]): string;
export function matrixCaption(b: MatrixBlock): string;

export interface Renderer {
  Value: ComponentType<{ v: Cell | undefined }>;
  InlineBar: ComponentType<{ pct: number | null; color: string; text: string }>;
  Slots: ComponentType<{ b: IRBlock }>;
  Matrix: ComponentType<{ b: MatrixBlock }>;
  Sparkline: ComponentType<{ points: SeriesPoint[]; color: string; label?: string }>;
  Series: ComponentType<{ b: IRBlock }>;
  Block: ComponentType<{ b: IRBlock }>;
  Section: ComponentType<{ s: IRSection | null }>;
  SectionImpl: ComponentType<{ s: IRSection | null }>;
  /** name filter + range shown + previous / next; the page owns the state */
  Pager: ComponentType<{
    p: PagerItem;
    onPage?: (page: number) => void;
    onFilter?: (filter: string) => void;
    onSort?: (sort: string) => void;
  }>;
  Page: ComponentType<{
    vm: PageVM;
    onRefresh?: () => void;
    onPage?: (page: number) => void;
    onFilter?: (filter: string) => void;
    onSort?: (sort: string) => void;
  }>;
}

export function createRenderer(React: ReactLike, CC: CommonComponentsLike): Renderer;
