/**
 * Types of the view IR (./ir.js): what every view-model in ./pages.js
 * returns and what ./react.js renders. Replaces the untyped `IR = any` of
 * round 1; the reference's convention is "no `any`, unknown + guards"
 * (reference CLAUDE.md:76).
 */
import type { Status } from '../api/types';

export type { Status };

/** A status label cell (StatusLabel). */
export interface StatusCell {
  t: 'status';
  status: Status;
  text: string;
}

/** Inline allocation / power bar cell; `pct` null draws the text only. */
export interface BarCell {
  t: 'bar';
  used: number;
  total: number | null;
  pct: number | null;
  color: string;
  text: string;
}

/** Multi-line cell: "<strong>label</strong>: text" per line. */
export interface LinesCell {
  t: 'lines';
  lines: Array<{ label: string; text: string }>;
}

export type Cell = string | number | null | StatusCell | BarCell | LinesCell;

export interface KvRow {
  name: string;
  value: Cell;
}

export interface KvBlock {
  t: 'kv';
  rows: KvRow[];
}

export interface TableBlock {
  t: 'table';
  columns: string[];
  rows: Cell[][];
  /** Stable row keys (uids) when the rows are Kubernetes objects. */
  keys: string[] | null;
}

export interface PctbarDatum {
  name: string;
  value: number;
  fill: string;
}

export interface PctbarBlock {
  t: 'pctbar';
  label: string;
  data: PctbarDatum[];
  total: number;
}

/** One schedulable device of a node (src/api/topology.js buildGpuSlots). */
export interface GpuSlot {
  index: number;
  board: number;
  partition: number | null;
  pod: string | null;
  namespace: string | null;
  inferred: boolean;
}

export interface SlotsBlock {
  t: 'slots';
  slots: GpuSlot[];
  /** Owners came from exporter pod labels (else inferred from pod order). */
  exact: boolean;
  partitionsPerGpu: number;
}

export interface XgmiCell {
  kind: 'self' | 'xgmi' | 'pcie' | 'none';
  hops: number;
  peakGBs: number;
  /** GB/s placed on this link (a series pinned its peer); on a `self` cell, the GPU's xGMI total over all links. */
  measuredGBs: number | null;
}

export interface XgmiMatrix {
  size: number;
  cells: XgmiCell[][];
  linksPerGpu: number;
  perGpuPeakGBs: number;
  ringBusGBs: number;
}

export interface MatrixBlock {
  t: 'matrix';
  matrix: XgmiMatrix;
  fullMesh: boolean;
  /** Link types / hops were measured (exporter link series) rather than assumed. */
  measuredTopology: boolean;
  /** Throughput sits on links: a series pinned each xgmi_neighbor_<k> row to its peer (topology.js placeThroughput). */
  measuredThroughput: boolean;
  /** Per-GPU xGMI totals were measured (the diagonal cells); true whenever any throughput was. */
  throughputPerGpu?: boolean;
  /** Renderers draw the grid (true) or its summary line with the grid one click away (false). */
  open: boolean;
  /** Facts pages/nodes.js matrixBlock reads from the link maps (topology.js linkFacts) without building
   * the grid; absent on a hand-made block, where matrixCaption / matrixSummary read `matrix`. */
  size?: number;
  linksPerGpu?: number;
  linkGBs?: number;
  ringBusGBs?: number;
  linkStats?: { links: number; maxGBs: number; meanGBs: number } | null;
  gpuStats?: { gpus: number; maxGBs: number; meanGBs: number } | null;
}

/** [unix seconds, value] */
export type SeriesPoint = [number, number];

export interface SeriesBlock {
  t: 'series';
  power: Record<string, SeriesPoint[]>;
  vram: Record<string, SeriesPoint[]>;
  /** Header of the first column (default "Node"; "Pod" on the Pod detail page). */
  label?: string;
  /** Mean power per node over the window (W); nodes without samples are absent. */
  avgPower?: Record<string, number>;
}

export type Block = KvBlock | TableBlock | PctbarBlock | SlotsBlock | MatrixBlock | SeriesBlock;

export interface Section {
  t: 'section';
  title: string;
  key: string;
  blocks: Block[];
}

export interface LoaderItem {
  t: 'loader';
  title: string;
}

/** Page-level pager over a long list (GPU nodes): the slice shown and the name filter. */
export interface PagerItem {
  t: 'pager';
  key: 'pager';
  /** what is counted, e.g. "GPU nodes" */
  noun: string;
  /** what the controls are named after ("Filter <label> by name", "Sort <label>"): stable across orders */
  label: string;
  /** 0-based */
  page: number;
  pages: number;
  /** slice [from, to) of the matching list */
  from: number;
  to: number;
  total: number;
  matched: number;
  filter: string;
  perPage: number;
  /** the current order, when the list offers several (`sorts`) */
  sort?: string;
  sorts?: ReadonlyArray<{ value: string; label: string }>;
  /** a ranked page past the end (the count shrank): the component moves to the last page */
  beyond?: boolean;
}

export interface RefreshButton {
  label: string;
  ariaLabel: string;
  disabled: boolean;
}

export interface PageVM {
  t: 'page';
  /** null while the page is only a loader */
  title: string | null;
  refresh: RefreshButton | null;
  items: Array<Section | LoaderItem | PagerItem>;
}

export function status(st: Status, text: string | number): StatusCell;
export function bar(used: number, total: number | null, pctValue: number | null, color: string, text: string): BarCell;
export function lines(items: Array<{ label: string; text: string }>): LinesCell;
export function kv(rows: KvRow[]): KvBlock;
export function row(name: string, value: Cell): KvRow;
export function table(columns: string[], rows: Cell[][], keys?: string[]): TableBlock;
export function pctbar(label: string, data: PctbarDatum[], total: number): PctbarBlock;
export function section(title: string, blocks: Block[], key?: string): Section;
export function loader(title: string): LoaderItem;
export function page(title: string | null, refresh: RefreshButton | null, items: Array<Section | LoaderItem | PagerItem>): PageVM;
export function pager(
  p: { page: number; pages: number; from: number; to: number; total: number; matched: number; filter: string; perPage: number; beyond?: boolean },
  noun: string,
  sorting?: { sort?: string; sorts?: ReadonlyArray<{ value: string; label: string }>; label?: string }
): PagerItem;
/** "Showing 17–24 of 1000 GPU nodes · page 3 of 125" */
export function pagerText(p: PagerItem): string;
/** One page, no filter, the default order: renderers show the count with the controls one click away. */
export function pagerIdle(p: PagerItem): boolean;
export function pagerOf(vm: PageVM | null): PagerItem | null;

export interface Memo {
  /** `now` (epoch ms): also hold the value only until the first age label inside it changes. */
  <T>(key: string, deps: readonly unknown[], compute: () => T, now?: number): T;
  clear(): void;
  size(): number;
}
export function createMemo(limit?: number): Memo;

/** Per-object cache (WeakMap keyed on the Kubernetes object); same contract as Memo. */
export interface ObjectCache {
  <T>(obj: object, deps: readonly unknown[], compute: () => T, now?: number): T;
  clear(): void;
}
export function createObjectCache(): ObjectCache;

/** Record that the value being built changes at epoch-ms `t` (age labels). */
export function noteExpiry(t: number | null | undefined): void;

/** Caption of the xGMI matrix: measured topology or the platform model; link or per-GPU throughput. */
export function matrixCaption(b: MatrixBlock): string;
/** " · measured: max X, mean Y GB/s over N links", the per-GPU form, or '' without measured throughput. */
export function matrixSummary(b: MatrixBlock): string;
/** Text of one matrix cell: "Σ N" for a GPU's total, GB/s on a link, `xgmiMark` on an unmeasured xGMI link. */
export function matrixCellText(c: XgmiCell, xgmiMark: string): string;
/** matrixCaption(b) + matrixSummary(b), formatted once per distinct content (the facts; the statistics object). */
export function matrixLine(b: MatrixBlock): string;
/** "namespace/pod" or "free". */
export function slotOwner(s: GpuSlot): string;
/** Owners in runs: "GPU 0–3 ml/train-a · GPU 4–7 free". */
export function slotsText(slots: GpuSlot[]): string;

export function sections(vm: PageVM | Section | null): Section[];
export function sectionTitles(vm: PageVM | Section | null): string[];
export function findSection(vm: PageVM | Section | null, title: string): Section | null;
export function loaders(vm: PageVM | null): string[];
export function rowValue(scope: PageVM | Section | null, name: string): Cell | undefined;
export function rowNames(sec: Section | null): string[];
export function firstTable(sec: Section | null): TableBlock | null;
export function firstBlock(sec: Section | null, t: Block['t']): Block | null;
export function text(v: Cell | undefined): string;
export function countRows(vm: PageVM | Section | null): { sections: number; tableRows: number; kvRows: number; gpuCells: number };
