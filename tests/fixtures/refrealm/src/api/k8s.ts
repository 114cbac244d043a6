// Fixture for the reference realm specs (tests/test_render_compare.py): the two
// filters the realm's context value calls, in the shape of the reference's helpers.
export interface Named {
  metadata: { name: string };
  status?: { capacity?: Record<string, string> };
}

export function filterIntelGpuNodes(items: unknown[]): Named[] {
  return (items as Named[]).filter((n) => !!n?.status?.capacity?.['gpu.intel.com/i915']);
}

export function filterGpuRequestingPods(items: unknown[]): Named[] {
  return (items as Named[]).filter((p) => JSON.stringify(p).indexOf('gpu.intel.com/') >= 0);
}
