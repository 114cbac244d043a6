import { describe, expect, it, vi } from 'vitest';

const calls = vi.hoisted(() => ({ sidebar: [] as any[], routes: [] as any[], details: [] as any[], columns: [] as any[] }));

vi.mock('@kinvolk/headlamp-plugin/lib', () => ({
  registerSidebarEntry: (e: unknown) => calls.sidebar.push(e),
  registerRoute: (r: unknown) => calls.routes.push(r),
  registerDetailsViewSection: (f: unknown) => calls.details.push(f),
  registerResourceTableColumnsProcessor: (f: unknown) => calls.columns.push(f),
  K8s: { ResourceClasses: { Node: { useList: () => [[], null] }, Pod: { useList: () => [[], null] } } },
  ApiProxy: { request: () => Promise.resolve({ items: [] }) },
}));
vi.mock('@kinvolk/headlamp-plugin/lib/CommonComponents', async () => (await import('./test-utils')).commonComponentsMock);

describe('plugin registration', () => {
  it('registers the sidebar, routes, detail sections and column processor', async () => {
    await import('./index');
    expect(calls.sidebar).toHaveLength(6);
    expect(calls.routes).toHaveLength(5);
    expect(calls.routes.every((r: any) => r.exact === true)).toBe(true);
    expect(calls.details).toHaveLength(2);
    expect(calls.columns).toHaveLength(1);
  });

  it('detail sections ignore other kinds', async () => {
    await import('./index');
    expect(calls.details[0]({ resource: { kind: 'Pod' } })).toBeNull();
    expect(calls.details[1]({ resource: { kind: 'Node' } })).toBeNull();
  });

  it('column processor only touches the Nodes table', async () => {
    await import('./index');
    const proc = calls.columns[0];
    expect(proc({ id: 'headlamp-nodes', columns: [] }).map((c: any) => c.label)).toEqual([
      'GPU Model',
      'GPU Devices',
      'GPU HBM',
    ]);
    const cols = [{ label: 'x' }];
    expect(proc({ id: 'other', columns: cols })).toBe(cols);
  });
});
