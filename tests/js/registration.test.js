/**
 * Registration data (src/routes.js) — untested in the reference (SURVEY.md §4
 * gaps: "index.tsx registration is untested").
 */
import { BASE_URL, NODES_TABLE_ID, ROOT, ROUTES, SIDEBAR, processColumns } from '../../src/routes.js';
import { clusterFromPath } from '../../src/api/cluster.js';

describe('sidebar', () => {
  it('has one root and five children in reference order', () => {
    expect(SIDEBAR).toHaveLength(6);
    expect(SIDEBAR[0].parent).toBeNull();
    expect(SIDEBAR.slice(1).every((e) => e.parent === ROOT)).toBe(true);
    expect(SIDEBAR.slice(1).map((e) => e.label)).toEqual(['Overview', 'Device Plugins', 'GPU Nodes', 'GPU Pods', 'Metrics']);
  });
  it('labels the root with the product name, not the slug', () => {
    expect(SIDEBAR[0].label).toBe('AMD GPU');
    expect(SIDEBAR[0].name).toBe('amd-gpu');
  });
  it('gives every entry an icon and a URL under the base', () => {
    SIDEBAR.forEach((e) => {
      expect(e.icon).toMatch(/^mdi:/);
      expect(e.url.indexOf(BASE_URL)).toBe(0);
    });
  });
  it('has unique names', () => {
    const names = SIDEBAR.map((e) => e.name);
    expect(new Set(names).size).toBe(names.length);
  });
});

describe('routes', () => {
  it('registers five routes, each bound to a sidebar entry', () => {
    expect(ROUTES).toHaveLength(5);
    const names = SIDEBAR.map((e) => e.name);
    ROUTES.forEach((r) => expect(names).toContain(r.sidebar));
  });
  it('route paths match sidebar URLs', () => {
    const urls = SIDEBAR.slice(1).map((e) => e.url);
    expect(ROUTES.map((r) => r.path)).toEqual(urls);
  });
  it('maps to the five pages', () => {
    expect(ROUTES.map((r) => r.page)).toEqual(['overview', 'device-plugins', 'nodes', 'pods', 'metrics']);
  });
});

describe('columns processor', () => {
  const build = () => [{ label: 'GPU Model' }, { label: 'GPU Devices' }];
  it('appends GPU columns to the native Nodes table', () => {
    const out = processColumns({ id: NODES_TABLE_ID, columns: [{ label: 'Name' }] }, build);
    expect(out.map((c) => c.label)).toEqual(['Name', 'GPU Model', 'GPU Devices']);
  });
  it('leaves other tables untouched', () => {
    const cols = [{ label: 'Name' }];
    expect(processColumns({ id: 'headlamp-pods', columns: cols }, build)).toBe(cols);
  });
});

describe('cluster key', () => {
  it('parses Headlamp cluster URLs', () => {
    expect(clusterFromPath('/c/prod-east/amd-gpu/nodes')).toBe('prod-east');
    expect(clusterFromPath('#/c/lab%201/amd-gpu')).toBe('lab 1');
  });
  it('falls back to a default key', () => {
    expect(clusterFromPath('/amd-gpu')).toBe('__default__');
    expect(clusterFromPath(undefined)).toBe('__default__');
  });
});
