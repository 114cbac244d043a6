import { ApiProxy, K8s } from '@kinvolk/headlamp-plugin/lib';
import { renderHook, waitFor } from '@testing-library/react';
import React from 'react';
import { beforeEach, describe, expect, it, vi } from 'vitest';
import { makeDeviceConfig, makeGpuNode, makePluginPod } from '../../tests/js/fixtures.js';
import { AmdGpuDataProvider, useAmdGpuContext, useNodeGpuMetrics } from './AmdGpuDataContext';
import { resetSharedStores } from './clusterStore.js';

vi.mock('@kinvolk/headlamp-plugin/lib', () => ({
  K8s: { ResourceClasses: { Node: { useList: vi.fn() }, Pod: { useList: vi.fn() } } },
  ApiProxy: { request: vi.fn() },
}));

function Wrapper({ children }: { children: React.ReactNode }) {
  return <AmdGpuDataProvider>{children}</AmdGpuDataProvider>;
}

beforeEach(() => {
  resetSharedStores();
  vi.mocked(ApiProxy.request).mockReset();
});

describe('useAmdGpuContext', () => {
  it('throws outside the provider', () => {
    const spy = vi.spyOn(console, 'error').mockImplementation(() => {});
    expect(() => renderHook(() => useAmdGpuContext())).toThrow(
      'useAmdGpuContext must be used within an AmdGpuDataProvider'
    );
    spy.mockRestore();
  });
});

describe('AmdGpuDataProvider', () => {
  it('is loading while the lists are null', () => {
    vi.mocked(K8s.ResourceClasses.Node.useList).mockReturnValue([null, null] as any);
    vi.mocked(K8s.ResourceClasses.Pod.useList).mockReturnValue([null, null] as any);
    vi.mocked(ApiProxy.request).mockReturnValue(new Promise(() => {}));
    const { result } = renderHook(() => useAmdGpuContext(), { wrapper: Wrapper });
    expect(result.current.loading).toBe(true);
  });

  it('exposes GPU nodes from KubeObject wrappers and DeviceConfigs', async () => {
    vi.mocked(K8s.ResourceClasses.Node.useList).mockReturnValue([[{ jsonData: makeGpuNode('g0') }], null] as any);
    vi.mocked(K8s.ResourceClasses.Pod.useList).mockReturnValue([[], null] as any);
    vi.mocked(ApiProxy.request).mockImplementation((path: string) =>
      Promise.resolve(path.indexOf('deviceconfigs') >= 0 ? { items: [makeDeviceConfig()] } : { items: [] })
    );
    const { result } = renderHook(() => useAmdGpuContext(), { wrapper: Wrapper });
    await waitFor(() => expect(result.current.loading).toBe(false));
    expect(result.current.gpuNodes).toHaveLength(1);
    expect(result.current.crdAvailable).toBe(true);
    expect(result.current.deviceConfigs[0].metadata.name).toBe('gpu-operator');
  });

  it('degrades silently when the CRD is missing', async () => {
    vi.mocked(K8s.ResourceClasses.Node.useList).mockReturnValue([[], null] as any);
    vi.mocked(K8s.ResourceClasses.Pod.useList).mockReturnValue([[], null] as any);
    vi.mocked(ApiProxy.request).mockImplementation((path: string) =>
      path.indexOf('deviceconfigs') >= 0 ? Promise.reject(new Error('404')) : Promise.resolve({ items: [] })
    );
    const { result } = renderHook(() => useAmdGpuContext(), { wrapper: Wrapper });
    await waitFor(() => expect(result.current.loading).toBe(false));
    expect(result.current.crdAvailable).toBe(false);
    expect(result.current.error).toBeNull();
  });

  it('derives operator pods from the watched pod list (no plugin-pod requests)', async () => {
    vi.mocked(K8s.ResourceClasses.Node.useList).mockReturnValue([[], null] as any);
    vi.mocked(K8s.ResourceClasses.Pod.useList).mockReturnValue([[{ jsonData: makePluginPod('dp-0') }], null] as any);
    vi.mocked(ApiProxy.request).mockResolvedValue({ items: [] });
    const { result } = renderHook(() => useAmdGpuContext(), { wrapper: Wrapper });
    await waitFor(() => expect(result.current.loading).toBe(false));
    expect(result.current.pluginPods.map((p: any) => p.metadata.name)).toEqual(['dp-0']);
    expect(result.current.pluginInstalled).toBe(true);
    const paths = vi.mocked(ApiProxy.request).mock.calls.map(c => String(c[0]));
    expect(paths.every(p => p.indexOf('deviceconfigs') >= 0)).toBe(true);
  });

  it('refresh() re-issues the CRD request', async () => {
    vi.mocked(K8s.ResourceClasses.Node.useList).mockReturnValue([[], null] as any);
    vi.mocked(K8s.ResourceClasses.Pod.useList).mockReturnValue([[], null] as any);
    vi.mocked(ApiProxy.request).mockResolvedValue({ items: [] });
    const { result } = renderHook(() => useAmdGpuContext(), { wrapper: Wrapper });
    await waitFor(() => expect(result.current.loading).toBe(false));
    const before = vi.mocked(ApiProxy.request).mock.calls.length;
    result.current.refresh();
    await waitFor(() => expect(vi.mocked(ApiProxy.request).mock.calls.length).toBeGreaterThan(before));
  });
});

describe('useNodeGpuMetrics', () => {
  it('asks Prometheus for the one node only (hostname matcher)', async () => {
    vi.mocked(ApiProxy.request).mockResolvedValue({
      status: 'success',
      data: {
        resultType: 'vector',
        result: [{ metric: { __name__: 'gpu_power_usage', hostname: 'g0', gpu_id: '0' }, value: [0, '700'] }],
      },
    });
    const { result } = renderHook(() => useNodeGpuMetrics('g0'));
    await waitFor(() => expect(result.current.metrics).not.toBeNull());
    expect(result.current.metrics!.gpus.map(g => [g.nodeName, g.powerWatts])).toEqual([['g0', 700]]);
    const paths = vi.mocked(ApiProxy.request).mock.calls.map(c => decodeURIComponent(String(c[0])));
    expect(paths.every(p => p.indexOf('hostname="g0"') >= 0)).toBe(true);
  });

  it('fetches nothing without a node name', () => {
    renderHook(() => useNodeGpuMetrics(null));
    expect(vi.mocked(ApiProxy.request)).not.toHaveBeenCalled();
  });
});
