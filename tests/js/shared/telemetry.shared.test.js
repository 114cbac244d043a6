/**
 * Telemetry paths of the shipped React layer, on the harness React and on
 * real React 18.3.1: the Pod detail section's one wave (node telemetry + the
 * pod's power history) and the Metrics page when RBAC denies the Prometheus
 * proxy (access denied, with the missing permission — not "unreachable").
 */
import { React, render, tier } from 'amd-test-harness';
import * as lib from '@kinvolk/headlamp-plugin/lib';
import * as CC from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import '../../../src/index.tsx';
import { createPlugin } from '../../../src/plugin.js';
import { resetSharedStores } from '../../../src/api/clusterStore.js';
import { clearViewMemo } from '../../../src/view/pages/common.js';
import { DEVICE_CONFIG_LIST_PATH } from '../../../src/api/k8sCore.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod } from '../fixtures.js';
import { exporterData, prom } from '../promFake.js';

const h = React.createElement;
const reg = { details: lib.registry.details.slice() };

function cluster(prometheus) {
  lib.lists.Node = [[makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1')], null];
  lib.lists.Pod = [[makeGpuPod('train-a', { gpus: 4, node: 'mi355x-0' })], null];
  lib.api.handler = (p) => {
    if (p === DEVICE_CONFIG_LIST_PATH) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
    if (p.indexOf('/proxy/api/v1/') >= 0) return prometheus(p);
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
}

beforeEach(() => {
  lib.resetHeadlamp();
  resetSharedStores();
  clearViewMemo();
});

describe('shared: telemetry on the detail and Metrics pages (' + tier + ')', () => {
  it('Pod detail sends the node-scoped query and the pod\'s power-history range query in one wave and shows the history', async () => {
    const fake = prom({ data: exporterData(['mi355x-0', 'mi355x-1']) });
    cluster(fake);
    const pod = makeGpuPod('train-a', { gpus: 4, node: 'mi355x-0' });
    const r = render(reg.details[1]({ resource: { kind: 'Pod', jsonData: pod } }));
    await r.settle();
    const paths = fake.mock.calls.map((c) => decodeURIComponent(c[0]));
    expect(paths.filter((p) => p.indexOf('hostname="mi355x-0"') >= 0)).toHaveLength(1);
    expect(paths.filter((p) => p.indexOf('/query_range') >= 0 && p.indexOf('pod="train-a"') >= 0)).toHaveLength(1);
    expect(r.text()).toContain('Peak GPU Power');
    r.unmount();
  });

  it('Metrics shows the instant telemetry while its range series are still in flight, then the series', async () => {
    const fake = prom({ data: exporterData(['mi355x-0', 'mi355x-1']) });
    const held = [];
    cluster((p) => (p.indexOf('/query_range') >= 0
      ? new Promise((res) => { held.push(() => res(fake(p))); })
      : fake(p)));
    const fresh = createPlugin({ React, lib, CommonComponents: CC });
    const r = render(h(fresh.AmdGpuDataProvider, null, h(fresh.MetricsPage)));
    await r.settle();
    expect(held.length).toBeGreaterThan(0);
    expect(r.text()).toContain('GPUs Monitored');
    expect(r.text()).not.toContain('Power & HBM (last');
    held.splice(0).forEach((go) => go());
    await r.settle();
    expect(r.text()).toContain('GPUs Monitored');
    expect(r.text()).toContain('Power & HBM (last');
    r.unmount();
  });

  it('Metrics without RBAC for the Prometheus proxy says access was denied and which permission is missing', async () => {
    cluster(() => Promise.reject(Object.assign(new Error('services "kube-prometheus-stack-prometheus" is forbidden'), { status: 403 })));
    // A fresh plugin: no metrics client state from earlier specs.
    const fresh = createPlugin({ React, lib, CommonComponents: CC });
    const r = render(h(fresh.AmdGpuDataProvider, null, h(fresh.MetricsPage)));
    await r.settle();
    expect(r.text()).toContain('Prometheus Access Denied');
    expect(r.text()).not.toContain('Prometheus Unreachable');
    expect(r.text()).toContain('services/proxy');
    r.unmount();
  });
});
