/**
 * Pages that render before every request is in (ADR 011): the Overview once
 * its node list is in, its DeviceConfig section loading in place.
 */
import { overviewView } from '../../src/view/pages/overview.js';
import { loaders, sectionTitles } from '../../src/view/ir.js';
import { makeContext, makeGpuNode, NOW } from './fixtures.js';

const opts = { now: NOW };

describe('overviewView: progressive', () => {
  it('renders once the node list is in; the DeviceConfig section loads in place (a slow or absent CRD holds nothing else)', () => {
    const ctx = makeContext({ nodesLoading: false, crdLoading: true, podsLoading: true, pluginPodsLoading: true, nodes: [makeGpuNode('g')] });
    const vm = overviewView(ctx, opts);
    expect(vm.title).toBe('AMD GPU — Overview');
    expect(loaders(vm)).toEqual(['Loading DeviceConfigs...', 'Loading GPU pods...']);
    const titles = sectionTitles(vm);
    expect(titles).toContain('GPU Nodes');
    expect(titles).not.toContain('Plugin Not Detected');
    expect(titles).not.toContain('Notice');
    // the answer: no CRD, no operator pods → the notices come then
    const done = overviewView(makeContext({ nodesLoading: false, crdLoading: false, podsLoading: false, pluginPodsLoading: false,
      nodes: [makeGpuNode('g')] }), opts);
    expect(loaders(done)).toEqual([]);
    expect(sectionTitles(done)).toContain('Plugin Not Detected');
  });

});
