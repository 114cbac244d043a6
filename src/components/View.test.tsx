import { fireEvent, render, screen } from '@testing-library/react';
import React from 'react';
import { describe, expect, it, vi } from 'vitest';
import { makeContext, makeGpuNode, makeGpuPod, NOW } from '../../tests/js/fixtures.js';
import { nodesView, overviewView, podDetailView } from '../view/pages.js';
import { Page, Section } from './View';

vi.mock('@kinvolk/headlamp-plugin/lib/CommonComponents', async () => (await import('../test-utils')).commonComponentsMock);

describe('View renderer', () => {
  it('renders header, refresh button and sections', () => {
    const onRefresh = vi.fn();
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0' })] });
    render(<Page vm={nodesView(ctx, { now: NOW })} onRefresh={onRefresh} />);
    expect(screen.getByRole('heading', { level: 1 })).toHaveTextContent('AMD GPU — Nodes');
    expect(screen.getByText('GPU Node Summary')).toBeInTheDocument();
    fireEvent.click(screen.getByLabelText('Refresh node data'));
    expect(onRefresh).toHaveBeenCalledTimes(1);
  });

  it('renders only the loader on first load', () => {
    render(<Page vm={overviewView(makeContext({ loading: true, lastUpdated: null }))} />);
    expect(screen.getByTestId('loader')).toHaveTextContent('Loading AMD GPU data...');
  });

  it('renders status labels with their status', () => {
    const { container } = render(<Section s={podDetailView(makeGpuPod('p'))} />);
    expect(container.querySelector('[data-status="success"]')).toHaveTextContent('Running');
  });

  it('renders the per-GPU strip and the xGMI matrix', () => {
    const ctx = makeContext({ nodes: [makeGpuNode('g0')], pods: [makeGpuPod('a', { node: 'g0', gpus: 2 })] });
    render(<Page vm={nodesView(ctx, { now: NOW })} />);
    expect(screen.getAllByText(/GPU 7/).length).toBeGreaterThan(0);
    expect(screen.getByText(/xGMI topology/)).toBeInTheDocument();
  });
});
