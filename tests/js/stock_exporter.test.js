/**
 * The STOCK AMD Device Metrics Exporter path, end to end: a scrape with only
 * the stock names (tests/fixtures/stock_exporter — no gpu_power_cap, no
 * gpu_junction_temperature_slowdown, no gpu_xgmi_link_hops; synthetic, see
 * its header) goes through the real metrics client against a fake
 * Prometheus, and every Metrics / GPU Nodes / Node detail / GPU Pods cell is
 * checked. What the exporter does not report is shown as an MI355X platform
 * value and SAID to be one (caption, "Assumed Limits"), while what it does
 * report (per-link xGMI throughput, pod ownership) is used as measured.
 */
import fs from 'fs';
import path from 'path';
import { createMetricsSource } from '../../src/api/metrics.js';
import { splitByName } from '../../src/api/telemetry.js';
import { MI355X } from '../../src/api/k8sCore.js';
import { clearViewMemo } from '../../src/view/pages/common.js';
import { nodeDetailView } from '../../src/view/pages/details.js';
import { metricsView } from '../../src/view/pages/metricsPage.js';
import { nodesView } from '../../src/view/pages/nodes.js';
import { podsView } from '../../src/view/pages/pods.js';
import { findSection, firstBlock, firstTable, rowValue, sections } from '../../src/view/ir.js';
import { renderPage } from '../../src/view/html.js';
import { renderText } from '../../src/view/text.js';
import { parseExposition, prom } from './promFake.js';
import { NOW, makeContext, makeGpuNode, makeGpuPod } from './fixtures.js';

const HOST = 'mi355x-stock-0';
const FIXTURE = path.join(process.cwd(), 'tests', 'fixtures', 'stock_exporter', 'node_8x_mi355x.prom');
const rows = parseExposition(fs.readFileSync(FIXTURE, 'utf8'));

function fetchStock() {
  const request = prom({ data: splitByName(rows) });
  return createMetricsSource({ request }).fetchGpuMetrics();
}

function cluster() {
  return makeContext({
    nodes: [makeGpuNode(HOST)],
    pods: [makeGpuPod('train-a', { node: HOST, gpus: 4 }), makeGpuPod('infer-b', { node: HOST, gpus: 1 })],
  });
}

describe('stock AMD Device Metrics Exporter (no repo-specific series)', () => {
  beforeEach(() => clearViewMemo());

  it('the fixture carries only stock names', () => {
    const names = new Set(rows.map((r) => r.metric.__name__));
    ['gpu_power_cap', 'gpu_junction_temperature_slowdown', 'gpu_xgmi_link_hops', 'gpu_partition_info'].forEach((n) => expect(names.has(n)).toBe(false));
    ['gpu_power_usage', 'gpu_total_vram', 'gpu_used_vram', 'gpu_gfx_activity', 'gpu_umc_activity', 'gpu_junction_temperature',
      'gpu_ecc_correct_total', 'gpu_ecc_uncorrect_total', 'xgmi_neighbor_0_tx_throughput'].forEach((n) => expect(names.has(n)).toBe(true));
  });

  it('joins 8 GPUs; the missing cap is the MI355X board limit, flagged as assumed', async () => {
    const m = await fetchStock();
    expect(m.source).toBe('amd-exporter');
    expect(m.gpus).toHaveLength(8);
    m.gpus.forEach((g) => {
      expect(g.nodeName).toBe(HOST);
      expect(g.powerCapWatts).toBe(MI355X.tdpWatts);
      expect(g.powerCapAssumed).toBe(true);
      expect(g.tempSlowdownC).toBeNull();
      expect(g.vramTotalBytes).toBe(MI355X.hbmBytes);
    });
    expect(m.links).toEqual({});
    // no series says which peer neighbour k is: the rows stay per neighbour, placed on no peer
    expect(m.xgmi[HOST]['0>0']).toBeCloseTo(61.2, 6);
    expect(m.xgmi[HOST]['4>4']).toBe(0);
    expect(Object.keys(m.xgmi[HOST]).filter((k) => k.indexOf('-') >= 0)).toEqual([]);
  });

  it('Metrics page: summary says which limits are assumed; every per-GPU cell', async () => {
    const m = await fetchStock();
    const vm = metricsView(cluster(), { metrics: m, fetchError: null, fetching: false }, { now: NOW });
    const s = findSection(vm, 'GPU Power Summary');
    expect(rowValue(s, 'GPUs Monitored')).toBe('8');
    const total = m.gpus.reduce((a, g) => a + g.powerWatts, 0);
    expect(rowValue(s, 'Total Power').text).toBe(total.toFixed(1) + ' W / 11200.0 W (' + Math.round((100 * total) / 11200) + '%)');
    const assumed = rowValue(s, 'Assumed Limits');
    expect(assumed.status).toBe('warning');
    expect(assumed.text).toContain('MI355X board limit; no gpu_power_cap series for 8 of 8 GPUs');
    expect(assumed.text).toContain('throttle threshold 100 °C (MI355X; no gpu_junction_temperature_slowdown series for 8 of 8 GPUs)');
    expect(rowValue(s, 'RAS Errors').status).toBe('error');
    expect(rowValue(s, 'Source')).toBe('AMD Device Metrics Exporter');
    expect(rowValue(s, 'Query')).toContain('gpu_power_usage');

    const t = firstTable(findSection(vm, HOST + ' — 8 × MI355X'));
    expect(t.columns).toEqual(['GPU', 'Power', 'HBM Used', 'GFX', 'HBM Activity', 'Temp', 'ECC', 'Pod']);
    expect(t.rows).toHaveLength(8);
    const r = (g) => t.rows[g];
    // Power against the assumed 1400 W: GPU 0 at 1150 W = 82 % → warning colour.
    expect(r(0)[1].text).toBe('1150.0 W / 1400.0 W (82%)');
    expect(r(7)[1].text).toBe('187.0 W / 1400.0 W (13%)');
    expect(r(0)[2].text).toContain('/ 288 GiB');
    expect(r(0)[3]).toBe('97%');
    expect(r(7)[3]).toBe('0%');
    expect(r(0)[4]).toBe('61%');
    // Junction temperature against the MI355X 100 °C threshold.
    expect(r(2)[5].status).toBe('error');
    expect(r(2)[5].text).toBe('101 °C (throttling at 100 °C)');
    expect(r(3)[5].status).toBe('warning');
    expect(r(0)[5]).toBe('74 °C');
    // RAS: one GPU with corrected, one with uncorrected errors.
    expect(r(5)[6].status).toBe('warning');
    expect(r(6)[6].status).toBe('error');
    expect(r(0)[6]).toBe('OK');
    // Pod ownership from the exporter's pod/namespace labels.
    expect(r(0)[7]).toBe('ml/train-a');
    expect(r(4)[7]).toBe('ml/infer-b');
    expect(r(7)[7]).toBe('—');
  });

  it('GPU Nodes page: exact per-GPU owners, assumed full mesh, xGMI throughput per GPU only (neighbour order unknown)', async () => {
    const m = await fetchStock();
    const vm = nodesView(cluster(), { now: NOW, metrics: m });
    const card = sections(vm).find((x) => x.title === HOST);
    const slots = firstBlock(card, 'slots');
    expect(slots.exact).toBe(true);
    expect(slots.slots.map((x) => x.pod)).toEqual(['train-a', 'train-a', 'train-a', 'train-a', 'infer-b', null, null, null]);
    const mx = firstBlock(card, 'matrix');
    expect(mx.measuredTopology).toBe(false);
    expect(mx.measuredThroughput).toBe(false);
    expect(mx.throughputPerGpu).toBe(true);
    expect(mx.fullMesh).toBe(true);
    expect(mx.matrix.cells[0][1].kind).toBe('xgmi');
    // no link cell claims a measurement; each GPU's total sits on the diagonal
    mx.matrix.cells.forEach((row, i) => row.forEach((c, j) => { if (i !== j) expect(c.measuredGBs).toBeNull(); }));
    const sent = {};
    m.gpus.forEach((g) => { sent[g.gpu] = 0; });
    Object.keys(m.xgmi[HOST]).forEach((k) => { sent[k.split('>')[0]] += m.xgmi[HOST][k]; });
    mx.matrix.cells.forEach((row, i) => expect(row[i].measuredGBs).toBeCloseTo(sent[String(i)], 6));
    const html = renderPage(vm);
    expect(html).toContain('data-topology="assumed" data-throughput="per-gpu"');
    expect(html).not.toContain('link throughput measured');
    expect(html).toContain('xGMI topology (assumed MI355X full mesh; xGMI throughput measured per GPU, neighbour order not reported)');
    expect(renderText(vm)).toContain('xGMI topology (assumed MI355X full mesh; xGMI throughput measured per GPU, neighbour order not reported) — full mesh, 7 links/GPU');
  });

  it('Node detail and GPU Pods pages use the same stock series', async () => {
    const m = await fetchStock();
    const ctx = cluster();
    const sec = nodeDetailView(ctx.gpuNodes[0], ctx, { now: NOW, metrics: m });
    expect(firstBlock(sec, 'matrix').measuredThroughput).toBe(false);
    expect(firstBlock(sec, 'matrix').throughputPerGpu).toBe(true);
    expect(firstBlock(sec, 'slots').exact).toBe(true);
    const pods = firstTable(findSection(podsView(ctx, { now: NOW, metrics: m }), 'All GPU Pods'));
    expect(pods.columns).toContain('Assigned GPUs');
    const byName = {};
    pods.rows.forEach((row) => { byName[row[0]] = row[pods.columns.indexOf('Assigned GPUs')]; });
    expect(byName['train-a']).toBe(HOST + ': GPU 0, 1, 2, 3');
    expect(byName['infer-b']).toBe(HOST + ': GPU 4');
  });
});
