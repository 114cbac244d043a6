/**
 * Real MI355X captures (tests/fixtures/mi355x, taken on a GPU box with
 * tools/capture_box.sh, serials scrubbed) run through the metrics client's
 * join — the exporter schema the plugin assumes, checked against hardware
 * rather than against our own synthetic telemetry.
 */
import fs from 'fs';
import path from 'path';
import { SERIES } from '../../src/api/series.js';
import { joinExporterResults, splitByName } from '../../src/api/telemetry.js';
import { shortProductName } from '../../src/api/amdNodes.js';
import { formatBytes, MI355X } from '../../src/api/k8sCore.js';
import { parseExposition } from './promFake.js';

const DIR = path.join(process.cwd(), 'tests', 'fixtures', 'mi355x');

function load(name) {
  return fs.readFileSync(path.join(DIR, name), 'utf8');
}

describe('MI355X hardware fixtures', () => {
  const rows = parseExposition(load('exporter_once.prom'));
  const smiStatic = JSON.parse(load('amd_smi_static.json')).gpu_data[0];
  const smiMetric = JSON.parse(load('amd_smi_metric.json')).gpu_data[0];

  it('the real exporter scrape carries every per-GPU series the plugin reads', () => {
    const names = rows.map((r) => r.metric.__name__);
    const E = SERIES.exporter;
    [E.power, E.powerCap, E.vramUsed, E.vramTotal, E.gfx, E.umc, E.temp].forEach((n) => expect(names).toContain(n));
  });

  it('joins into one GPU with the board facts amd-smi reports', () => {
    const j = joinExporterResults(splitByName(rows));
    expect(j.gpus).toHaveLength(1);
    const g = j.gpus[0];
    expect(g.nodeName).toBe('mi355x-node-0');
    expect(g.vramTotalBytes).toBe(smiMetric.mem_usage.total_vram.value * 1024 * 1024);
    expect(g.vramTotalBytes).toBe(MI355X.hbmBytes);
    expect(formatBytes(g.vramTotalBytes)).toBe('288 GiB');
    expect(g.powerCapWatts).toBe(smiStatic.limit.ppt0.max_power_limit.value);
    expect(g.powerCapWatts).toBe(MI355X.tdpWatts);
    expect(g.tempC).toBe(smiMetric.temperature.hotspot.value);
    expect(Math.abs(g.powerWatts - smiMetric.power.socket_power.value)).toBeLessThan(30);
  });

  it('amd-smi identifies the board the way the node model expects', () => {
    expect(smiStatic.asic.target_graphics_version).toBe('gfx950');
    expect(smiStatic.asic.num_compute_units).toBe(MI355X.computeUnits);
    expect(shortProductName(smiStatic.asic.device_id, smiStatic.asic.market_name)).toBe('MI355X');
    expect(smiStatic.vram.type).toBe('HBM3E');
    expect(smiStatic.limit.slowdown_hotspot_temperature.value).toBe(MI355X.junctionSlowdownC);
  });
});
