#!/usr/bin/env node
/**
 * Verify a plugin archive — the exact file a release uploads — by loading it.
 *
 *   node tools/verify_archive.js dist-offline/amd-gpu-X.Y.Z.tar.gz [--sha256 <hex>]
 *
 * Gunzips and untars the archive, checks its layout (`<name>/main.js`,
 * `<name>/package.json`, nothing else) and manifest, then evaluates the
 * archive's own main.js the way Headlamp evaluates a plugin script: one
 * script, the host library handed in as `pluginLib` (here the harness
 * stand-ins of tests/js/stubs). It checks every extension point the reference
 * registers (/root/reference/src/index.tsx:35-182): 6 sidebar entries, 5
 * routes, 2 detail sections, 1 column processor — and mounts each route, both
 * detail sections and the columns on a small MI355X cluster. Prints one JSON
 * line; exits 1 on any failure.
 *
 * The release job runs this on the archive it then publishes
 * (.github/workflows/release.yaml); the CPU gate runs it on the archive the
 * tree builds (tests/test_package.py).
 */
import crypto from 'crypto';
import fs from 'fs';
import path from 'path';
import { fileURLToPath } from 'url';
import zlib from 'zlib';
import React, { render } from '../tests/js/stubs/react.js';
import * as lib from '../tests/js/stubs/headlamp-lib.js';
import * as CC from '../tests/js/stubs/CommonComponents.js';
import { makeDeviceConfig, makeGpuNode, makeGpuPod, makeNode, makePlainPod, makePluginPod } from '../tests/js/fixtures.js';

const ROOT = path.resolve(path.dirname(fileURLToPath(import.meta.url)), '..');
const h = React.createElement;

export const EXPECTED = {
  sidebar: ['AMD GPU', 'Overview', 'Device Plugins', 'GPU Nodes', 'GPU Pods', 'Metrics'],
  routes: ['/amd-gpu', '/amd-gpu/device-plugins', '/amd-gpu/nodes', '/amd-gpu/pods', '/amd-gpu/metrics'],
  titles: ['AMD GPU — Overview', 'AMD GPU — Device Plugins', 'AMD GPU — Nodes', 'AMD GPU — Pods', 'AMD GPU — Metrics'],
  detailSections: 2,
  columnProcessors: 1,
  columns: ['GPU Model', 'GPU Devices', 'GPU HBM'],
};

/** ustar entries of a tar buffer → [{name, body}]. */
export function untar(tar) {
  const out = [];
  let off = 0;
  while (off + 512 <= tar.length) {
    const hdr = tar.subarray(off, off + 512);
    if (hdr.every(function (b) { return b === 0; })) break;
    const name = hdr.subarray(0, 100).toString('ascii').replace(/\0.*$/, '');
    const size = parseInt(hdr.subarray(124, 136).toString('ascii').replace(/\0.*$/, '').trim(), 8);
    const type = String.fromCharCode(hdr[156] || 0x30);
    if (!(size >= 0)) throw new Error('archive: bad size in tar header of ' + JSON.stringify(name));
    out.push({ name: name, type: type, body: tar.subarray(off + 512, off + 512 + size) });
    off += 512 + Math.ceil(size / 512) * 512;
  }
  return out;
}

function check(cond, msg, errors) {
  if (!cond) errors.push(msg);
}

function cluster() {
  lib.lists.Node = [[makeGpuNode('mi355x-0'), makeGpuNode('mi355x-1'), makeNode('cpu-0')], null];
  lib.lists.Pod = [[makeGpuPod('train-a', { gpus: 4 }), makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' }), makePlainPod('web-0'),
    makePluginPod('amdgpu-dp-0')], null];
  lib.api.handler = function (p) {
    if (/deviceconfigs$/.test(p)) return Promise.resolve({ kind: 'List', metadata: {}, items: [makeDeviceConfig()] });
    return Promise.reject(Object.assign(new Error('503 Service Unavailable'), { status: 503 }));
  };
}

/**
 * Verify the archive bytes → {ok, errors, summary}. `expect` may name the
 * manifest (`name`, `version`) and `sha256` the archive must have.
 */
export async function verifyArchive(bytes, expect) {
  expect = expect || {};
  const errors = [];
  const summary = { bytes: bytes.length, sha256: crypto.createHash('sha256').update(bytes).digest('hex') };
  if (expect.sha256) check(summary.sha256 === expect.sha256, 'sha256 ' + summary.sha256 + ' is not the expected ' + expect.sha256, errors);
  let entries;
  try {
    entries = untar(zlib.gunzipSync(bytes));
  } catch (e) {
    return { ok: false, errors: errors.concat(['not a gzip tar archive: ' + e.message]), summary: summary };
  }
  const pkg = JSON.parse(fs.readFileSync(path.join(ROOT, 'package.json'), 'utf8'));
  const name = expect.name || pkg.name;
  summary.entries = entries.map(function (e) { return e.name; });
  check(JSON.stringify(summary.entries) === JSON.stringify([name + '/main.js', name + '/package.json']),
    'entries ' + JSON.stringify(summary.entries) + ' are not [' + name + '/main.js, ' + name + '/package.json]', errors);
  entries.forEach(function (e) { check(e.type === '0', e.name + ' is not a regular file', errors); });
  const main = entries.find(function (e) { return e.name === name + '/main.js'; });
  const manifest = entries.find(function (e) { return e.name === name + '/package.json'; });
  if (manifest) {
    const m = JSON.parse(manifest.body.toString('utf8'));
    summary.version = m.version;
    check(m.name === name, 'manifest name ' + m.name + ' is not ' + name, errors);
    if (expect.version) check(m.version === expect.version, 'manifest version ' + m.version + ' is not ' + expect.version, errors);
    check(m.main === 'main.js', 'manifest main ' + m.main + ' is not main.js', errors);
  }
  if (!main) return { ok: false, errors: errors.concat(['no main.js']), summary: summary };
  lib.resetHeadlamp();
  const pluginLib = Object.assign({}, lib, { React: React, CommonComponents: Object.assign({}, CC) });
  let mod;
  try {
    // eslint-disable-next-line no-new-func
    mod = new Function('pluginLib', 'return (' + main.body.toString('utf8').trim().replace(/;$/, '') + '\n);')(pluginLib);
  } catch (e) {
    return { ok: false, errors: errors.concat(['main.js does not evaluate: ' + e.message]), summary: summary };
  }
  const reg = lib.registry;
  summary.registered = {
    sidebar: reg.sidebar.length, routes: reg.routes.length, detailSections: reg.details.length, columnProcessors: reg.columns.length,
  };
  check(JSON.stringify(reg.sidebar.map(function (e) { return e.label; })) === JSON.stringify(EXPECTED.sidebar),
    'sidebar ' + JSON.stringify(reg.sidebar.map(function (e) { return e.label; })), errors);
  check(JSON.stringify(reg.routes.map(function (r) { return r.path; })) === JSON.stringify(EXPECTED.routes),
    'routes ' + JSON.stringify(reg.routes.map(function (r) { return r.path; })), errors);
  reg.routes.forEach(function (r) { check(r.exact === true, 'route ' + r.path + ' is not exact', errors); });
  check(reg.details.length === EXPECTED.detailSections, reg.details.length + ' detail sections', errors);
  check(reg.columns.length === EXPECTED.columnProcessors, reg.columns.length + ' column processors', errors);
  check(mod && mod.registered && mod.registered.routes === 5, 'the entry module does not report its registrations', errors);
  if (errors.length) return { ok: false, errors: errors, summary: summary };

  cluster();
  summary.mounted = [];
  for (let i = 0; i < reg.routes.length; i++) {
    const r = render(h(reg.routes[i].component));
    await r.settle();
    const text = r.text();
    check(text.indexOf(EXPECTED.titles[i]) >= 0, reg.routes[i].path + ' does not render ' + JSON.stringify(EXPECTED.titles[i]), errors);
    summary.mounted.push(reg.routes[i].path);
    r.unmount();
  }
  const nodeSec = reg.details.map(function (f) { return f({ resource: { kind: 'Node', jsonData: makeGpuNode('mi355x-1') } }); }).filter(Boolean);
  const podSec = reg.details.map(function (f) { return f({ resource: { kind: 'Pod', jsonData: makeGpuPod('train-b', { gpus: 2, node: 'mi355x-1' }) } }); })
    .filter(Boolean);
  check(nodeSec.length === 1 && podSec.length === 1, 'one Node and one Pod section expected, got ' + nodeSec.length + ' and ' + podSec.length, errors);
  for (const el of [nodeSec[0], podSec[0]]) {
    if (!el) continue;
    const r = render(el);
    await r.settle();
    check(r.text().indexOf('AMD GPU') >= 0, 'a detail section does not render its AMD GPU title', errors);
    summary.mounted.push(el === nodeSec[0] ? 'node-detail' : 'pod-detail');
    r.unmount();
  }
  const cols = reg.columns[0]({ id: 'headlamp-nodes', columns: [{ label: 'Name' }] });
  check(JSON.stringify(cols.map(function (c) { return c.label; })) === JSON.stringify(['Name'].concat(EXPECTED.columns)),
    'headlamp-nodes columns ' + JSON.stringify(cols.map(function (c) { return c.label; })), errors);
  const other = [{ label: 'Name' }];
  check(reg.columns[0]({ id: 'headlamp-pods', columns: other }) === other, 'the column processor changes a table other than headlamp-nodes', errors);
  summary.mounted.push('headlamp-nodes columns');
  lib.resetHeadlamp();
  return { ok: errors.length === 0, errors: errors, summary: summary };
}

async function main(argv) {
  let file = null;
  const expect = {};
  for (let i = 0; i < argv.length; i++) {
    if (argv[i] === '--sha256') expect.sha256 = argv[++i].replace(/^sha256:/, '');
    else if (argv[i] === '--version') expect.version = argv[++i];
    else if (!file) file = argv[i];
    else {
      process.stderr.write('usage: node tools/verify_archive.js <archive.tar.gz> [--sha256 <hex>] [--version X.Y.Z]\n');
      return 2;
    }
  }
  if (!file) {
    process.stderr.write('usage: node tools/verify_archive.js <archive.tar.gz> [--sha256 <hex>] [--version X.Y.Z]\n');
    return 2;
  }
  const res = await verifyArchive(fs.readFileSync(file), expect);
  process.stdout.write(JSON.stringify(Object.assign({ archive: path.basename(file), ok: res.ok, errors: res.errors }, res.summary)) + '\n');
  return res.ok ? 0 : 1;
}

if (process.argv[1] && path.resolve(process.argv[1]) === fileURLToPath(import.meta.url)) {
  main(process.argv.slice(2)).then(function (code) { process.exitCode = code; }, function (e) {
    process.stderr.write(String(e && e.stack || e) + '\n');
    process.exitCode = 1;
  });
}
