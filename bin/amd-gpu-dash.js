#!/usr/bin/env node
/**
 * amd-gpu-dash — the plugin's dashboard in a terminal.
 *
 * Runs the plugin's own data layer (src/api: cluster store, metrics client)
 * and view-models (src/view/pages/*.js) against a cluster reached through
 * `kubectl proxy` (or any URL that speaks the Kubernetes API with the
 * caller's credentials), and prints the pages with the text renderer. Same
 * requests, same degradation rules, same numbers as the Headlamp pages.
 *
 *   kubectl proxy --port 8001 &
 *   node bin/amd-gpu-dash.js --url http://127.0.0.1:8001 --page nodes
 *   node bin/amd-gpu-dash.js --page all --watch 10 --color
 *   node bin/amd-gpu-dash.js --prometheus monitoring/my-prom:9090 --page metrics
 *   node bin/amd-gpu-dash.js --json --page pods          # the view-model IR
 *   node bin/amd-gpu-dash.js --svg --page nodes > nodes.svg   # a picture of the page
 *
 * Plain ES2019 modules: runs on the Node 12 of the development image.
 */
import http from 'http';
import https from 'https';
import { createClusterStore } from '../src/api/clusterStore.js';
import { createMetricsSource } from '../src/api/metrics.js';
import { parsePrometheus, prometheusCandidates } from '../src/api/settings.js';
import { nodeDetailView, podDetailView } from '../src/view/pages/details.js';
import { devicePluginsView } from '../src/view/pages/devicePlugins.js';
import { metricsView } from '../src/view/pages/metricsPage.js';
import { nodesView } from '../src/view/pages/nodes.js';
import { overviewView } from '../src/view/pages/overview.js';
import {
  NODE_SORTS,
  NODES_PER_PAGE,
  POD_SORTS,
  PODS_PER_PAGE,
  RANKED_NODE_SORTS,
  RANKED_POD_SORTS,
} from '../src/view/pages/paging.js';
import { podsView } from '../src/view/pages/pods.js';
import { renderPageSvg, renderSectionSvg } from '../src/view/svg.js';
import { renderText, textSection } from '../src/view/text.js';
import { PAGE_NEEDS } from '../src/plugin.js';

const PAGES = ['overview', 'device-plugins', 'nodes', 'pods', 'metrics'];

function usage(msg) {
  if (msg) process.stderr.write('amd-gpu-dash: ' + msg + '\n');
  process.stderr.write(
    'usage: amd-gpu-dash [--url http://127.0.0.1:8001] [--page ' + PAGES.join('|') + '|all|node:NAME|pod:NS/NAME]\n' +
      '                    [--watch SECONDS] [--filter TEXT] [--page-number N] [--per-page N]\n' +
      '                    [--sort name|in-use|free|attention (nodes) | gpus|newest|attention (pods) | power (nodes, metrics, pods)]\n' +
      '                    [--prometheus NAMESPACE/SERVICE:PORT] [--timeout MS] [--token TOKEN] [--insecure]\n' +
      '                    [--color] [--json | --svg]\n'
  );
  process.exit(2);
}

export function parseArgs(argv) {
  const a = { url: 'http://127.0.0.1:8001', page: 'overview', watch: 0, prometheus: null, timeout: 2000,
    token: null, insecure: false, color: false, json: false, svg: false, pager: { page: 0, filter: '' } };
  for (let i = 0; i < argv.length; i++) {
    const k = argv[i];
    const v = argv[i + 1];
    if (k === '--url') a.url = v;
    else if (k === '--page') a.page = v;
    else if (k === '--watch') a.watch = Number(v);
    else if (k === '--timeout') a.timeout = Number(v);
    // The paged lists (GPU nodes, GPU / operator pods): which page, and a name filter (pages.js nodePage / podPage).
    else if (k === '--filter') a.pager.filter = v;
    else if (k === '--page-number') a.pager.page = Number(v) - 1;
    else if (k === '--per-page') a.pager.perPage = Number(v);
    // The GPU node order (pages.js NODE_SORTS): name, most GPUs in use / free, not ready first.
    else if (k === '--sort') a.pager.sort = v;
    else if (k === '--token') a.token = v;
    else if (k === '--prometheus') {
      const m = /^([^/]+)\/([^:]+):(.+)$/.exec(v || '');
      a.prometheus = m ? parsePrometheus({ namespace: m[1], service: m[2], port: m[3] }) : null;
      if (!a.prometheus) return { error: 'bad --prometheus ' + v + ' (want namespace/service:port)' };
    } else if (k === '--insecure') {
      a.insecure = true;
      continue;
    } else if (k === '--color') {
      a.color = true;
      continue;
    } else if (k === '--json') {
      a.json = true;
      continue;
    } else if (k === '--svg') {
      // One page or detail section as an SVG picture (src/view/svg.js), once.
      a.svg = true;
      continue;
    } else if (k === '--help' || k === '-h') return { error: '' };
    else return { error: 'unknown argument ' + k };
    if (v === undefined) return { error: 'missing value for ' + k };
    i++;
  }
  // node:NAME / pod:NAMESPACE/NAME — the sections the plugin adds to Headlamp's native detail pages.
  const node = /^node:(.+)$/.exec(a.page);
  const pod = /^pod:([^/]+)\/(.+)$/.exec(a.page);
  if (node) a.detail = { kind: 'node', name: node[1] };
  else if (pod) a.detail = { kind: 'pod', namespace: pod[1], name: pod[2] };
  else if (a.page !== 'all' && PAGES.indexOf(a.page) < 0) return { error: 'unknown page ' + a.page };
  if (!(a.watch >= 0) || !(a.timeout > 0)) return { error: 'bad --watch / --timeout' };
  if (a.svg && (a.json || a.watch > 0 || a.page === 'all')) return { error: '--svg draws one page once (no --json, --watch or --page all)' };
  if (!(a.pager.page >= 0) || (a.pager.perPage !== undefined && !(a.pager.perPage > 0))) return { error: 'bad --page-number / --per-page' };
  // Node orders apply to the GPU node pages, pod orders to GPU Pods ('name' to both).
  const sorts = NODE_SORTS.concat(POD_SORTS, RANKED_NODE_SORTS, RANKED_POD_SORTS).map(function (o) { return o.value; })
    .filter(function (v, i, all) { return all.indexOf(v) === i; });
  if (a.pager.sort !== undefined && sorts.indexOf(a.pager.sort) < 0) return { error: 'bad --sort (one of ' + sorts.join(', ') + ')' };
  return a;
}

/** GET path → parsed JSON; rejects with `.status` set on HTTP errors (like Headlamp's ApiProxy). */
function makeRequest(a) {
  const base = new URL(a.url);
  const mod = base.protocol === 'https:' ? https : http;
  const agent = new mod.Agent({ keepAlive: true, maxSockets: 6, rejectUnauthorized: !a.insecure });
  const prefix = base.pathname.replace(/\/$/, '');
  return function request(path) {
    return new Promise(function (resolve, reject) {
      const headers = { Accept: 'application/json' };
      if (a.token) headers.Authorization = 'Bearer ' + a.token;
      const req = mod.get(
        { protocol: base.protocol, hostname: base.hostname, port: base.port, path: prefix + path, agent: agent, headers: headers },
        function (res) {
          const chunks = [];
          res.on('data', function (c) { chunks.push(c); });
          res.on('end', function () {
            let json = null;
            try {
              json = JSON.parse(Buffer.concat(chunks).toString('utf8'));
            } catch (e) {
              json = null;
            }
            if (res.statusCode >= 400) {
              if (json && json.status === 'error') return resolve(json); // Prometheus error body
              const err = new Error((json && json.message) || 'HTTP ' + res.statusCode);
              err.status = res.statusCode;
              return reject(err);
            }
            if (json === null) return reject(new Error('bad JSON from ' + path));
            resolve(json);
          });
        }
      );
      req.on('error', reject);
    });
  };
}

export function views(ctx, mstate, page, pager) {
  const opts = { metrics: mstate.metrics, pager: pager };
  const all = {
    overview: function () { return overviewView(ctx, opts); },
    'device-plugins': function () { return devicePluginsView(ctx, opts); },
    nodes: function () { return nodesView(ctx, opts); },
    pods: function () { return podsView(ctx, opts); },
    metrics: function () { return metricsView(ctx, mstate, opts); },
  };
  return (page === 'all' ? PAGES : [page]).map(function (p) { return all[p](); });
}

async function main() {
  const a = parseArgs(process.argv.slice(2));
  if (a.error !== undefined) usage(a.error);
  const request = makeRequest(a);
  const store = createClusterStore({ request: request, timeoutMs: a.timeout });
  const settings = { prometheus: a.prometheus };
  const metrics = createMetricsSource({ request: request, timeoutMs: a.timeout, services: prometheusCandidates(settings) });
  const mstate = { metrics: null, series: null, fetchError: null, fetching: false };

  // Telemetry per page, as the plugin's pages ask for it (ADR 008): none for
  // Overview / Device Plugins, the page's view for Nodes / Metrics, every
  // series for `all`; range series only where the Metrics page draws them.
  const VIEW = { all: 'all', nodes: 'topology', pods: 'owners', metrics: 'gauges' };
  const view = VIEW[a.page] || null;

  // Detail sections: the node's (or the pod's node's) telemetry + the power
  // history, one wave, as src/plugin.js wires the native detail pages.
  async function showDetail(first) {
    await Promise.all(first ? [store.refresh(), store.loadLists()] : [store.refresh()]);
    const ctx = store.getSnapshot();
    const d = a.detail;
    let section = null;
    let what = d.kind + ' ' + (d.namespace ? d.namespace + '/' : '') + d.name;
    if (d.kind === 'node') {
      const n = ctx.gpuNodes.filter(function (x) { return x.metadata.name === d.name; })[0];
      if (n) {
        const r = await Promise.all([metrics.fetchNodeMetrics(d.name), metrics.fetchNodeSeries(d.name, 1800, 30)]);
        section = nodeDetailView(n, ctx, { metrics: r[0], series: r[1] });
      } else what += ' (not an AMD GPU node, or not found)';
    } else {
      const p = ctx.gpuPods.filter(function (x) { return x.metadata.name === d.name && (x.metadata.namespace || '') === d.namespace; })[0];
      if (p) {
        const node = p.spec && p.spec.nodeName;
        const r = await Promise.all([
          node ? metrics.fetchNodeMetrics(node) : Promise.resolve(null),
          metrics.fetchPodSeries(d.namespace, d.name, 1800, 30),
        ]);
        section = podDetailView(p, { metrics: r[0], series: r[1] });
      } else what += ' (not a GPU pod, or not found)';
    }
    if (a.json) {
      process.stdout.write(JSON.stringify(section) + '\n');
      return;
    }
    if (a.svg) {
      process.stdout.write(renderSectionSvg(section || { t: 'section', title: 'No AMD GPU section for ' + what, key: 'none', blocks: [] }));
      return;
    }
    if (a.watch > 0) process.stdout.write('\u001b[2J\u001b[H');
    process.stdout.write(section ? textSection(section, a.color).join('\n') + '\n' : 'No AMD GPU section for ' + what + '\n');
  }
  if (a.detail) {
    await showDetail(true);
    while (a.watch > 0) {
      await new Promise(function (r) { setTimeout(r, a.watch * 1000); });
      await store.loadLists();
      await showDetail(false);
    }
    return;
  }

  // --sort power on one page: Prometheus ranks and returns that page (metrics.js rankedClusterQuery / rankedOwnersQuery).
  const rank = a.pager.sort === 'power' && (view === 'topology' || view === 'gauges' || view === 'owners')
    ? { by: 'power', page: a.pager.page, per: a.pager.perPage || (view === 'owners' ? PODS_PER_PAGE : NODES_PER_PAGE),
      filter: (a.pager.filter || '').trim().toLowerCase() }
    : null;

  // The lists the page draws, as its plugin route mounts them (PAGE_NEEDS):
  // Device Plugins reads its operator pods with the plugin-pod requests
  // (store.refresh, no pod list), Metrics the node list alone.
  const byAllocation = a.pager.sort === 'in-use' || a.pager.sort === 'free'; // Metrics ranks nodes by GPUs pods hold
  const needs = a.page === 'metrics' && byAllocation ? { nodes: true, pods: true } : PAGE_NEEDS[a.page] || { nodes: true, pods: true };
  function loadLists() {
    return needs.nodes || needs.pods ? store.loadLists({ nodes: needs.nodes, pods: needs.pods }) : Promise.resolve();
  }

  async function fetchAll(first) {
    const jobs = [
      store.refresh(),
      view === 'owners' ? metrics.fetchGpuOwners(rank ? { rank: rank } : undefined)
        : view ? metrics.fetchGpuMetrics(view, rank ? { rank: rank, summary: view === 'gauges' } : undefined) : Promise.resolve(null),
      view === 'all' || view === 'gauges' ? metrics.fetchSeries(1800, 30) : Promise.resolve(null),
    ];
    if (first) jobs.push(loadLists());
    const r = await Promise.all(jobs);
    mstate.metrics = r[1];
    mstate.series = r[2];
    mstate.fetchError = r[1] || !view ? null : 'Could not reach Prometheus';
  }

  function print() {
    const vms = views(store.getSnapshot(), mstate, a.page, a.pager);
    if (a.json) {
      process.stdout.write(JSON.stringify(vms.length === 1 ? vms[0] : vms) + '\n');
      return;
    }
    if (a.svg) {
      process.stdout.write(renderPageSvg(vms[0]));
      return;
    }
    if (a.watch > 0) process.stdout.write('\u001b[2J\u001b[H');
    process.stdout.write(vms.map(function (vm) { return renderText(vm, { color: a.color }); }).join('\n') + '\n');
  }

  await fetchAll(true);
  print();
  while (a.watch > 0) {
    await new Promise(function (r) { setTimeout(r, a.watch * 1000); });
    await loadLists(); // no watch here: re-list what the page draws each cycle
    await fetchAll(false);
    print();
  }
}

if (process.argv[1] && /amd-gpu-dash(\.js)?$/.test(process.argv[1])) {
  main().then(
    function () { process.exit(0); },
    function (e) {
      process.stderr.write('amd-gpu-dash: ' + (e && e.stack ? e.stack : e) + '\n');
      process.exit(1);
    }
  );
}
