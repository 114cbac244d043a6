/**
 * MI355X node topology: per-GPU allocation slots and the xGMI neighbour matrix.
 *
 * Not present in the reference (it has no topology concept — SURVEY.md §7.1
 * "Topology | none"). An 8×MI355X node is a point-to-point xGMI full mesh:
 * every GPU has 7 links, one to each peer, ≈153 GB/s per link (task brief /
 * MI355X_MICROARCH.md). Ring collectives over that mesh are per-link bound,
 * which is why the panel shows per-link figures rather than one node number.
 *
 * Kubernetes does not expose which device a pod holds. When the metrics
 * exporter attaches `pod`/`namespace` labels to per-GPU series, slots are
 * exact; otherwise they are filled in pod order and flagged `inferred`.
 */

import { getNodeGpuCount, partitionsPerGpu } from './amdNodes.js';
import { podFacts } from './clusterIndex.js';
import { MI355X } from './k8sCore.js';

/**
 * One schedulable device. On a partitioned node (DPX/QPX/CPX) device `index`
 * is partition `partition` of board `board`; otherwise board === index and
 * partition is null.
 * @typedef {{ index: number, board: number, partition: number|null, pod: string|null, namespace: string|null,
 *             inferred: boolean }} GpuSlot
 */

/**
 * @param {any} node
 * @param {any[]} podsOnNode  GPU pods bound to the node
 * @param {Array<{gpu: string, pod?: string|null, namespace?: string|null}>} [perGpuOwners]
 *        exporter-derived owners keyed by gpu index (as string)
 * @param {{capacity: number, partitionsPerGpu: number}} [dims]  the node's device count and partitions per
 *        board when the caller has them (clusterIndex.js nodeFacts), instead of reading the node's labels again
 * @returns {{ slots: GpuSlot[], exact: boolean, partitionsPerGpu: number }}
 */
export function buildGpuSlots(node, podsOnNode, perGpuOwners, dims) {
  const n = (dims ? dims.capacity : getNodeGpuCount(node)) || 0;
  const pp = dims ? dims.partitionsPerGpu : partitionsPerGpu(node);
  const slots = [];
  for (let i = 0; i < n; i++) {
    slots.push({
      index: i, board: Math.floor(i / pp), partition: pp > 1 ? i % pp : null, pod: null, namespace: null, inferred: false,
    });
  }
  if (perGpuOwners && perGpuOwners.length) {
    for (let i = 0; i < perGpuOwners.length; i++) {
      const o = perGpuOwners[i];
      const idx = parseInt(o.gpu, 10);
      if (idx >= 0 && idx < n && o.pod) {
        slots[idx].pod = o.pod;
        slots[idx].namespace = o.namespace || null;
      }
    }
    return { slots: slots, exact: true, partitionsPerGpu: pp };
  }
  let next = 0;
  for (let p = 0; p < podsOnNode.length; p++) {
    const pod = podsOnNode[p];
    // What the pod holds (0 once terminated), derived when the pod list arrived.
    const g = podFacts(pod).gpus;
    for (let k = 0; k < g && next < n; k++, next++) {
      slots[next].pod = pod.metadata.name;
      slots[next].namespace = pod.metadata.namespace || null;
      slots[next].inferred = true;
    }
  }
  return { slots: slots, exact: false, partitionsPerGpu: pp };
}

const placeCache = typeof WeakMap === 'function' ? new WeakMap() : null;

/**
 * Measured xGMI throughput of one node (telemetry.js join: "src-dst" when the
 * series named the peer, "src>k" for neighbour k) placed on the matrix:
 *   * "src-dst" as given;
 *   * "src>k" on the peer whose link series carries `neighbor: k` (this
 *     repo's amdgpu-exporter publishes its KFD io_link order) — else on no
 *     peer: the stock exporter does not say which peer its neighbour k is,
 *     and KFD does not promise index order;
 *   * "i-i": GPU i's throughput summed over all its rows, placed or not —
 *     the figure that needs no neighbour order.
 * → {map, pinned: a row landed on a peer, perGpu: a total exists}; null
 * without measurements. Cached on the maps (their identity holds while the
 * values do).
 * @param {Record<string, number>|null|undefined} measured
 * @param {Record<string, {type: string, hops: number, neighbor?: number}>|null|undefined} probed
 */
export function placeThroughput(measured, probed) {
  if (!measured || typeof measured !== 'object') return null;
  if (placeCache) {
    const hit = placeCache.get(measured);
    if (hit && hit.probed === (probed || null)) return hit.placed;
  }
  let byNeighbor = null;
  if (probed) {
    for (const k in probed) {
      const p = probed[k];
      const dash = k.indexOf('-');
      if (!p || typeof p.neighbor !== 'number' || dash <= 0) continue;
      (byNeighbor || (byNeighbor = {}))[k.slice(0, dash) + '>' + p.neighbor] = k.slice(dash + 1);
    }
  }
  const map = {};
  let pinned = false;
  let perGpu = false;
  for (const key in measured) {
    const v = measured[key];
    if (typeof v !== 'number') continue;
    const dash = key.indexOf('-');
    let src;
    let dst;
    if (dash > 0) {
      src = key.slice(0, dash);
      dst = key.slice(dash + 1);
      if (dst === src) continue;
    } else {
      const gt = key.indexOf('>');
      if (gt <= 0) continue;
      src = key.slice(0, gt);
      dst = byNeighbor ? byNeighbor[key] : undefined;
    }
    if (dst !== undefined) {
      map[src + '-' + dst] = v;
      pinned = true;
    }
    const self = src + '-' + src;
    map[self] = (map[self] || 0) + v;
    perGpu = true;
  }
  const placed = perGpu ? { map: map, pinned: pinned, perGpu: perGpu } : null;
  if (placeCache) placeCache.set(measured, { probed: probed || null, placed: placed });
  return placed;
}

/**
 * xGMI neighbour matrix for one node.
 *
 * @param {number} gpuCount
 * @param {Record<string, number>} [measured]  GB/s observed (exporter xGMI
 *        throughput series, telemetry.js keys), optional; placed by placeThroughput
 * @param {Record<string, {type: string, hops: number, neighbor?: number}>} [probed]  `${src}-${dst}` →
 *        link type/hops from the exporter's link series (KFD io_links / hipExtGetLinkTypeAndHopCount)
 * @returns {{ size: number, cells: Array<Array<{ kind: 'self'|'xgmi'|'pcie'|'none', hops: number, peakGBs: number, measuredGBs: number|null }>>,
 *             linksPerGpu: number, perGpuPeakGBs: number, ringBusGBs: number }}
 *          a `self` cell's measuredGBs is the GPU's xGMI throughput summed over its links
 */
export function buildXgmiMatrix(gpuCount, measured, probed) {
  const n = gpuCount > 0 ? gpuCount : 0;
  const placed = placeThroughput(measured, probed);
  const pm = placed ? placed.map : null;
  const cells = [];
  let linksPerGpu = 0;
  for (let i = 0; i < n; i++) {
    const row = [];
    let links = 0;
    for (let j = 0; j < n; j++) {
      const key = i + '-' + j;
      const m = pm && typeof pm[key] === 'number' ? pm[key] : null;
      if (i === j) {
        row.push({ kind: 'self', hops: 0, peakGBs: 0, measuredGBs: m });
        continue;
      }
      let kind = 'xgmi';
      let hops = 1;
      if (probed) {
        // A measured topology is authoritative: a pair it does not list is not
        // xGMI-connected.
        const p = probed[key];
        kind = !p ? 'none' : p.type === 'XGMI' ? 'xgmi' : p.type === 'PCIE' ? 'pcie' : 'none';
        hops = p ? p.hops : 0;
      }
      if (kind === 'xgmi') links++;
      row.push({ kind: kind, hops: hops, peakGBs: kind === 'xgmi' ? MI355X.xgmiLinkGBs : 0, measuredGBs: m });
    }
    if (links > linksPerGpu) linksPerGpu = links;
    cells.push(row);
  }
  return {
    size: n,
    cells: cells,
    linksPerGpu: linksPerGpu,
    perGpuPeakGBs: linksPerGpu * MI355X.xgmiLinkGBs,
    // A ring all-reduce moves each byte over one link per step, so its bus
    // bandwidth is bounded by a single link, not by the sum of the mesh.
    ringBusGBs: linksPerGpu > 0 ? MI355X.xgmiLinkGBs : 0,
  };
}

/** "i-j" link keys of the maps, made once: a lookup by an interned string skips hashing a new one. */
const LINK_KEYS = [];
function linkKey(i, j) {
  const row = LINK_KEYS[i] || (LINK_KEYS[i] = []);
  return row[j] || (row[j] = i + '-' + j);
}

const factCache = typeof WeakMap === 'function' ? new WeakMap() : null;

/**
 * What buildXgmiMatrix + isFullMesh say of a node's links, without the grid:
 * {fullMesh, linksPerGpu, stats, gpuStats} — `stats` ({links, meanGBs,
 * maxGBs} | null) over the throughput placed on xGMI links (every pair of
 * distinct GPUs in the platform model; the pairs `probed` types XGMI
 * otherwise), `gpuStats` ({gpus, meanGBs, maxGBs} | null) over the per-GPU
 * totals (placeThroughput). Cached on the map objects (the metrics client
 * keeps a map's identity while its values are unchanged; the measured
 * topology is static), so a page that re-renders reads it once per answer.
 * The metrics client derives them when an answer arrives
 * (nodeSummaries.js primeSnapshot).
 * @param {number} n  GPUs of the node
 * @param {Record<string, number>|null} measured
 * @param {Record<string, {type: string, hops: number, neighbor?: number}>|null} probed  (non-empty, or null)
 */
export function linkFacts(n, measured, probed) {
  const key = measured || probed;
  if (factCache && key) {
    const hit = factCache.get(key);
    if (hit && hit.n === n && hit.measured === measured && hit.probed === probed) return hit.facts;
  }
  let linksPerGpu = probed ? 0 : Math.max(0, n - 1);
  let full = n > 1;
  let cnt = 0;
  let sum = 0;
  let max = 0;
  let gCnt = 0;
  let gSum = 0;
  let gMax = 0;
  const placed = placeThroughput(measured, probed);
  const pm = placed ? placed.map : null;
  if (probed || pm) {
    for (let i = 0; i < n; i++) {
      let links = 0;
      for (let j = 0; j < n; j++) {
        const k = linkKey(i, j);
        if (i === j) {
          const t = pm ? pm[k] : undefined;
          if (typeof t === 'number') {
            gCnt++;
            gSum += t;
            if (t > gMax) gMax = t;
          }
          continue;
        }
        let xgmi = true;
        if (probed) {
          const p = probed[k];
          xgmi = !!p && p.type === 'XGMI';
          if (!xgmi || p.hops !== 1) full = false;
          if (xgmi) links++;
        }
        const v = pm && placed.pinned && xgmi ? pm[k] : undefined;
        if (typeof v === 'number') {
          cnt++;
          sum += v;
          if (v > max) max = v;
        }
      }
      if (probed && links > linksPerGpu) linksPerGpu = links;
    }
  }
  const facts = {
    fullMesh: full,
    linksPerGpu: linksPerGpu,
    stats: cnt ? { links: cnt, meanGBs: sum / cnt, maxGBs: max } : null,
    gpuStats: gCnt ? { gpus: gCnt, meanGBs: gSum / gCnt, maxGBs: gMax } : null,
  };
  if (factCache && key) factCache.set(key, { n: n, measured: measured, probed: probed, facts: facts });
  return facts;
}

/** True when the matrix is the full point-to-point mesh an 8×MI355X node should have. */
export function isFullMesh(matrix) {
  if (matrix.size < 2) return false;
  for (let i = 0; i < matrix.size; i++) {
    for (let j = 0; j < matrix.size; j++) {
      if (i !== j && (matrix.cells[i][j].kind !== 'xgmi' || matrix.cells[i][j].hops !== 1)) return false;
    }
  }
  return true;
}
