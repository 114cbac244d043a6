/**
 * What the telemetry client reads from Prometheus, by name: the candidate
 * Prometheus services, the AMD series and their labels, and the size limits
 * the paged views ask with. Pure data — the query builders (./promql.js),
 * the joins (./telemetry.js) and the client (./metrics.js) all read it.
 *
 * Reference analog: the constants of src/api/metrics.ts:61-65 (services) and
 * the i915 hwmon names inlined in its queries (:101-116).
 */

/** Candidate Prometheus services, highest priority first (reference metrics.ts:61-65). */
export const PROMETHEUS_SERVICES = [
  { namespace: 'monitoring', service: 'kube-prometheus-stack-prometheus', port: '9090' },
  { namespace: 'monitoring', service: 'prometheus-operated', port: '9090' },
  { namespace: 'monitoring', service: 'prometheus', port: '9090' },
];

export function servicePath(svc) {
  return '/api/v1/namespaces/' + svc.namespace + '/services/' + svc.service + ':' + svc.port + '/proxy';
}

/**
 * Series names. Exporter names follow the AMD Device Metrics Exporter field
 * list (lower-cased); node-exporter names follow its hwmon/drm collectors.
 * (verify both against the deployed versions)
 */
export const SERIES = {
  exporter: {
    power: 'gpu_power_usage', // W
    powerCap: 'gpu_power_cap', // W (board power cap; 1400 on MI355X)
    vramUsed: 'gpu_used_vram', // MiB
    vramTotal: 'gpu_total_vram', // MiB: an MI355X reads 294896 = 288 GiB (tests/fixtures/mi355x)
    gfx: 'gpu_gfx_activity', // %
    umc: 'gpu_umc_activity', // % — HBM controller busy
    temp: 'gpu_junction_temperature', // °C
    tempSlowdown: 'gpu_junction_temperature_slowdown', // °C throttle threshold (this repo's amdgpu-exporter)
    eccCorrect: 'gpu_ecc_correct_total', // corrected RAS errors, all IP blocks
    eccUncorrect: 'gpu_ecc_uncorrect_total', // uncorrected RAS errors, all IP blocks
    xgmiRe: 'xgmi_neighbor_[0-6]_tx_throughput', // bytes/s per neighbour
    linkHops: 'gpu_xgmi_link_hops', // measured link topology (this repo's native amdgpu-exporter)
  },
  // Rows the ONE-node query (promql.js exporterNodeQuery) shapes server-side:
  // xGMI throughput placed on its peer, each GPU's unplaced total, and the
  // count of one-hop xGMI links per GPU (recording-rule style names: they
  // exist only in that answer, no exporter emits them).
  nodeShaped: {
    xgmiLink: 'amdgpu:xgmi_link_tx', // bytes/s on link gpu_id → peer_gpu_id
    xgmiGpu: 'amdgpu:xgmi_gpu_tx', // bytes/s of gpu_id over the links no series pins to a peer
    oneHopLinks: 'amdgpu:xgmi_1hop_links', // one-hop xGMI links of gpu_id
  },
  exporterVramUnitBytes: 1024 * 1024,
  nodeExporter: {
    chips: 'node_hwmon_chip_names{chip_name="amdgpu"}',
    power: 'node_hwmon_power_average_watt',
    // hwmon power1_input. An MI355X exposes power1_input and no power1_average
    // (tests/fixtures/mi355x/sysfs_amdgpu_files.txt), so this is its only power
    // series through node-exporter; the average wins where both exist.
    powerInput: 'node_hwmon_power_input_watt',
    powerCap: 'node_hwmon_power_cap_watt',
    busy: 'node_drm_gpu_busy_percent',
    vramUsed: 'node_drm_memory_vram_used_bytes',
    vramTotal: 'node_drm_memory_vram_size_bytes',
    // hwmon temperatures (m°C read as °C) and their labels: amdgpu's junction
    // sensor is the one labelled "junction" (temp2 on an MI355X; edge reads N/A).
    temp: 'node_hwmon_temp_celsius',
    tempCrit: 'node_hwmon_temp_crit_celsius',
    sensorLabel: 'node_hwmon_sensor_label',
    uname: 'node_uname_info',
  },
};

/** Discovery cache lifetime. Prometheus services move rarely. */
export const DISCOVERY_TTL_MS = 5 * 60 * 1000;
/** Consecutive failed metrics fetches before the page switches to "Prometheus Unreachable". */
export const STALE_FAILURES = 3;
/**
 * GPU nodes (exporter hostnames) up to which a paged view asks for the whole
 * cluster instead of its page: one page of nodes (pages.js NODES_PER_PAGE).
 * Prometheus evaluates the guard inside the same request
 * (smallClusterQuery), so a page opened while the node list is still loading
 * needs no second wave on a small cluster, and a large one gets nothing it
 * did not ask for.
 */
export const SMALL_CLUSTER_NODES = 8;
/**
 * GPU pods (exporter `pod` labels) up to which the Pods page asks for every
 * owner: as many as a cluster of one page of nodes can run (8 × 8 GPUs, one
 * each). Their owner series are at most a few KB; the table still shows one
 * page of PODS_PER_PAGE, and paging through it needs no request.
 */
export const SMALL_CLUSTER_PODS = 64;
/**
 * amdgpu hwmon chips (node-exporter) up to which the first query of a session
 * carries node-exporter's GPU series too (promql.js sourceProbe): one page of
 * 8-GPU nodes. A node-exporter-only cluster of that size then gets its
 * telemetry in the first wave, like an exporter cluster.
 */
export const SMALL_HWMON_GPUS = SMALL_CLUSTER_NODES * 8;

/**
 * Labels the exporter join reads. The combined query projects every series
 * onto them (`max by (...)`), so the response carries no per-series
 * card/driver/serial/job labels: the Device Metrics Exporter attaches a
 * dozen of those to every gauge, which would otherwise dominate the bytes
 * moved through the Headlamp proxy on each refresh. `max` also folds
 * duplicate scrapes of one GPU (two jobs scraping one exporter).
 * `neighbor` is on this repo's exporter's link series only: the link's place
 * in the GPU's neighbour order, which pins the stock exporter's per-neighbour
 * throughput to a peer (topology.js placeThroughput).
 */
export const EXPORTER_JOIN_LABELS = ['__name__', 'hostname', 'node', 'instance', 'gpu_id', 'peer_gpu_id', 'neighbor', 'pod', 'namespace'];

/**
 * The projection of the per-refresh (live-only) query once the static query
 * has shown that every exporter series carries `hostname` (the Device Metrics
 * Exporter labels all its gauges with it): `node` / `instance` are then only
 * fallback keys, and `instance` ("10.0.0.17:5000") is ~18 % of the response
 * bytes. The GPU's `instance` is kept from the static query (STATIC_GPU_FIELDS).
 */
export const EXPORTER_LEAN_LABELS = ['__name__', 'hostname', 'gpu_id', 'peer_gpu_id', 'pod', 'namespace'];

/** Labels the node-exporter join reads (hwmon chip, DRM card, uname). */
export const NODE_EXPORTER_JOIN_LABELS = ['__name__', 'instance', 'node', 'nodename', 'chip', 'chip_name', 'card'];

/**
 * What a cluster-wide fetch is for — each page asks only for the live series
 * it draws (the same idea as the Pods page's ownersQuery):
 *   all       every live gauge and every xGMI link (terminal client, detail fallback);
 *   gauges    the Metrics page: per-GPU power / HBM / activity / temperature /
 *             RAS, no xGMI links (7 of the 14 live series of a GPU);
 *   topology  the GPU Nodes page: per-GPU pod owners and node power (from the
 *             power gauge), the junction temperature (each node's hottest GPU)
 *             and the per-link xGMI throughput of the neighbour matrix.
 */
export const METRIC_VIEWS = ['all', 'gauges', 'topology'];

/** Fields of GpuTelemetry that come from the static series (promql.js exporterNames). */
export const STATIC_GPU_FIELDS = ['powerCapWatts', 'powerCapAssumed', 'vramTotalBytes', 'tempSlowdownC', 'instance'];

/** Key of the cluster-wide line in a scoped series answer (no node name can be this). */
export const TOTAL_SERIES = '\u0000cluster';
