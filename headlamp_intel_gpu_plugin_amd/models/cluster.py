"""Synthetic AMD MI355X Kubernetes clusters for tests and the benchmark.

The reference has no fake cluster at all ("no fake API server,
no kind/k3d, no recorded HTTP fixtures, no Prometheus fake"); its multi-node
coverage is two-element fixture arrays. This module generates deterministic
clusters of N nodes × 8 MI355X with:

* AMD node-labeller / NFD labels and ``amd.com/gpu`` capacity;
* the AMD GPU Operator ``DeviceConfig`` CR and its operand pods in
  ``kube-amd-gpu`` (device plugin, node labeller, metrics exporter);
* workload pods requesting ``amd.com/gpu`` (BASELINE config #3: 4 GPU pods per
  8-GPU node), some pending, plus the non-GPU system/app pods every real
  cluster carries — the all-pods list is what dominates at scale;
* a CPU-only control plane.

BASELINE.json configs map to ``PRESETS``.

Label, CRD and pod-naming conventions must match ``src/api/k8sCore.js`` / ``amdNodes.js``; the
JS constants are the single source of truth and tests cross-check them.
"""
from __future__ import annotations

import copy
import dataclasses
import datetime as _dt
import hashlib
from typing import Dict, List, Optional

GPUS_PER_NODE = 8
#: devices per MI355X board in each compute-partition mode (src/api/amdNodes.js COMPUTE_PARTITIONS)
COMPUTE_PARTITIONS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
HBM_BYTES = 294896 * 2**20  # 288 GiB less 16 MiB, as the device reports it (309,220,868,096 B)
OPERATOR_NS = "kube-amd-gpu"
NFD_LABEL = "feature.node.kubernetes.io/amd-gpu"
EPOCH = _dt.datetime(2026, 10, 1, tzinfo=_dt.timezone.utc)


def _ts(days: float = 0.0, hours: float = 0.0) -> str:
    t = EPOCH + _dt.timedelta(days=days, hours=hours)
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


def _uid(*parts: str) -> str:
    h = hashlib.sha1("/".join(parts).encode()).hexdigest()
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:32]}"


@dataclasses.dataclass
class ClusterSpec:
    """Shape of a synthetic cluster."""

    gpu_nodes: int = 1
    gpus_per_node: int = GPUS_PER_NODE
    cpu_nodes: int = 3
    #: GPU counts of the workload pods placed on every GPU node (sum ≤ gpus_per_node)
    pods_per_node: tuple = (1, 1, 2, 2)
    #: extra pending GPU pods per node (unschedulable or image-pulling)
    pending_per_node: int = 1
    #: non-GPU pods per node (daemonsets + apps) — size of the all-pods list
    plain_pods_per_node: int = 24
    operator: bool = True  # DeviceConfig CRD + operator-managed operands
    standalone_plugin: bool = False  # k8s-device-plugin DaemonSets (name=amdgpu-dp-ds)
    node_labeller: bool = True
    metrics_exporter: bool = True
    partition: Optional[str] = None  # e.g. "cpx/nps4"
    seed: int = 0


#: BASELINE.json configs → specs
PRESETS: Dict[str, ClusterSpec] = {
    # 1: CPU-only cluster, mocked CRD, 0 GPU nodes
    "cpu-only": ClusterSpec(gpu_nodes=0, cpu_nodes=3, pods_per_node=(), pending_per_node=0),
    # 2: single 1×MI355X node
    "1x1": ClusterSpec(gpu_nodes=1, gpus_per_node=1, pods_per_node=(1,), pending_per_node=0),
    # 3: single 8×MI355X node, 4 GPU pods
    "1x8": ClusterSpec(gpu_nodes=1),
    # 4: 4 nodes × 8 + Prometheus exporter
    "4x8": ClusterSpec(gpu_nodes=4),
    # 5: 8-node scaling point
    "8x8": ClusterSpec(gpu_nodes=8),
}


def spec_for_nodes(n: int) -> ClusterSpec:
    """Scaling-curve spec: ``n`` nodes of 8×MI355X (n=0 → CPU-only)."""
    if n <= 0:
        return copy.deepcopy(PRESETS["cpu-only"])
    return ClusterSpec(gpu_nodes=n)


def gpu_node_name(i: int) -> str:
    return f"mi355x-{i:03d}"


def _node(name: str, labels: Dict[str, str], capacity: Dict[str, str], age_days: float, ready: bool = True) -> dict:
    alloc = dict(capacity)
    alloc["cpu"] = str(int(capacity["cpu"]) - 1)
    return {
        "apiVersion": "v1",
        "kind": "Node",
        "metadata": {
            "name": name,
            "uid": _uid("node", name),
            "labels": labels,
            "creationTimestamp": _ts(days=-age_days),
            "resourceVersion": "1",
        },
        "spec": {},
        "status": {
            "capacity": capacity,
            "allocatable": alloc,
            "conditions": [
                {"type": "MemoryPressure", "status": "False"},
                {"type": "DiskPressure", "status": "False"},
                {"type": "Ready", "status": "True" if ready else "False"},
            ],
            "nodeInfo": {
                "osImage": "Ubuntu 24.04.1 LTS",
                "kernelVersion": "6.8.0-52-generic",
                "kubeletVersion": "v1.31.4",
                "architecture": "amd64",
                "containerRuntimeVersion": "containerd://1.7.24",
            },
            "addresses": [{"type": "Hostname", "address": name}],
        },
    }


def _pod(name: str, ns: str, node: Optional[str], containers: List[dict], phase: str = "Running",
         labels: Optional[dict] = None, init: Optional[List[dict]] = None, waiting: Optional[str] = None,
         restarts: int = 0, age_hours: float = 2.0, sched_msg: Optional[str] = None) -> dict:
    ready = phase == "Running"
    statuses = []
    for c in containers:
        st = {"running": {"startedAt": _ts(hours=-age_hours)}} if ready else {}
        if waiting:
            st = {"waiting": {"reason": waiting}}
        statuses.append({"name": c["name"], "ready": ready, "restartCount": restarts, "image": c.get("image", ""), "state": st})
    conds = [{"type": "Ready", "status": "True" if ready else "False"}]
    if node is None:
        c = {"type": "PodScheduled", "status": "False", "reason": "Unschedulable"}
        if sched_msg:
            c["message"] = sched_msg
        conds.append(c)
    pod = {
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {
            "name": name,
            "namespace": ns,
            "uid": _uid("pod", ns, name),
            "labels": labels or {},
            "creationTimestamp": _ts(hours=-age_hours),
            "resourceVersion": "1",
        },
        "spec": {"containers": containers},
        "status": {"phase": phase, "conditions": conds, "containerStatuses": statuses if node else []},
    }
    if node:
        pod["spec"]["nodeName"] = node
    if init:
        pod["spec"]["initContainers"] = init
    return pod


def _gpu_container(name: str, gpus: int, image: str = "rocm/pytorch:rocm7.0_ubuntu24.04_py3.12_pytorch_2.8") -> dict:
    return {
        "name": name,
        "image": image,
        "resources": {
            "requests": {"amd.com/gpu": str(gpus), "cpu": "8", "memory": "64Gi"},
            "limits": {"amd.com/gpu": str(gpus), "memory": "128Gi"},
        },
    }


class SyntheticCluster:
    """Deterministic cluster state (nodes, pods, DeviceConfigs)."""

    def __init__(self, spec: ClusterSpec):
        self.spec = spec
        self.nodes: List[dict] = []
        self.pods: List[dict] = []
        self.device_configs: List[dict] = []
        #: (node, gpu index) → (namespace, pod) for workload pods — feeds exporter pod labels
        self.gpu_owner: Dict[tuple, tuple] = {}
        self._build()

    # ------------------------------------------------------------------
    def _build(self) -> None:
        s = self.spec
        for i in range(s.cpu_nodes):
            name = f"cp-{i}"
            self.nodes.append(_node(name, {"node-role.kubernetes.io/control-plane": "", "kubernetes.io/hostname": name},
                                    {"cpu": "32", "memory": "128Gi", "pods": "110"}, age_days=30))
        for i in range(s.gpu_nodes):
            name = gpu_node_name(i)
            labels = {
                "kubernetes.io/hostname": name,
                NFD_LABEL: "true",
                "feature.node.kubernetes.io/pci-1002.present": "true",
            }
            if s.node_labeller:
                labels.update({
                    "amd.com/gpu.product-name": "AMD_Instinct_MI355X",
                    "amd.com/gpu.family": "AI",
                    "amd.com/gpu.device-id": "75a3",
                    "amd.com/gpu.vram": "288G",
                    "amd.com/gpu.cu-count": "256",
                    "amd.com/gpu.simd-count": "1024",
                    "amd.com/gpu.driver-version": "6.12.12",
                })
            devices = s.gpus_per_node
            if s.partition:
                cp, mp = s.partition.split("/")
                labels["amd.com/compute-partitioning-mode"] = cp
                labels["amd.com/memory-partitioning-mode"] = mp
                # Each MI355X (8 XCDs) exposes one device per compute partition.
                devices *= COMPUTE_PARTITIONS.get(cp.upper(), 1)
            capacity = {"cpu": "256", "memory": "3Ti", "pods": "110", "amd.com/gpu": str(devices)}
            self.nodes.append(_node(name, labels, capacity, age_days=14))
        self._operator_objects()
        self._workloads()
        self._plain_pods()

    def _operator_objects(self) -> None:
        s = self.spec
        n = s.gpu_nodes
        if s.operator:
            self.device_configs.append({
                "apiVersion": "amd.com/v1alpha1",
                "kind": "DeviceConfig",
                "metadata": {"name": "gpu-operator", "namespace": OPERATOR_NS, "uid": _uid("dc", "gpu-operator"),
                             "creationTimestamp": _ts(days=-14), "generation": 1},
                "spec": {
                    "driver": {"enable": False},
                    "devicePlugin": {"devicePluginImage": "rocm/k8s-device-plugin:latest",
                                     "nodeLabellerImage": "rocm/k8s-device-plugin:labeller-latest",
                                     "enableNodeLabeller": s.node_labeller},
                    "metricsExporter": {"enable": s.metrics_exporter, "port": 5000, "serviceType": "ClusterIP",
                                        "image": "rocm/device-metrics-exporter:v1.3.0"},
                    "selector": {NFD_LABEL: "true"},
                },
                "status": {
                    "devicePlugin": {"nodesMatchingSelectorNumber": n, "desiredNumber": n, "availableNumber": n},
                    "nodeLabeller": {"nodesMatchingSelectorNumber": n, "desiredNumber": n if s.node_labeller else 0,
                                     "availableNumber": n if s.node_labeller else 0},
                    "metricsExporter": {"nodesMatchingSelectorNumber": n, "desiredNumber": n if s.metrics_exporter else 0,
                                        "availableNumber": n if s.metrics_exporter else 0},
                },
            })
            self.pods.append(_pod("amd-gpu-operator-gpu-operator-charts-controller-manager-7d9f8", OPERATOR_NS, "cp-0",
                                  [{"name": "manager", "image": "rocm/gpu-operator:v1.3.0"}],
                                  labels={"app.kubernetes.io/name": "gpu-operator-charts"}, age_hours=24 * 14))
        for i in range(n):
            node = gpu_node_name(i)
            suffix = hashlib.sha1(node.encode()).hexdigest()[:5]
            if s.operator:
                self.pods.append(_pod(f"gpu-operator-device-plugin-{suffix}", OPERATOR_NS, node,
                                      [{"name": "device-plugin", "image": "rocm/k8s-device-plugin:latest"}],
                                      labels={"daemonset-name": "gpu-operator-device-plugin"}, age_hours=24 * 14))
                if s.node_labeller:
                    self.pods.append(_pod(f"gpu-operator-node-labeller-{suffix}", OPERATOR_NS, node,
                                          [{"name": "node-labeller"}], labels={"daemonset-name": "gpu-operator-node-labeller"},
                                          age_hours=24 * 14))
                if s.metrics_exporter:
                    self.pods.append(_pod(f"gpu-operator-metrics-exporter-{suffix}", OPERATOR_NS, node,
                                          [{"name": "metrics-exporter"}], labels={"daemonset-name": "gpu-operator-metrics-exporter"},
                                          age_hours=24 * 14, restarts=1 if i == 0 else 0))
            if s.standalone_plugin:
                self.pods.append(_pod(f"amdgpu-device-plugin-daemonset-{suffix}", "kube-system", node,
                                      [{"name": "amdgpu-dp-cntr"}], labels={"name": "amdgpu-dp-ds"}, age_hours=24 * 7))
                self.pods.append(_pod(f"amdgpu-labeller-daemonset-{suffix}", "kube-system", node,
                                      [{"name": "amdgpu-labeller-cntr"}], labels={"name": "amdgpu-labeller-ds"}, age_hours=24 * 7))

    def _workloads(self) -> None:
        s = self.spec
        for i in range(s.gpu_nodes):
            node = gpu_node_name(i)
            slot = 0
            for j, g in enumerate(s.pods_per_node):
                if slot + g > s.gpus_per_node:
                    break
                name = f"train-{i:03d}-{j}"
                init = None
                if j == 3:  # one pod per node runs a GPU warm-up init container
                    init = [{"name": "rccl-warmup", "resources": {"limits": {"amd.com/gpu": str(g)}}}]
                self.pods.append(_pod(name, "ml", node, [_gpu_container("trainer", g)], init=init, age_hours=3 + j))
                for k in range(g):
                    self.gpu_owner[(node, slot + k)] = ("ml", name)
                slot += g
            for j in range(s.pending_per_node):
                # kube-scheduler's fit-error wording: no GPU node has 8 free GPUs
                n_all = s.gpu_nodes + s.cpu_nodes
                msg = (f"0/{n_all} nodes are available: {s.gpu_nodes} Insufficient amd.com/gpu"
                       + (f", {s.cpu_nodes} node(s) didn't match Pod's node affinity/selector" if s.cpu_nodes else "") + ".")
                self.pods.append(_pod(f"queued-{i:03d}-{j}", "ml", None, [_gpu_container("trainer", 8)],
                                      phase="Pending", age_hours=0.2, sched_msg=msg))
        # one finished job on the first node
        if s.gpu_nodes > 0 and s.pods_per_node:
            self.pods.append(_pod("eval-000-done", "ml", gpu_node_name(0), [_gpu_container("eval", 1)],
                                  phase="Succeeded", age_hours=20))

    def _plain_pods(self) -> None:
        s = self.spec
        names = [n["metadata"]["name"] for n in self.nodes]
        ds = ["kube-proxy", "node-exporter", "calico-node", "fluent-bit", "csi-node"]
        for node in names:
            suffix = hashlib.sha1(node.encode()).hexdigest()[:5]
            for d in ds:
                self.pods.append(_pod(f"{d}-{suffix}", "kube-system", node,
                                      [{"name": d, "image": f"registry.k8s.io/{d}:v1",
                                        "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}}}],
                                      labels={"app": d}, age_hours=24 * 14))
        gpu_nodes = [gpu_node_name(i) for i in range(s.gpu_nodes)] or names
        total = s.plain_pods_per_node * max(1, s.gpu_nodes)
        for k in range(total):
            node = gpu_nodes[k % len(gpu_nodes)]
            self.pods.append(_pod(f"web-{k:04d}", "apps", node,
                                  [{"name": "web", "image": "nginx:1.27",
                                    "resources": {"requests": {"cpu": "250m", "memory": "256Mi"}}}],
                                  labels={"app": "web"}, age_hours=10))

    # ------------------------------------------------------------------
    @property
    def gpu_nodes(self) -> List[dict]:
        return [n for n in self.nodes if NFD_LABEL in n["metadata"]["labels"]]

    def gpu_pods(self) -> List[dict]:
        out = []
        for p in self.pods:
            for c in p["spec"].get("containers", []) + p["spec"].get("initContainers", []):
                res = c.get("resources", {})
                keys = list(res.get("requests", {})) + list(res.get("limits", {}))
                if any(k.startswith("amd.com/") for k in keys):
                    out.append(p)
                    break
        return out

    def operator_pods(self) -> List[dict]:
        return [p for p in self.pods if p["metadata"]["namespace"] == OPERATOR_NS
                or p["metadata"]["labels"].get("name") in ("amdgpu-dp-ds", "amdgpu-labeller-ds")]

    def expected_counts(self) -> Dict[str, int]:
        """What the dashboard should render for this cluster (test oracle)."""
        gp = self.gpu_pods()
        return {
            "gpu_nodes": self.spec.gpu_nodes,
            "gpus": self.spec.gpu_nodes * self.spec.gpus_per_node,
            "gpu_pods": len(gp),
            "running_gpu_pods": sum(1 for p in gp if p["status"]["phase"] == "Running"),
            "pending_gpu_pods": sum(1 for p in gp if p["status"]["phase"] == "Pending"),
            "gpus_in_use": len(self.gpu_owner),
            "operator_pods": len(self.operator_pods()),
            "device_configs": len(self.device_configs),
        }
