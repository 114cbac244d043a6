"""Deployment manifests agree with the code they deploy (deploy/)."""
import os
import re
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")
JS = open(os.path.join(ROOT, "src", "api", "k8sCore.js")).read()
METRICS_JS = open(os.path.join(ROOT, "src", "api", "series.js")).read()


def docs(path):
    with open(os.path.join(DEPLOY, path)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def by_kind(ds, kind):
    return [d for d in ds if d["kind"] == kind]


def js_const(name):
    m = re.search(r"export const " + name + r" = '([^']*)'", JS)
    assert m, name
    return m.group(1)


def test_exporter_manifests_are_consistent():
    ds = docs("exporter/daemonset.yaml")
    dset = by_kind(ds, "DaemonSet")[0]
    svc = by_kind(ds, "Service")[0]
    sm = by_kind(ds, "ServiceMonitor")[0]
    pod_labels = dset["spec"]["template"]["metadata"]["labels"]
    assert dset["spec"]["selector"]["matchLabels"].items() <= pod_labels.items()
    assert svc["spec"]["selector"].items() <= pod_labels.items()
    assert sm["spec"]["selector"]["matchLabels"].items() <= svc["metadata"]["labels"].items()
    port_names = {p["name"] for p in svc["spec"]["ports"]}
    assert {e["port"] for e in sm["spec"]["endpoints"]} <= port_names
    # Runs where the plugin looks for operator pods, on the NFD-labelled GPU nodes.
    assert dset["metadata"]["namespace"] == js_const("AMD_GPU_OPERATOR_NAMESPACE")
    assert js_const("AMD_NFD_GPU_LABEL") in dset["spec"]["template"]["spec"]["nodeSelector"]
    assert "metrics-exporter" in dset["metadata"]["name"]  # classified as the metrics-exporter operand


def test_exporter_daemonset_is_least_privilege():
    ds = docs("exporter/daemonset.yaml")
    pod = by_kind(ds, "DaemonSet")[0]["spec"]["template"]["spec"]
    c = pod["containers"][0]
    sc = c["securityContext"]
    assert sc.get("privileged") is not True and sc["allowPrivilegeEscalation"] is False
    assert sc["readOnlyRootFilesystem"] is True and sc["capabilities"]["drop"] == ["ALL"]
    assert pod["securityContext"]["runAsNonRoot"] is True and pod["securityContext"]["runAsUser"] != 0
    # No device nodes and no host /dev: the exporter runs without the HIP runtime.
    assert "--sysfs-only" in c["args"]
    host_paths = [v["hostPath"]["path"] for v in pod["volumes"] if "hostPath" in v]
    assert host_paths == ["/sys"]
    assert all(m.get("readOnly") for m in c["volumeMounts"])
    # A pinned image, and ingress only from Prometheus on the metrics port.
    assert not c["image"].endswith(":latest") and (":" in c["image"].split("/")[-1] or "@sha256:" in c["image"])
    np = by_kind(ds, "NetworkPolicy")[0]
    assert np["spec"]["podSelector"]["matchLabels"].items() <= pod_labels_of(ds).items()
    assert [p["port"] for r in np["spec"]["ingress"] for p in r["ports"]] == ["metrics"]


def pod_labels_of(ds):
    return by_kind(ds, "DaemonSet")[0]["spec"]["template"]["metadata"]["labels"]


def test_exporter_daemonset_args_are_accepted_by_the_binary():
    from headlamp_intel_gpu_plugin_amd.ops import build as native_build

    exe = native_build.build(["amdgpu-exporter"])["amdgpu-exporter"]
    c = by_kind(docs("exporter/daemonset.yaml"), "DaemonSet")[0]["spec"]["template"]["spec"]["containers"][0]
    args = [a.replace("$(NODE_NAME)", "node-a") for a in c["args"]]
    r = subprocess.run([exe] + args + ["--once"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "# TYPE gpu_power_usage gauge" in r.stdout
    probes = [c["readinessProbe"]["httpGet"]["path"], c["livenessProbe"]["httpGet"]["path"]]
    assert probes == ["/healthz", "/healthz"]


def test_viewer_rbac_covers_every_request_the_plugin_makes():
    ds = docs("rbac/headlamp-amd-gpu-viewer.yaml")
    rules = by_kind(ds, "ClusterRole")[0]["rules"]

    def allowed(group, resource, verb):
        return any(group in r["apiGroups"] and resource in r["resources"] and verb in r["verbs"] for r in rules)

    assert allowed("", "nodes", "watch") and allowed("", "pods", "list") and allowed("", "pods", "watch")
    assert allowed(js_const("AMD_GPU_OPERATOR_API_GROUP"), "deviceconfigs", "list")
    role = by_kind(ds, "Role")[0]
    namespaces = set(re.findall(r"namespace: '([a-z-]+)'", METRICS_JS))
    assert namespaces == {role["metadata"]["namespace"]}
    assert role["rules"][0]["resources"] == ["services/proxy"] and role["rules"][0]["verbs"] == ["get"]
    # read-only: no write verbs anywhere
    for d in by_kind(ds, "ClusterRole") + by_kind(ds, "Role"):
        for r in d["rules"]:
            assert not set(r["verbs"]) & {"create", "update", "patch", "delete", "deletecollection"}


@pytest.mark.parametrize("path", ["exporter/Dockerfile"])
def test_dockerfile_builds_the_same_source(path):
    text = open(os.path.join(DEPLOY, path)).read()
    assert "amdgpu_exporter.cpp" in text and "EXPOSE 9400" in text
