"""Hardware captures from an MI355X box (tests/fixtures/mi355x, tools/capture_box.sh).

They pin the assumptions the native probe and the synthetic cluster make about
real hardware: sysfs file names, units and board facts.
"""
import json
import os
import re

from headlamp_intel_gpu_plugin_amd.models.cluster import HBM_BYTES, SyntheticCluster, spec_for_nodes
from headlamp_intel_gpu_plugin_amd.models.telemetry import BOARD_POWER_W
from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "fixtures", "mi355x")
PROBE = open(os.path.join(ROOT, "headlamp_intel_gpu_plugin_amd", "ops", "csrc", "probe_core.h")).read()


def _json(name):
    with open(os.path.join(FIX, name)) as f:
        return json.load(f)["gpu_data"][0]


def test_probe_reads_sysfs_files_that_exist_on_mi355x():
    files = set(open(os.path.join(FIX, "sysfs_amdgpu_files.txt")).read().split())
    read = set(re.findall(r'"/((?:gpu_busy|mem_info_vram|current_|power1_|temp\d_|freq\d_)[a-z_0-9]*)"', PROBE))
    assert read, "probe_core.h reads no sysfs files?"
    # temp%d / freq%d names are built at run time; check the ones the capture lists
    assert {"gpu_busy_percent", "mem_info_vram_used", "mem_info_vram_total", "current_compute_partition",
            "current_memory_partition", "power1_input", "power1_cap", "freq1_input", "freq2_input",
            "temp2_input", "temp2_label"} <= files
    # power1_average is the pre-MI300 name; MI355X has only power1_input, which
    # the probe falls back to.
    assert "power1_average" not in files
    assert read - {"power1_average"} <= files, read - files


def test_synthetic_cluster_matches_device_capacity_and_power_cap():
    smi = _json("amd_smi_metric.json")
    static = _json("amd_smi_static.json")
    assert smi["mem_usage"]["total_vram"]["value"] * 2**20 == HBM_BYTES
    assert static["limit"]["ppt0"]["max_power_limit"]["value"] == BOARD_POWER_W
    node = SyntheticCluster(spec_for_nodes(1)).gpu_nodes[0]
    assert "0x" + node["metadata"]["labels"]["amd.com/gpu.device-id"] == static["asic"]["device_id"]
    assert int(node["metadata"]["labels"]["amd.com/gpu.cu-count"]) == static["asic"]["num_compute_units"]


def test_exporter_capture_units():
    rows = {n: v for n, _, v in parse_exposition(open(os.path.join(FIX, "exporter_once.prom")).read())}
    smi = _json("amd_smi_metric.json")
    assert rows["gpu_total_vram"] == smi["mem_usage"]["total_vram"]["value"]  # MiB on both sides
    assert rows["gpu_junction_temperature"] == smi["temperature"]["hotspot"]["value"]
    assert rows["gpu_memory_temperature"] == smi["temperature"]["mem"]["value"]
    assert rows["gpu_power_cap"] == BOARD_POWER_W
    limits = _json("amd_smi_static.json")["limit"]
    assert rows["gpu_junction_temperature_slowdown"] == limits["slowdown_hotspot_temperature"]["value"]
    assert rows["gpu_junction_temperature_shutdown"] == limits["shutdown_hotspot_temperature"]["value"]
    assert rows["gpu_memory_temperature_slowdown"] == limits["slowdown_vram_temperature"]["value"]
    labels = [lb for n, lb, _ in parse_exposition(open(os.path.join(FIX, "exporter_once.prom")).read())
              if n == "gpu_power_usage"][0]
    assert labels["card_model"] == "AMD Instinct MI355X"
