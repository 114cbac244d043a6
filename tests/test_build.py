"""The native extensions cross-compile for gfx950 here (no GPU needed) and import."""
import os
import shutil

import pytest

from headlamp_intel_gpu_plugin_amd.ops import build as native_build

pytestmark = pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")),
                                reason="hipcc not available")


def test_extensions_build_and_import():
    built = native_build.build()
    assert set(built) == {"_amdgpu_probe", "_workload", "amdgpu-exporter"}
    from headlamp_intel_gpu_plugin_amd.ops import probe, workload

    assert probe.native().device_count() >= 0
    assert workload.tile() == (128, 128, 64)


def test_workload_targets_gfx950():
    cmd = native_build.command("_workload")
    assert "--offload-arch=gfx950" in cmd


def test_probe_reports_absence_cleanly_without_gpu():
    from headlamp_intel_gpu_plugin_amd.ops import probe

    if probe.native().device_count() == 0:
        assert not probe.available()
        assert "hip" in probe.native().last_error().lower() or probe.native().last_error() == ""


def test_parse_exposition_roundtrip():
    from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition

    text = '# HELP x y\ngpu_power_usage{hostname="n\\"1",gpu_id="0"} 712.5\n'
    assert parse_exposition(text) == [("gpu_power_usage", {"hostname": 'n"1', "gpu_id": "0"}, 712.5)]


def test_workload_rejects_cpu_tensors():
    import torch

    from headlamp_intel_gpu_plugin_amd.ops import workload

    a = torch.zeros(128, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        workload.gemm_bf16_nt(a, a)
    with pytest.raises(TypeError):
        workload.gemm_bf16_nt(a.float(), a.float())


def test_concurrent_builds_do_not_clobber_each_other(tmp_path):
    # One rank per GPU may all find an extension stale at start-up; the build
    # lock + atomic rename must leave one complete, loadable library.
    import subprocess
    import sys

    from headlamp_intel_gpu_plugin_amd.ops import build as b

    so = b.so_path("_amdgpu_probe")
    if os.path.exists(so):
        os.utime(so, (0, 0))  # make it stale for every process below
    code = ("from headlamp_intel_gpu_plugin_amd.ops import build as b; "
            "b.build(['_amdgpu_probe']); "
            "import importlib; m = importlib.import_module('headlamp_intel_gpu_plugin_amd.ops._amdgpu_probe'); "
            "print('ok', m.device_count() >= 0)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = [subprocess.Popen([sys.executable, "-c", code], cwd=root, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for _ in range(3)]
    outs = [p.communicate(timeout=600) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-500:] for o in outs]
    assert all("ok True" in o[0] for o in outs)
    assert not [f for f in os.listdir(os.path.dirname(so)) if ".tmp" in f]
