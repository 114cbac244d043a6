"""RAS / ECC counters of the native probe (ops/csrc/probe_core.h read_ras).

The MI355X tree is rebuilt from a capture of a real card's ``ras/`` directory
(tests/fixtures/mi355x/sysfs_ras.txt, tools/diag/ras_capture.sh): per-block
``aca_*`` files of ``ue/ce/de`` counts, ``event_state``, ``features`` and an
empty ``gpu_vram_bad_pages``. Pure file parsing, so these run on the CPU.
"""
import os
import shutil

import pytest

from headlamp_intel_gpu_plugin_amd.ops import probe

HAS_HIPCC = bool(shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc"))
pytestmark = pytest.mark.skipif(not HAS_HIPCC, reason="hipcc not available")

FIXTURE = os.path.join(os.path.dirname(__file__), "fixtures", "mi355x", "sysfs_ras.txt")


def captured_tree(root):
    """Write the captured ras/ files under ``root``; returns the block names."""
    files, cur = {}, None
    with open(FIXTURE) as f:
        for line in f:
            if line.startswith("-- "):
                cur = os.path.basename(line[3:].strip())
                files[cur] = ""
            elif cur is not None:
                files[cur] += line
    os.makedirs(root, exist_ok=True)
    for name, text in files.items():
        with open(os.path.join(root, name), "w") as f:
            f.write(text.strip("\n") + ("\n" if text.strip() else ""))
    return sorted(n for n in files if n.startswith("aca_"))


@pytest.fixture(scope="module")
def native():
    from headlamp_intel_gpu_plugin_amd.ops import build as native_build
    native_build.build(["_amdgpu_probe"])
    return probe


def test_mi355x_capture_reads_zero_counters(native, tmp_path):
    blocks = captured_tree(str(tmp_path / "ras"))
    assert blocks == ["aca_gfx", "aca_jpeg", "aca_mmhub", "aca_sdma", "aca_umc", "aca_vcn", "aca_xgmi_wafl"]
    r = native.read_ras(str(tmp_path / "ras"))
    assert r == {"ce": 0.0, "ue": 0.0, "de": 0.0, "retired_pages": 0.0, "blocks": len(blocks)}


def test_counts_sum_over_blocks_and_retired_pages(native, tmp_path):
    d = tmp_path / "ras"
    captured_tree(str(d))
    (d / "aca_umc").write_text("ue: 1\nce: 17\nde: 2\n")
    (d / "aca_xgmi_wafl").write_text("ue: 0\nce: 3\nde: 0\n")
    (d / "gpu_vram_bad_pages").write_text("0x00000123 : 0x00001000 : R\n0x00000456 : 0x00001000 : R\n\n")
    r = native.read_ras(str(d))
    assert (r["ce"], r["ue"], r["de"], r["retired_pages"]) == (20.0, 1.0, 2.0, 2.0)


def test_legacy_err_count_files_when_no_aca(native, tmp_path):
    d = tmp_path / "ras"
    d.mkdir()
    (d / "umc_err_count").write_text("ue: 0\nce: 5\n")
    (d / "gfx_err_count").write_text("ue: 2\nce: 1\n")
    (d / "features").write_text("feature mask: 0x1\n")
    r = native.read_ras(str(d))
    assert (r["ce"], r["ue"], r["de"], r["blocks"]) == (6.0, 2.0, None, 2)
    assert r["retired_pages"] is None  # no bad-page table: not reported, not zero


def test_aca_files_win_over_legacy_duplicates(native, tmp_path):
    d = tmp_path / "ras"
    d.mkdir()
    (d / "aca_umc").write_text("ue: 0\nce: 4\nde: 0\n")
    (d / "umc_err_count").write_text("ue: 0\nce: 4\n")
    assert native.read_ras(str(d))["ce"] == 4.0


def test_missing_directory_reports_nothing(native, tmp_path):
    r = native.read_ras(str(tmp_path / "absent"))
    assert r["blocks"] == 0 and r["ce"] is None and r["ue"] is None


def test_exporter_help_declares_ecc_counters(tmp_path):
    from headlamp_intel_gpu_plugin_amd.ops import build as native_build
    import subprocess
    exe = native_build.build(["amdgpu-exporter"])["amdgpu-exporter"]
    out = subprocess.run([exe, "--once", "--hostname", "n0"], capture_output=True, text=True, timeout=60).stdout
    assert "# TYPE gpu_ecc_correct_total counter" in out
    assert "# TYPE gpu_ecc_uncorrect_total counter" in out
    assert "# TYPE gpu_ecc_retired_pages gauge" in out


@pytest.mark.gpu
def test_real_card_reports_ras_counters(native):
    assert native.available()
    s = native.sample(0)
    # An MI355X exposes ras/aca_* (tests/fixtures/mi355x/sysfs_ras.txt): the
    # counters are numbers (normally 0), never absent.
    assert s["ecc_correct"] is not None and s["ecc_uncorrect"] is not None
    assert s["ecc_correct"] >= 0 and s["ecc_uncorrect"] >= 0
    text = native.render_metrics("n0")
    assert "gpu_ecc_correct_total{" in text and "gpu_ecc_uncorrect_total{" in text
