"""tools/render_compare.py: opt-in only (ADR 014), and the pooling of several driver processes' samples."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import render_compare  # noqa: E402


def test_refuses_to_run_the_reference_without_the_flag(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "render_compare.py"), "--out", str(tmp_path / "x")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "--allow-reference-exec" in r.stderr
    assert not (tmp_path / "x.json").exists()


def _run(ref_mounts, amd_mounts):
    def side(ms):
        return {"mount": ms, "rerender": [m / 4 for m in ms], "elements": 10}
    page = {"reference": {"elements": 10, "mountMs": sorted(ref_mounts)[len(ref_mounts) // 2]},
            "amd": {"elements": 8, "mountMs": sorted(amd_mounts)[len(amd_mounts) // 2]},
            "samples": {"reference": side(ref_mounts), "amd": side(amd_mounts),
                        "prebuilt": {"mount": [m * 0.7 for m in amd_mounts], "vm": [m * 0.3 for m in amd_mounts]}}}
    return {"gpuPods": 6, "referenceProviderFilterMs": 0.1, "pages": {"nodes": page}}


def test_pooling_recomputes_the_quantiles_over_every_process_sample():
    runs = [_run([1.0, 1.0, 1.0], [0.9, 0.9, 0.9]), _run([2.0, 2.0, 2.0], [1.1, 1.1, 1.1]), _run([3.0, 3.0, 3.0], [3.0, 3.0, 3.0])]
    p = render_compare.pooled(runs)
    a, ref = p["pages"]["nodes"]["amd"], p["pages"]["nodes"]["reference"]
    assert p["runs"] == 3 and ref["reps"] == 9 and a["reps"] == 9
    assert ref["mountMs"] == 2.0 and ref["mountQ1"] == 1.0 and ref["mountQ3"] == 3.0
    assert a["mountMs"] == 1.1 and a["runMountMs"] == [0.9, 1.1, 3.0]
    assert render_compare.verdict(a, ref) == "≤"
    assert abs(a["vmBuildMs"] - 0.33) < 1e-9 and "samples" not in p["pages"]["nodes"]


def test_verdict():
    ref = {"mountMs": 1.0, "mountQ3": 1.2}
    assert render_compare.verdict({"mountMs": 0.9}, ref) == "≤"
    assert render_compare.verdict({"mountMs": 1.1}, ref) == "≈"
    assert render_compare.verdict({"mountMs": 1.3}, ref) == ">"
