"""Build `_workload` variants for same-process A/B (tools/ab_two_builds.py).

    python tools/build_variants.py NAME=-DFLAG[,-DFLAG2] [NAME2=...]

Each variant is the in-tree `kernels/workload.hip` compiled with extra flags
into `tools/microbench/<NAME>/_workload.so` (git-ignored); the in-tree build
itself is brought up to date first.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from headlamp_intel_gpu_plugin_amd.ops import build as B  # noqa: E402


def main(argv):
    B.build(["_workload"])
    rc = 0
    for spec in argv:
        name, _, flags = spec.partition("=")
        out_dir = os.path.join(ROOT, "tools", "microbench", name)
        os.makedirs(out_dir, exist_ok=True)
        cmd = B.command("_workload", os.path.join(out_dir, "_workload.so")) + [f for f in flags.split(",") if f]
        r = subprocess.run(cmd, capture_output=True, text=True)
        print(name, "ok" if r.returncode == 0 else "FAILED", flags, r.stderr[-2000:], flush=True)
        rc |= r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
