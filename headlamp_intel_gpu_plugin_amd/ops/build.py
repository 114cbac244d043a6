"""Build the native extensions in-tree with hipcc for gfx950.

Extensions (output next to this file so they travel with the repo snapshot
to the GPU box; ``*.so`` is git-ignored):

* ``_amdgpu_probe``  — C++ against the HIP runtime + amdgpu sysfs
  (csrc/amdgpu_probe.cpp);
* ``_workload``      — HIP kernels for gfx950 that the synthetic GPU pods run
  (kernels/workload.hip).

Rebuilds only when a source is newer than its ``.so``. Usage::

    python -m headlamp_intel_gpu_plugin_amd.ops.build [--force]
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from typing import Dict, List

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"

EXTENSIONS: Dict[str, Dict] = {
    "_amdgpu_probe": {"sources": ["csrc/amdgpu_probe.cpp"], "hip": False},
    "_workload": {"sources": ["kernels/workload.hip"], "hip": True},
}


def hipcc() -> str:
    for c in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build the native extensions)")


def so_path(name: str) -> str:
    return os.path.join(HERE, name + ".so")


def _stale(name: str) -> bool:
    out = so_path(name)
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    srcs = [os.path.join(HERE, s) for s in EXTENSIONS[name]["sources"]]
    deps = srcs + [os.path.join(HERE, "kernels", f) for f in os.listdir(os.path.join(HERE, "kernels"))
                   if f.endswith((".h", ".hpp"))] if os.path.isdir(os.path.join(HERE, "kernels")) else srcs
    return any(os.path.exists(s) and os.path.getmtime(s) > t for s in deps)


def command(name: str) -> List[str]:
    spec = EXTENSIONS[name]
    py_inc = sysconfig.get_paths()["include"]
    cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", "-shared", f"-I{py_inc}", "-Wall", "-Wno-unused-function"]
    if spec["hip"]:
        cmd += [f"--offload-arch={ARCH}", "-x", "hip", "-munsafe-fp-atomics"]
    cmd += [os.path.join(HERE, s) for s in spec["sources"]]
    cmd += ["-o", so_path(name), f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"]
    return cmd


def build(names=None, force: bool = False, verbose: bool = False) -> Dict[str, str]:
    """Compile the given extensions (default: all). Returns name → .so path."""
    out = {}
    for name in names or EXTENSIONS:
        src_ok = all(os.path.exists(os.path.join(HERE, s)) for s in EXTENSIONS[name]["sources"])
        if not src_ok:
            continue
        if force or _stale(name):
            cmd = command(name)
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"building {name} failed:\n{r.stderr[-4000:]}")
        out[name] = so_path(name)
    return out


if __name__ == "__main__":
    for k, v in build(force="--force" in sys.argv, verbose=True).items():
        print(k, v)
