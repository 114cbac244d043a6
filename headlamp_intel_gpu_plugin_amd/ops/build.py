"""Build the native code in-tree with hipcc for gfx950.

Targets (outputs next to this file so they travel with the repo snapshot to
the GPU box; ``*.so`` and ``bin/`` are git-ignored):

* ``_amdgpu_probe``   CPython extension — C++ over the HIP runtime + amdgpu
  sysfs (csrc/amdgpu_probe.cpp + csrc/probe_core.h);
* ``_workload``       CPython extension — HIP kernels for gfx950 run by the
  synthetic GPU pods (kernels/workload.hip);
* ``amdgpu-exporter`` standalone Prometheus exporter daemon built from the
  same probe core (csrc/amdgpu_exporter.cpp) → ``bin/amdgpu-exporter``.

Rebuilds only when a source (or header) is newer than its output. Usage::

    python -m headlamp_intel_gpu_plugin_amd.ops.build [--force]
"""
from __future__ import annotations

import fcntl
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import Dict, List

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"

TARGETS: Dict[str, Dict] = {
    "_amdgpu_probe": {"sources": ["csrc/amdgpu_probe.cpp"], "hip": False, "kind": "ext"},
    "_workload": {"sources": ["kernels/workload.hip"], "hip": True, "kind": "ext"},
    "amdgpu-exporter": {"sources": ["csrc/amdgpu_exporter.cpp"], "hip": False, "kind": "exe"},
}
# Backwards-compatible alias used by the import helper.
EXTENSIONS = TARGETS


def hipcc() -> str:
    for c in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build the native code)")


def so_path(name: str) -> str:
    """Output path of a target (``.so`` for extensions, ``bin/<name>`` for executables)."""
    if TARGETS[name]["kind"] == "exe":
        return os.path.join(HERE, "bin", name)
    return os.path.join(HERE, name + ".so")


def _deps(name: str) -> List[str]:
    srcs = [os.path.join(HERE, s) for s in TARGETS[name]["sources"]]
    headers = glob.glob(os.path.join(HERE, "csrc", "*.h")) + glob.glob(os.path.join(HERE, "kernels", "*.h"))
    return srcs + headers


def _stale(name: str) -> bool:
    out = so_path(name)
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.exists(s) and os.path.getmtime(s) > t for s in _deps(name))


def command(name: str, out: str = "") -> List[str]:
    spec = TARGETS[name]
    cmd = [hipcc(), "-O3", "-std=c++17", "-Wall", "-Wno-unused-function", f"-I{os.path.join(HERE, 'csrc')}"]
    if spec["kind"] == "ext":
        cmd += ["-fPIC", "-shared", f"-I{sysconfig.get_paths()['include']}"]
    if spec["hip"]:
        cmd += [f"--offload-arch={ARCH}", "-x", "hip", "-munsafe-fp-atomics"]
    else:
        # Host-only sources (HIP runtime API, no kernels): hipcc still runs a
        # device pass over them, which must target gfx950 like everything else.
        cmd += [f"--offload-arch={ARCH}"]
    cmd += [os.path.join(HERE, s) for s in spec["sources"]]
    cmd += ["-o", out or so_path(name), f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"]
    return cmd


def build(names=None, force: bool = False, verbose: bool = False) -> Dict[str, str]:
    """Compile the given targets (default: all). Returns name → output path.

    Safe to call from several processes at once (one rank per GPU): each
    target builds under an exclusive file lock into a temporary file that is
    renamed into place, so no process ever loads a half-written library.
    """
    out = {}
    for name in names or TARGETS:
        if not all(os.path.exists(os.path.join(HERE, s)) for s in TARGETS[name]["sources"]):
            continue
        target = so_path(name)
        if force or _stale(name):
            os.makedirs(os.path.dirname(target), exist_ok=True)
            with open(target + ".lock", "w") as lock:
                fcntl.flock(lock, fcntl.LOCK_EX)
                if force or _stale(name):  # another process may have built it meanwhile
                    tmp = f"{target}.tmp{os.getpid()}"
                    cmd = command(name, tmp)
                    if verbose:
                        print(" ".join(cmd), file=sys.stderr)
                    r = subprocess.run(cmd, capture_output=True, text=True)
                    if r.returncode != 0:
                        if os.path.exists(tmp):
                            os.unlink(tmp)
                        raise RuntimeError(f"building {name} failed:\n{r.stderr[-4000:]}")
                    os.replace(tmp, target)
        out[name] = target
    return out


if __name__ == "__main__":
    for k, v in build(force="--force" in sys.argv, verbose=True).items():
        print(k, v)
