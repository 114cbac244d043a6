"""Native code: MI355X telemetry probe (C++/HIP runtime) and workload kernels (HIP, gfx950).

Import the wrappers, not the raw modules::

    from headlamp_intel_gpu_plugin_amd.ops import probe, workload
"""
import importlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def load_native(name: str):
    """Import an in-tree extension, building it first if it is missing or stale.

    Raises ImportError with the build log when the extension cannot be
    built or loaded — there is deliberately no Python fallback for native ops.
    """
    from . import build as _build

    so = _build.so_path(name)
    if not os.path.exists(so) or _build._stale(name):
        _build.build([name])
    return importlib.import_module(f"{__name__}.{name}")
