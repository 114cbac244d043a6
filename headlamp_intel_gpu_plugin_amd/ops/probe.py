"""MI355X telemetry probe (native: ops/csrc/amdgpu_probe.cpp).

Thin typed wrapper over ``_amdgpu_probe``. ``available()`` is False on a host
without a HIP device (this container); on a GPU host the native module must
load — a missing or broken extension raises instead of silently degrading.
"""
from __future__ import annotations

import socket
from typing import Dict, List, Optional, Tuple

from . import load_native

_mod = None

#: sample() keys → AMD-exporter metric names the plugin reads
EXPORTER_FIELDS = {
    "power_w": "gpu_power_usage",
    "gfx_busy_pct": "gpu_gfx_activity",
    "mem_busy_pct": "gpu_umc_activity",
    "temp_junction_c": "gpu_junction_temperature",
}


def native():
    global _mod
    if _mod is None:
        _mod = load_native("_amdgpu_probe")
    return _mod


def available() -> bool:
    try:
        return native().device_count() > 0
    except (ImportError, RuntimeError, OSError):
        return False


def device_count() -> int:
    return native().device_count()


def device_info(i: int) -> Dict:
    return native().device_info(i)


def sample(i: int) -> Dict[str, Optional[float]]:
    return native().sample(i)


def link(a: int, b: int) -> Tuple[str, int, int]:
    """(type, hops, can_access_peer) — type is XGMI / PCIE / OTHER / SELF / UNKNOWN."""
    return native().link(a, b)


def topology() -> Dict[str, Dict]:
    """All-pairs link matrix in the shape ``src/api/topology.js`` accepts (``"i-j" → {type, hops}``)."""
    n = device_count()
    out = {}
    for a in range(n):
        for b in range(n):
            if a != b:
                t, hops, _ = link(a, b)
                out[f"{a}-{b}"] = {"type": t, "hops": hops}
    return out


def render_metrics(hostname: Optional[str] = None) -> str:
    """Exporter-format text exposition for every local device (rendered natively)."""
    return native().render_metrics(hostname or socket.gethostname())


def parse_exposition(text: str) -> List[Tuple[str, Dict[str, str], float]]:
    """Parse Prometheus text exposition (the subset the probe emits)."""
    out = []
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        head, _, val = line.rpartition(" ")
        name, _, rest = head.partition("{")
        labels: Dict[str, str] = {}
        body = rest[:-1] if rest.endswith("}") else rest
        i = 0
        while i < len(body):
            eq = body.index("=", i)
            key = body[i:eq].strip(", ")
            j = eq + 2  # skip ="
            buf = []
            while body[j] != '"':
                if body[j] == "\\":
                    j += 1
                    buf.append({"n": "\n"}.get(body[j], body[j]))
                else:
                    buf.append(body[j])
                j += 1
            labels[key] = "".join(buf)
            i = j + 1
        out.append((name, labels, float(val)))
    return out


def read_ras(ras_dir: str) -> Dict[str, Optional[float]]:
    """Summed RAS counters of an amdgpu ``ras/`` sysfs directory: ``ce``/``ue``/``de``
    (corrected / uncorrected / deferred), ``retired_pages`` and the number of IP
    ``blocks`` that reported. Pure file parsing: works without a GPU."""
    return native().read_ras(ras_dir)
