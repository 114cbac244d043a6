"""Per-GPU MI355X telemetry series for the fake Prometheus.

Two sources fill the TSDB, mirroring the two exporters the plugin reads
(src/api/metrics.js ``SERIES``):

* ``amd-exporter`` — AMD Device Metrics Exporter style ``gpu_*`` gauges keyed
  by ``hostname`` + ``gpu_id``, with ``pod``/``namespace`` labels on GPUs a
  workload holds, ``xgmi_neighbor_N_tx_throughput`` per link and the
  native exporter's ``gpu_xgmi_link_hops`` per peer (with its ``neighbor``
  order, which places the per-neighbour throughput on a peer);
* ``node-exporter`` — ``node_hwmon_*`` (chip = PCI address, chip_name
  ``amdgpu``) and ``node_drm_*`` (card) series plus ``node_uname_info``.

Synthetic values are deterministic functions of time shaped by the
cluster's workload placement: a GPU held by a pod runs hot (GFX 80-99 %,
1.0-1.35 kW of the 1.4 kW board power, 120-260 GB of 288 GB HBM in use), a
free GPU idles. Multi-GPU pods drive traffic on the xGMI links between
their GPUs. :class:`LiveGpu` overrides one (node, gpu) with real samples
from the native probe (``ops.probe``) when a GPU is present.
"""
from __future__ import annotations

import hashlib
import math
from typing import Dict, Optional, Tuple

from ..sim.promql import TSDB, Series
from .cluster import GPUS_PER_NODE, HBM_BYTES, SyntheticCluster, gpu_node_name

MIB = 1024 * 1024
BOARD_POWER_W = 1400.0
IDLE_POWER_W = 185.0
XGMI_LINK_GBS = 153.0
JUNCTION_SLOWDOWN_C = 100.0  # amd-smi slowdown_hotspot_temperature on an MI355X


def _phase(*parts) -> float:
    h = hashlib.sha1("/".join(map(str, parts)).encode()).digest()
    return (h[0] * 256 + h[1]) / 65536.0 * 2 * math.pi


def pci_address(node_index: int, gpu: int) -> str:
    """hwmon-style chip id of GPU ``gpu`` (node-exporter replaces ':' / '.' with '_')."""
    bus = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5][gpu % 8]
    return f"0000:{bus:02x}:00_0"


class LiveGpu:
    """Real samples for one (node, gpu) pushed by the probe sampler."""

    def __init__(self) -> None:
        self.series: Dict[str, Series] = {}


def _ce(node_index: int, gpu: int) -> int:
    """Corrected-error count of a synthetic GPU (non-zero on one GPU in 37)."""
    return 3 if (node_index * 8 + gpu) % 37 == 5 else 0


def populate(db: TSDB, cluster: SyntheticCluster, source: str = "amd-exporter", interval: float = 15.0,
             live: Optional[Dict[Tuple[str, int], Dict[str, Series]]] = None) -> int:
    """Register telemetry series for every GPU in ``cluster``. Returns the series count.

    ``live`` maps (node, gpu) → {metric name → pushed Series}; those replace the
    synthetic functions for that GPU.
    """
    live = live or {}
    n0 = len(db)
    spec = cluster.spec
    for i in range(spec.gpu_nodes):
        node = gpu_node_name(i)
        instance = f"10.0.{i // 250}.{i % 250 + 10}"
        # Pod groups on this node (for xGMI traffic between their GPUs).
        groups: Dict[Tuple[str, str], list] = {}
        for g in range(spec.gpus_per_node):
            owner = cluster.gpu_owner.get((node, g))
            if owner:
                groups.setdefault(owner, []).append(g)
        if source == "node-exporter":
            db.add(Series({"__name__": "node_uname_info", "instance": f"{instance}:9100", "nodename": node,
                           "job": "node-exporter"}, fn=lambda t: 1.0, interval=interval))
            # The host CPU's hwmon chip: temperatures the plugin must not take for a GPU's.
            cpu = {"chip": "platform_coretemp_0", "instance": f"{instance}:9100"}
            db.add(Series(dict(cpu, __name__="node_hwmon_chip_names", chip_name="coretemp"), fn=lambda t: 1.0,
                          interval=interval))
            db.add(Series(dict(cpu, __name__="node_hwmon_temp_celsius", sensor="temp1"), fn=lambda t: 47.0,
                          interval=interval))
            db.add(Series(dict(cpu, __name__="node_hwmon_temp_crit_celsius", sensor="temp1"), fn=lambda t: 100.0,
                          interval=interval))
            db.add(Series(dict(cpu, __name__="node_hwmon_sensor_label", sensor="temp1", label="Package id 0"),
                          fn=lambda t: 1.0, interval=interval))
        for g in range(spec.gpus_per_node):
            owner = cluster.gpu_owner.get((node, g))
            busy = owner is not None
            ph = _phase(node, g)
            lv = live.get((node, g), {})

            def gfx(t, busy=busy, ph=ph):
                return 88.0 + 10.0 * math.sin(t / 47.0 + ph) if busy else 0.5 + 0.5 * math.sin(t / 90.0 + ph)

            def power(t, busy=busy, ph=ph):
                return (1180.0 + 160.0 * math.sin(t / 47.0 + ph)) if busy else IDLE_POWER_W + 8.0 * math.sin(t / 90.0 + ph)

            hbm_fill = 0.42 + 0.45 * ((ph / (2 * math.pi)) % 1.0)

            def vram_mib(t, busy=busy, fill=hbm_fill):
                return (HBM_BYTES * fill if busy else 512 * MIB) / MIB

            def umc(t, busy=busy, ph=ph):
                return 55.0 + 15.0 * math.sin(t / 31.0 + ph) if busy else 0.0

            def temp(t, busy=busy, ph=ph):
                return 38.0 + (power(t, busy, ph) / BOARD_POWER_W) * 42.0

            if source == "amd-exporter":
                base = {"hostname": node, "gpu_id": str(g), "instance": f"{instance}:5000", "job": "amd-metrics-exporter",
                        "card_model": "AMD Instinct MI355X", "serial_number": f"MI355X{i:03d}{g}"}
                own = {"pod": owner[1], "namespace": owner[0]} if owner else {}
                for name, fn, extra in (("gpu_power_usage", power, own), ("gpu_power_cap", lambda t: BOARD_POWER_W, {}),
                                        ("gpu_gfx_activity", gfx, {}),
                                        ("gpu_used_vram", vram_mib, {}),
                                        ("gpu_total_vram", lambda t: HBM_BYTES / MIB, {}),
                                        ("gpu_umc_activity", umc, {}), ("gpu_junction_temperature", temp, {}),
                                        ("gpu_junction_temperature_slowdown", lambda t: JUNCTION_SLOWDOWN_C, {}),
                                        # RAS counters: a healthy fleet reads 0; one GPU in 37
                                        # carries a few corrected HBM errors.
                                        ("gpu_ecc_correct_total", lambda t, c=float(_ce(i, g)): c, {}),
                                        ("gpu_ecc_uncorrect_total", lambda t: 0.0, {})):
                    labels = dict(base, __name__=name, **extra)
                    if name in lv:
                        s = lv[name]
                        s.labels.update(labels)
                        s._key = tuple(sorted(s.labels.items()))
                        db.add(s)
                    else:
                        db.add(Series(labels, fn=fn, interval=interval))
                # xGMI: neighbour k of GPU g is the k-th peer skipping g.
                peers = [p for p in range(spec.gpus_per_node) if p != g]
                mates = set(groups.get(owner, [])) if owner else set()
                for k, peer in enumerate(peers):
                    active = peer in mates
                    lph = _phase(node, g, peer)

                    def xgmi(t, active=active, lph=lph):
                        return (0.55 + 0.3 * math.sin(t / 23.0 + lph)) * XGMI_LINK_GBS * 1e9 if active else 0.0

                    db.add(Series(dict(base, __name__=f"xgmi_neighbor_{k}_tx_throughput"), fn=xgmi, interval=interval))
                    # Link hop count as the framework's amdgpu-exporter reports it
                    # (ops/csrc/probe_core.h, --sysfs-only): one hop to every peer on
                    # the mesh, and the link's place in the GPU's neighbour order (KFD
                    # io_link order), which pins xgmi_neighbor_<k> to its peer.
                    db.add(Series(dict(base, __name__="gpu_xgmi_link_hops", peer_gpu_id=str(peer), neighbor=str(k)),
                                  fn=lambda t: 1.0, interval=interval))
            else:
                chip = pci_address(i, g)
                inst = f"{instance}:9100"
                db.add(Series({"__name__": "node_hwmon_chip_names", "chip": chip, "chip_name": "amdgpu", "instance": inst},
                              fn=lambda t: 1.0, interval=interval))
                # An MI355X exposes hwmon power1_input only (no power1_average).
                db.add(Series({"__name__": "node_hwmon_power_input_watt", "chip": chip, "sensor": "power1",
                               "instance": inst}, fn=power, interval=interval))
                db.add(Series({"__name__": "node_hwmon_power_cap_watt", "chip": chip, "sensor": "power1",
                               "instance": inst}, fn=lambda t: BOARD_POWER_W, interval=interval))
                # amdgpu hwmon temperatures: temp2 "junction" (its crit is the throttle threshold) and
                # temp3 "mem"; an MI355X reports no edge temperature.
                for sensor, label, fn, crit in (("temp2", "junction", temp, JUNCTION_SLOWDOWN_C),
                                                ("temp3", "mem", lambda t, f=temp: f(t) - 6.0, 95.0)):
                    hw = {"chip": chip, "sensor": sensor, "instance": inst}
                    db.add(Series(dict(hw, __name__="node_hwmon_temp_celsius"), fn=fn, interval=interval))
                    db.add(Series(dict(hw, __name__="node_hwmon_temp_crit_celsius"), fn=lambda t, c=crit: c,
                                  interval=interval))
                    db.add(Series(dict(hw, __name__="node_hwmon_sensor_label", label=label), fn=lambda t: 1.0,
                                  interval=interval))
                card = f"card{g}"
                db.add(Series({"__name__": "node_drm_gpu_busy_percent", "card": card, "instance": inst},
                              fn=gfx, interval=interval))
                db.add(Series({"__name__": "node_drm_memory_vram_used_bytes", "card": card, "instance": inst},
                              fn=lambda t, f=vram_mib: f(t) * MIB, interval=interval))
                db.add(Series({"__name__": "node_drm_memory_vram_size_bytes", "card": card, "instance": inst},
                              fn=lambda t: float(HBM_BYTES), interval=interval))
    return len(db) - n0


def expected_gpu_count(cluster: SyntheticCluster) -> int:
    return cluster.spec.gpu_nodes * cluster.spec.gpus_per_node


__all__ = ["populate", "LiveGpu", "pci_address", "expected_gpu_count", "GPUS_PER_NODE"]
