"""Latency statistics (same interpolation as bench/driver.js)."""
from __future__ import annotations

from typing import Dict, Sequence


def quantile(xs: Sequence[float], q: float) -> float:
    s = sorted(xs)
    if not s:
        return float("nan")
    idx = (len(s) - 1) * q
    lo, hi = int(idx), min(int(idx) + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (idx - lo)


def summarize(xs: Sequence[float]) -> Dict[str, float]:
    return {
        "n": len(xs),
        "p50": quantile(xs, 0.5),
        "p95": quantile(xs, 0.95),
        "min": min(xs) if xs else float("nan"),
        "max": max(xs) if xs else float("nan"),
        "mean": sum(xs) / len(xs) if xs else float("nan"),
    }
