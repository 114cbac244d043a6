"""The fake Prometheus' storage: labelled series and an in-memory TSDB.

Series are stored either as a deterministic function of time sampled on a
fixed scrape grid (synthetic telemetry) or as explicit pushed samples (live
GPU telemetry from the native probe). Staleness/lookback follow Prometheus'
5-minute default. Queried by :mod:`.promql`.
"""
from __future__ import annotations

import bisect
import json
import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple


LOOKBACK_S = 300.0
Labels = Dict[str, str]


# ---------------------------------------------------------------------------
# Storage
# ---------------------------------------------------------------------------

# Bumped on every sample push / series add: instant-query results cached by
# :func:`query` are valid only while it is unchanged.
_MUTATIONS = [0]

# What each mutation may have changed, as (mutation count, lo, hi): query
# results at evaluation times in [lo, hi]. A pushed sample at T changes what
# is seen at T and later only (samples are appended in time order); a sample
# dropped from the front of a capped series changes what its lookback window
# saw; a new series changes everything. Range-query memos (promql.query_range)
# drop just those steps, so a scrape landing between two refreshes does not
# make the fake re-evaluate a whole window in Python.
_CHANGES: List[Tuple[int, float, float]] = []
_CHANGES_MAX = 200_000


def _changed(lo: float, hi: float) -> None:
    _MUTATIONS[0] += 1
    _CHANGES.append((_MUTATIONS[0], lo, hi))
    if len(_CHANGES) > _CHANGES_MAX:
        del _CHANGES[: _CHANGES_MAX // 2]


def changes_since(stamp: int):
    """The (lo, hi) ranges changed after mutation ``stamp``, or None when the log no longer reaches back that far."""
    if stamp == _MUTATIONS[0]:
        return []
    if not _CHANGES or _CHANGES[0][0] > stamp + 1:
        return None
    i = bisect.bisect_right(_CHANGES, (stamp, math.inf, math.inf))
    return [(lo, hi) for _, lo, hi in _CHANGES[i:]]


class Series:
    """One time series: labels + samples.

    Either ``fn(t)`` sampled every ``interval`` seconds (aligned to the grid),
    or explicit samples appended with :meth:`push` (kept sorted, bounded).
    """

    __slots__ = ("labels", "fn", "interval", "ts", "vs", "cap", "_key", "_json", "_memo", "seq")

    def __init__(self, labels: Labels, fn: Optional[Callable[[float], float]] = None,
                 interval: float = 15.0, cap: int = 4096):
        self.labels = dict(labels)
        self.fn = fn
        self.interval = float(interval)
        self.ts: List[float] = []
        self.vs: List[float] = []
        self.cap = cap
        self._key = tuple(sorted(self.labels.items()))
        self.seq = 0  # insertion order in its TSDB
        self._json = None
        self._memo: Dict[float, float] = {}  # fn value per sample time (fn series are deterministic)

    def metric_json(self) -> str:
        """JSON of the label set (cached — series labels never change once stored)."""
        if self._json is None:
            self._json = json.dumps(self.labels, separators=(",", ":"))
        return self._json

    def push(self, t: float, v: float) -> None:
        if self.ts and t <= self.ts[-1]:
            if t == self.ts[-1]:
                _changed(t, math.inf)
                self.vs[-1] = v
            return
        _changed(t, math.inf)
        self.ts.append(t)
        self.vs.append(v)
        if len(self.ts) > self.cap:
            drop = len(self.ts) - self.cap
            _changed(-math.inf, self.ts[drop - 1] + LOOKBACK_S)
            del self.ts[:drop]
            del self.vs[:drop]

    def _fn_at(self, ts: float) -> float:
        v = self._memo.get(ts)
        if v is None:
            if len(self._memo) >= 4096:
                self._memo.clear()
            v = self._memo[ts] = self.fn(ts)
        return v

    def samples(self, start: float, end: float) -> List[Tuple[float, float]]:
        """Samples with start < t <= end."""
        if self.fn is not None:
            iv = self.interval
            k0 = math.floor(start / iv) + 1
            k1 = math.floor(end / iv)
            return [(k * iv, self._fn_at(k * iv)) for k in range(k0, k1 + 1)]
        lo = bisect.bisect_right(self.ts, start)
        hi = bisect.bisect_right(self.ts, end)
        return list(zip(self.ts[lo:hi], self.vs[lo:hi]))

    def at(self, t: float) -> Optional[Tuple[float, float]]:
        """Latest sample within the lookback window ending at ``t``."""
        if self.fn is not None:
            k = math.floor(t / self.interval) * self.interval
            return (k, self._fn_at(k))
        i = bisect.bisect_right(self.ts, t) - 1
        if i < 0 or t - self.ts[i] > LOOKBACK_S:
            return None
        return (self.ts[i], self.vs[i])


class TSDB:
    """Series indexed by metric name."""

    def __init__(self) -> None:
        self.by_name: Dict[str, List[Series]] = {}
        self._index: Dict[tuple, Series] = {}
        self._select_cache: Dict[tuple, List[Series]] = {}
        self._by_labels_id: Dict[int, Series] = {}
        # `by (...)` projections of stored label sets: (id(labels), by) → (key, projected, labels, json)
        self._proj_cache: Dict[tuple, tuple] = {}
        self._proj_json: Dict[int, tuple] = {}
        self._fn_intervals: set = set()
        self._query_cache: Dict[str, tuple] = {}
        self._range_cache: Dict[str, tuple] = {}  # query → (mutation stamp, {t → rows})
        # Inverted index (label, value) → series, as a real TSDB's postings:
        # a `hostname=~"a|b|…"` page scope or `hostname="x"` detail query
        # reads the matching series only, not every series of its names.
        self._by_label: Dict[tuple, List[Series]] = {}
        self._name_rank: Dict[str, int] = {}
        # Aggregations over a plain selector: the function-backed series' part
        # per (query part, sample-grid bucket); pushed series are added each time.
        self._agg_cache: Dict[tuple, dict] = {}

    def label_json(self, labels: Labels) -> str:
        """JSON for a label set; cached when it is a stored series' own dict
        or a cached ``by`` projection of one."""
        s = self._by_labels_id.get(id(labels))
        if s is not None and s.labels is labels:
            return s.metric_json()
        p = self._proj_json.get(id(labels))
        if p is not None and p[0] is labels:
            return p[1]
        return json.dumps(labels, separators=(",", ":"))

    def project(self, labels: Labels, by: tuple) -> tuple:
        """(group key, projected labels) of ``labels`` onto ``by``, cached per
        stored label set so a repeated aggregation query does no dict work."""
        ck = (id(labels), by)
        hit = self._proj_cache.get(ck)
        if hit is not None and hit[2] is labels:
            return hit[0], hit[1]
        gl = {k: labels[k] for k in by if k in labels}
        key = tuple(sorted(gl.items()))
        if self._by_labels_id.get(id(labels)) is not None:
            self._proj_cache[ck] = (key, gl, labels)
            self._proj_json[id(gl)] = (gl, json.dumps(gl, separators=(",", ":")))
        return key, gl

    def add(self, series: Series) -> Series:
        key = series._key
        if key in self._index:
            return self._index[key]
        self._index[key] = series
        _changed(-math.inf, math.inf)
        series.seq = len(self._index)
        if series.fn is not None:
            self._fn_intervals.add(series.interval)
        name = series.labels.get("__name__", "")
        if name not in self.by_name:
            self._name_rank[name] = len(self._name_rank)
        self.by_name.setdefault(name, []).append(series)
        for kv in series.labels.items():
            self._by_label.setdefault(kv, []).append(series)
        self._by_labels_id[id(series.labels)] = series
        self._select_cache.clear()
        self._agg_cache.clear()
        return series

    def get_or_create(self, labels: Labels) -> Series:
        key = tuple(sorted(labels.items()))
        s = self._index.get(key)
        if s is None:
            s = self.add(Series(labels))
        return s

    def select(self, matchers: Sequence["Matcher"]) -> List[Series]:
        """Series matching every matcher. The series set only grows via
        :meth:`add`, so results are cached per matcher signature."""
        sig = tuple((m.label, m.op, m.value) for m in matchers)
        hit = self._select_cache.get(sig)
        if hit is not None:
            return hit
        # The most selective indexable matcher (= or a =~ of literal
        # alternatives) picks the candidates; every matcher then filters.
        best = None
        for m in matchers:
            vals = m.literals()
            if vals is None:
                continue
            lists = [self._by_label.get((m.label, v), []) for v in vals]
            n = sum(len(x) for x in lists)
            if best is None or n < best[0]:
                best = (n, lists)
        if best is not None:
            cands = best[1][0] if len(best[1]) == 1 else [x for lst in best[1] for x in lst]
            out = [x for x in cands if all(m.matches(x.labels.get(m.label, "")) for m in matchers)]
            # the order a scan by name would give: names in insertion order, then series
            rank = self._name_rank
            out.sort(key=lambda x: (rank.get(x.labels.get("__name__", ""), 0), x.seq))
            self._select_cache[sig] = out
            return out
        names = [m for m in matchers if m.label == "__name__" and m.op == "="]
        if names:
            cands = self.by_name.get(names[0].value, [])
        else:
            name_re = [m for m in matchers if m.label == "__name__" and m.op == "=~"]
            if name_re:
                cands = [s for n, lst in self.by_name.items() if name_re[0].matches(n) for s in lst]
            else:
                cands = [s for lst in self.by_name.values() for s in lst]
        out = [s for s in cands if all(m.matches(s.labels.get(m.label, "")) for m in matchers)]
        self._select_cache[sig] = out
        return out

    def __len__(self) -> int:
        return len(self._index)


# ---------------------------------------------------------------------------
