"""A PromQL subset evaluator over an in-memory TSDB.

Enough of the Prometheus HTTP API (``/api/v1/query``, ``/api/v1/query_range``)
to serve every query the plugin and the reference-schedule replay issue:

* vector selectors with ``= != =~ !~`` matchers, including ``__name__``;
* range selectors ``x[5m]`` with ``rate irate increase avg_over_time
  max_over_time min_over_time sum_over_time count_over_time last_over_time``;
* aggregations ``sum avg max min count`` with ``by (...)`` / ``without (...)``
  in either position;
* binary arithmetic/comparison between scalars and vectors, with
  ``on(...)`` / ``ignoring(...)`` and ``group_left(...)`` / ``group_right(...)``;
* the set operators ``or and unless`` between vectors (matching on every
  label but ``__name__``, or on ``on(...)`` / ``ignoring(...)``);
* ``label_replace(v, "dst", "replacement", "src", "regex")``;
* number literals (the reference's discovery probe is ``query=1``).

Series are stored either as a deterministic function of time sampled on a
fixed scrape grid (synthetic telemetry) or as explicit pushed samples (live
GPU telemetry from the native probe). Staleness/lookback follow Prometheus'
5-minute default.
"""
from __future__ import annotations

import bisect
import json
import math
import re
from typing import Callable, Dict, List, Optional, Sequence, Tuple

LOOKBACK_S = 300.0
Labels = Dict[str, str]


# ---------------------------------------------------------------------------
# Storage
# ---------------------------------------------------------------------------

# Bumped on every sample push / series add: instant-query results cached by
# :func:`query` are valid only while it is unchanged.
_MUTATIONS = [0]


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
        _MUTATIONS[0] += 1
        if self.ts and t <= self.ts[-1]:
            if t == self.ts[-1]:
                self.vs[-1] = v
            return
        self.ts.append(t)
        self.vs.append(v)
        if len(self.ts) > self.cap:
            drop = len(self.ts) - self.cap
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
        _MUTATIONS[0] += 1
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
# Lexer / parser
# ---------------------------------------------------------------------------

class PromQLError(ValueError):
    pass


_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?)
  | (?P<dur>\[\s*\d+[smhdw]\s*\])
  | (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
  | (?P<op>=~|!~|!=|==|>=|<=|[-+*/%^(){},=<>])
  | (?P<ident>[a-zA-Z_:][a-zA-Z0-9_:]*)
""", re.X)

_DUR = {"s": 1, "m": 60, "h": 3600, "d": 86400, "w": 604800}
AGGREGATIONS = {"sum", "avg", "max", "min", "count"}
RANK_AGGREGATIONS = {"topk", "bottomk"}
RANGE_FUNCS = {"rate", "irate", "increase", "avg_over_time", "max_over_time", "min_over_time",
               "sum_over_time", "count_over_time", "last_over_time"}
BIN_PREC = {"+": 1, "-": 1, "*": 2, "/": 2, "%": 2, "==": 0, "!=": 0, ">": 0, "<": 0, ">=": 0, "<=": 0,
            "and": -1, "unless": -1, "or": -2}
SET_OPS = {"and", "unless", "or"}
MIN_PREC = min(BIN_PREC.values())


def _tokenize(q: str) -> List[Tuple[str, str]]:
    pos = 0
    out = []
    while pos < len(q):
        m = _TOKEN_RE.match(q, pos)
        if not m:
            raise PromQLError(f"unexpected character {q[pos]!r} at {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        out.append((kind, m.group(kind)))
    out.append(("eof", ""))
    return out


class Matcher:
    __slots__ = ("label", "op", "value", "_re")

    def __init__(self, label: str, op: str, value: str):
        self.label, self.op, self.value = label, op, value
        self._re = re.compile("^(?:" + value + ")$") if op in ("=~", "!~") else None

    def literals(self) -> Optional[List[str]]:
        """The exact values this matcher accepts, when it is `=` / a `=~` of
        literal alternatives and none is empty (an empty value also matches
        series without the label); else None."""
        if self.op == "=":
            return [self.value] if self.value else None
        if self.op != "=~":
            return None
        out = []
        for part in re.split(r"(?<!\\)\|", self.value):
            if not part or re.search(r"(?<!\\)[.^$*+?()\[\]{}|]", part):
                return None
            out.append(re.sub(r"\\(.)", r"\1", part))
        return out

    def matches(self, v: str) -> bool:
        if self.op == "=":
            return v == self.value
        if self.op == "!=":
            return v != self.value
        ok = bool(self._re.match(v))
        return ok if self.op == "=~" else not ok


# AST nodes are tuples: ("num", v) ("sel", matchers, range_s|None) ("func", name, arg)
# ("agg", op, by|None, without|None, expr) ("bin", op, lhs, rhs, matching)

class _Parser:
    def __init__(self, q: str):
        self.toks = _tokenize(q)
        self.i = 0

    def peek(self, k: int = 0):
        return self.toks[self.i + k]

    def take(self, kind: Optional[str] = None, val: Optional[str] = None):
        t = self.toks[self.i]
        if (kind and t[0] != kind) or (val is not None and t[1] != val):
            raise PromQLError(f"expected {val or kind}, got {t[1]!r}")
        self.i += 1
        return t

    def parse(self):
        e = self.expr(MIN_PREC)
        self.take("eof")
        return e

    def expr(self, min_prec: int):
        lhs = self.unary()
        while True:
            k, v = self.peek()
            is_op = (k == "op" and v in BIN_PREC) or (k == "ident" and v in SET_OPS)
            if not is_op or BIN_PREC[v] < min_prec:
                return lhs
            self.i += 1
            matching = self.vector_matching()
            rhs = self.expr(BIN_PREC[v] + 1)
            lhs = ("bin", v, lhs, rhs, matching)

    def vector_matching(self):
        k, v = self.peek()
        if k == "ident" and v in ("on", "ignoring"):
            self.i += 1
            labels = self.label_list()
            group = None
            k2, v2 = self.peek()
            if k2 == "ident" and v2 in ("group_left", "group_right"):
                self.i += 1
                extra = self.label_list() if self.peek()[1] == "(" else []
                group = (v2, extra)
            return (v, labels, group)
        return None

    def label_list(self) -> List[str]:
        self.take("op", "(")
        out = []
        while self.peek()[1] != ")":
            out.append(self.take("ident")[1])
            if self.peek()[1] == ",":
                self.i += 1
        self.take("op", ")")
        return out

    def unary(self):
        k, v = self.peek()
        if k == "op" and v == "-":
            self.i += 1
            return ("bin", "*", ("num", -1.0), self.unary(), None)
        return self.primary()

    def primary(self):
        k, v = self.peek()
        if k == "num":
            self.i += 1
            return ("num", float(v))
        if k == "op" and v == "(":
            self.i += 1
            e = self.expr(MIN_PREC)
            self.take("op", ")")
            return e
        if k == "op" and v == "{":
            return self.selector(None)
        if k == "ident":
            if v in AGGREGATIONS and self.peek(1)[1] in ("(", "by", "without"):
                return self.aggregation()
            if v in RANK_AGGREGATIONS and self.peek(1)[1] in ("(", "by", "without"):
                return self.rank_aggregation()
            if v == "label_replace" and self.peek(1)[1] == "(":
                self.i += 2
                arg = self.expr(MIN_PREC)
                strs = []
                for _ in range(4):
                    self.take("op", ",")
                    raw = self.take("str")[1]
                    strs.append(bytes(raw[1:-1], "utf-8").decode("unicode_escape"))
                self.take("op", ")")
                return ("label_replace", arg, *strs)
            if v in RANGE_FUNCS and self.peek(1)[1] == "(":
                self.i += 2
                arg = self.expr(MIN_PREC)
                self.take("op", ")")
                if arg[0] != "sel" or arg[2] is None:
                    raise PromQLError(f"{v}() expects a range vector")
                return ("func", v, arg)
            self.i += 1
            return self.selector(v)
        raise PromQLError(f"unexpected token {v!r}")

    def aggregation(self):
        op = self.take("ident")[1]
        by = without = None
        if self.peek()[1] in ("by", "without"):
            kw = self.take("ident")[1]
            lst = self.label_list()
            by, without = (lst, None) if kw == "by" else (None, lst)
        self.take("op", "(")
        e = self.expr(MIN_PREC)
        self.take("op", ")")
        if self.peek()[1] in ("by", "without"):
            kw = self.take("ident")[1]
            lst = self.label_list()
            by, without = (lst, None) if kw == "by" else (None, lst)
        return ("agg", op, by, without, e)

    def rank_aggregation(self):
        """`topk(k, expr)` / `bottomk(k, expr)`, optionally `by (…)` / `without (…)`."""
        op = self.take("ident")[1]
        by = without = None
        if self.peek()[1] in ("by", "without"):
            kw = self.take("ident")[1]
            lst = self.label_list()
            by, without = (lst, None) if kw == "by" else (None, lst)
        self.take("op", "(")
        k = self.expr(MIN_PREC)
        self.take("op", ",")
        e = self.expr(MIN_PREC)
        self.take("op", ")")
        if self.peek()[1] in ("by", "without"):
            kw = self.take("ident")[1]
            lst = self.label_list()
            by, without = (lst, None) if kw == "by" else (None, lst)
        return ("rank", op, k, by, without, e)

    def selector(self, name: Optional[str]):
        matchers = []
        if name:
            matchers.append(Matcher("__name__", "=", name))
        if self.peek()[1] == "{":
            self.i += 1
            while self.peek()[1] != "}":
                label = self.take("ident")[1]
                op = self.take("op")[1]
                if op not in ("=", "!=", "=~", "!~"):
                    raise PromQLError(f"bad matcher op {op}")
                raw = self.take("str")[1]
                matchers.append(Matcher(label, op, bytes(raw[1:-1], "utf-8").decode("unicode_escape")))
                if self.peek()[1] == ",":
                    self.i += 1
            self.take("op", "}")
        if not matchers:
            raise PromQLError("empty selector")
        rng = None
        if self.peek()[0] == "dur":
            d = self.take("dur")[1].strip("[] ")
            rng = float(d[:-1]) * _DUR[d[-1]]
        return ("sel", matchers, rng)


def parse(q: str):
    return _Parser(q).parse()


# ---------------------------------------------------------------------------
# Evaluation
# ---------------------------------------------------------------------------

def _drop_name(labels: Labels) -> Labels:
    return {k: v for k, v in labels.items() if k != "__name__"}


def _key(labels: Labels, on: Optional[List[str]] = None, ignoring: Optional[List[str]] = None) -> tuple:
    if on is not None:
        return tuple((k, labels.get(k, "")) for k in sorted(on))
    ign = set(ignoring or []) | {"__name__"}
    return tuple(sorted((k, v) for k, v in labels.items() if k not in ign))


def _range_fn(name: str, samples: List[Tuple[float, float]], window: float) -> Optional[float]:
    if name == "count_over_time":
        return float(len(samples)) if samples else None
    if not samples:
        return None
    vs = [v for _, v in samples]
    if name == "avg_over_time":
        return sum(vs) / len(vs)
    if name == "max_over_time":
        return max(vs)
    if name == "min_over_time":
        return min(vs)
    if name == "sum_over_time":
        return sum(vs)
    if name == "last_over_time":
        return vs[-1]
    if len(samples) < 2:
        return None
    if name == "irate":
        (t0, v0), (t1, v1) = samples[-2], samples[-1]
        d = v1 - v0 if v1 >= v0 else v1
        return d / (t1 - t0) if t1 > t0 else None
    # rate / increase with counter-reset handling and extrapolation to the window
    inc = 0.0
    for (_, a), (_, b) in zip(samples, samples[1:]):
        inc += b - a if b >= a else b
    span = samples[-1][0] - samples[0][0]
    if span <= 0:
        return None
    per_s = inc / span
    return per_s if name == "rate" else per_s * window


def _apply(op: str, a: float, b: float) -> Optional[float]:
    if op == "+":
        return a + b
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if op == "/":
        return a / b if b != 0 else (math.nan if a == 0 else math.copysign(math.inf, a))
    if op == "%":
        return math.fmod(a, b) if b != 0 else math.nan
    cmp = {"==": a == b, "!=": a != b, ">": a > b, "<": a < b, ">=": a >= b, "<=": a <= b}[op]
    return a if cmp else None


class Evaluator:
    def __init__(self, db: TSDB):
        self.db = db

    def instant(self, node, t: float):
        """Returns ("scalar", v) or ("vector", [(labels, v), ...])."""
        kind = node[0]
        if kind == "num":
            return ("scalar", node[1])
        if kind == "sel":
            if node[2] is not None:
                raise PromQLError("range vector not allowed here")
            out = []
            for s in self.db.select(node[1]):
                smp = s.at(t)
                if smp is not None:
                    out.append((s.labels, smp[1]))
            return ("vector", out)
        if kind == "func":
            _, name, sel = node
            out = []
            for s in self.db.select(sel[1]):
                v = _range_fn(name, s.samples(t - sel[2], t), sel[2])
                if v is not None:
                    out.append((_drop_name(s.labels), v))
            return ("vector", out)
        if kind == "agg":
            _, op, by, without, e = node
            if e[0] == "sel" and e[2] is None and len(self.db._fn_intervals) <= 1:
                return self._agg_selector(node, t)
            typ, vec = self.instant(e, t)
            if typ != "vector":
                raise PromQLError("aggregation over scalar")
            groups: Dict[tuple, List] = {}
            glabels: Dict[tuple, Labels] = {}
            byt = tuple(by) if by is not None else None
            for labels, v in vec:
                if byt is not None:
                    k, gl = self.db.project(labels, byt)
                else:
                    gl = ({k: x for k, x in _drop_name(labels).items() if k not in without}
                          if without is not None else {})
                    k = tuple(sorted(gl.items()))
                groups.setdefault(k, []).append(v)
                glabels[k] = gl
            res = []
            for k, vs in groups.items():
                if op == "sum":
                    r = sum(vs)
                elif op == "avg":
                    r = sum(vs) / len(vs)
                elif op == "max":
                    r = max(vs)
                elif op == "min":
                    r = min(vs)
                else:
                    r = float(len(vs))
                res.append((glabels[k], r))
            return ("vector", res)
        if kind == "rank":
            return self._rank(node, t)
        if kind == "bin":
            return self._binary(node, t)
        if kind == "label_replace":
            return self._label_replace(node, t)
        raise PromQLError(f"cannot evaluate {kind}")

    def _rank(self, node, t):
        """topk / bottomk: the k largest (smallest) samples of each group, labels kept; NaN ranks last."""
        _, op, k_node, by, without, e = node
        kt, k = self.instant(k_node, t)
        if kt != "scalar":
            raise PromQLError(f"{op}: k must be a scalar")
        typ, vec = self.instant(e, t)
        if typ != "vector":
            raise PromQLError(f"{op} over a scalar")
        n = int(k)
        groups: Dict[tuple, List] = {}
        byt = tuple(by) if by is not None else None
        for labels, v in vec:
            key = self._group(labels, byt, without)[0] if (byt is not None or without is not None) else ()
            groups.setdefault(key, []).append((labels, v))
        out = []
        sign = -1.0 if op == "topk" else 1.0
        for members in groups.values():
            members.sort(key=lambda lv: (math.isnan(lv[1]), sign * lv[1] if not math.isnan(lv[1]) else 0.0))
            out.extend(members[:max(0, n)])
        return ("vector", out)

    def _group(self, labels, byt, without):
        if byt is not None:
            return self.db.project(labels, byt)
        gl = ({k: x for k, x in _drop_name(labels).items() if k not in without} if without is not None else {})
        return tuple(sorted(gl.items())), gl

    def _agg_selector(self, node, t):
        """`op by (…) (selector)`: the function-backed series change only on
        their sample grid, so their per-group partial (sum, count, max, min)
        is kept per grid bucket; pushed (live) series are folded in on every
        evaluation. Same result as aggregating the selected vector."""
        _, op, by, without, e = node
        byt = tuple(by) if by is not None else None
        wt = tuple(without) if without is not None else None
        db = self.db
        iv = next(iter(db._fn_intervals)) if db._fn_intervals else 1.0
        sig = tuple((m.label, m.op, m.value) for m in e[1])
        key = (sig, byt, wt, math.floor(t / iv))
        hit = db._agg_cache.get(key)
        if hit is None:
            parts: Dict[tuple, list] = {}
            pushed = []
            counting = op == "count"  # a function-backed series always has a sample: no value needed
            for s in db.select(e[1]):
                if s.fn is None:
                    pushed.append(s)
                    continue
                v = 1.0 if counting else s.at(t)[1]
                k, gl = self._group(s.labels, byt, wt)
                a = parts.get(k)
                if a is None:
                    parts[k] = [gl, v, 1, v, v]
                else:
                    a[1] += v
                    a[2] += 1
                    if v > a[3]:
                        a[3] = v
                    if v < a[4]:
                        a[4] = v
            if len(db._agg_cache) > 512:
                db._agg_cache.clear()
            hit = db._agg_cache[key] = (parts, pushed)
        parts, pushed = hit
        groups = parts
        if pushed:
            groups = {k: list(a) for k, a in parts.items()}
            for s in pushed:
                smp = s.at(t)
                if smp is None:
                    continue
                v = smp[1]
                k, gl = self._group(s.labels, byt, wt)
                a = groups.get(k)
                if a is None:
                    groups[k] = [gl, v, 1, v, v]
                else:
                    a[1] += v
                    a[2] += 1
                    if v > a[3]:
                        a[3] = v
                    if v < a[4]:
                        a[4] = v
        res = []
        for gl, total, n, hi, lo in groups.values():
            r = {"sum": total, "avg": total / n, "max": hi, "min": lo}.get(op, float(n))
            res.append((gl, r))
        return ("vector", res)

    def _label_replace(self, node, t):
        _, arg, dst, repl, src, regex = node
        typ, vec = self.instant(arg, t)
        if typ != "vector":
            raise PromQLError("label_replace expects a vector")
        try:
            rx = re.compile("^(?:" + regex + ")$")
        except re.error as e:
            raise PromQLError(f"bad regex {regex!r}: {e}") from None
        # Prometheus' $1 / ${1} / ${name} → Python's \g<...>
        template = re.sub(r"\$\{(\w+)\}|\$(\w+)", lambda m: "\\g<" + (m.group(1) or m.group(2)) + ">", repl)
        out = []
        for labels, v in vec:
            m = rx.match(labels.get(src, ""))
            if not m:
                out.append((labels, v))
                continue
            value = m.expand(template)
            nl = dict(labels)
            if value:
                nl[dst] = value
            else:
                nl.pop(dst, None)
            out.append((nl, v))
        return ("vector", out)

    def _set_op(self, op, lv, rv, matching):
        on = ignoring = None
        if matching:
            mode, labels, _ = matching
            on, ignoring = (labels, None) if mode == "on" else (None, labels)
        rkeys = {_key(l, on, ignoring) for l, _ in rv}
        if op == "and":
            return ("vector", [(l, v) for l, v in lv if _key(l, on, ignoring) in rkeys])
        if op == "unless":
            return ("vector", [(l, v) for l, v in lv if _key(l, on, ignoring) not in rkeys])
        lkeys = {_key(l, on, ignoring) for l, _ in lv}
        return ("vector", list(lv) + [(l, v) for l, v in rv if _key(l, on, ignoring) not in lkeys])

    def _binary(self, node, t):
        _, op, lhs, rhs, matching = node
        if op == "and":
            # `x and <empty>` is empty whatever x is: answered without evaluating x.
            # Prometheus evaluates both sides, on its own cores and in parallel
            # with other queries; this server's one event loop would instead
            # hold every other request behind a cluster-wide evaluation (the
            # client's size-guarded queries, metrics.js sizeGuard).
            rt, rv = self.instant(rhs, t)
            if rt == "vector" and not rv:
                return ("vector", [])
            lt, lv = self.instant(lhs, t)
            if lt != "vector" or rt != "vector":
                raise PromQLError(f"set operator {op} needs vectors on both sides")
            return self._set_op(op, lv, rv, matching)
        lt, lv = self.instant(lhs, t)
        rt, rv = self.instant(rhs, t)
        if op in SET_OPS:
            if lt != "vector" or rt != "vector":
                raise PromQLError(f"set operator {op} needs vectors on both sides")
            return self._set_op(op, lv, rv, matching)
        is_cmp = op in ("==", "!=", ">", "<", ">=", "<=")
        if lt == "scalar" and rt == "scalar":
            r = _apply(op, lv, rv)
            return ("scalar", r if r is not None else 0.0)
        if lt == "scalar" or rt == "scalar":
            out = []
            vec, sc, vec_left = (rv, lv, False) if lt == "scalar" else (lv, rv, True)
            for labels, v in vec:
                r = _apply(op, v, sc) if vec_left else _apply(op, sc, v)
                if r is None:
                    continue
                out.append((labels if is_cmp else _drop_name(labels), v if is_cmp else r))
            return ("vector", out)
        on = ignoring = None
        group = None
        if matching:
            mode, labels, group = matching
            if mode == "on":
                on = labels
            else:
                ignoring = labels
        # "one" side is indexed by key; group_left lets the left side be many.
        if group and group[0] == "group_right":
            many, one, many_is_left = rv, lv, False
        else:
            many, one, many_is_left = lv, rv, True
        index: Dict[tuple, Tuple[Labels, float]] = {}
        for labels, v in one:
            k = _key(labels, on, ignoring)
            if k in index and not group:
                raise PromQLError("many-to-many matching not allowed")
            index[k] = (labels, v)
        out = []
        seen = set()
        for labels, v in many:
            k = _key(labels, on, ignoring)
            if k not in index:
                continue
            if not group:
                if k in seen:
                    raise PromQLError("multiple matches on the left side; use group_left")
                seen.add(k)
            olabels, ov = index[k]
            a, b = (v, ov) if many_is_left else (ov, v)
            r = _apply(op, a, b)
            if r is None:
                continue
            if group:
                res_labels = _drop_name(labels) if not is_cmp else dict(labels)
                for extra in group[1]:
                    if extra in olabels:
                        res_labels[extra] = olabels[extra]
            elif on is not None:
                res_labels = {k2: labels[k2] for k2 in on if k2 in labels} if not is_cmp else dict(labels)
            else:
                res_labels = _drop_name(labels) if not is_cmp else dict(labels)
            out.append((res_labels, a if is_cmp else r))
        return ("vector", out)


def _fmt(v: float) -> str:
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    r = repr(float(v))
    return r[:-2] if r.endswith(".0") else r


class RawJSON(str):
    """A pre-encoded JSON response body (served as-is by the fake apiserver)."""


def query(db: TSDB, q: str, t: float):
    """Prometheus ``/api/v1/query`` response body (dict on error/scalar, RawJSON for vectors).

    Function-backed series only change at their sample interval and pushed
    series only on push, so a vector result is reused for repeated queries
    within one interval bucket while nothing was pushed — the evaluation
    cost of a Python TSDB would otherwise dominate the fake's latency, where
    a real Prometheus answers such a selector in well under a millisecond.
    """
    cacheable = len(db._fn_intervals) <= 1
    if cacheable:
        iv = next(iter(db._fn_intervals)) if db._fn_intervals else 1.0
        stamp = (math.floor(t / iv), _MUTATIONS[0])
        hit = db._query_cache.get(q)
        if hit is not None and hit[0] == stamp:
            return _vector_body(hit[1], t)
    try:
        typ, val = Evaluator(db).instant(parse(q), t)
    except PromQLError as e:
        return {"status": "error", "errorType": "bad_data", "error": str(e)}
    if typ == "scalar":
        return {"status": "success", "data": {"resultType": "scalar", "result": [t, _fmt(val)]}}
    rows = [(db.label_json(l), _fmt(v)) for l, v in val]
    if cacheable:
        db._query_cache[q] = (stamp, rows)
    return _vector_body(rows, t)


def _vector_body(rows, t: float) -> "RawJSON":
    ts = repr(float(t))
    parts = ['{"metric":' + lj + ',"value":[' + ts + ',"' + fv + '"]}' for lj, fv in rows]
    return RawJSON('{"status":"success","data":{"resultType":"vector","result":[' + ",".join(parts) + "]}}")


def query_range(db: TSDB, q: str, start: float, end: float, step: float):
    """Prometheus ``/api/v1/query_range`` response body."""
    if step <= 0 or end < start:
        return {"status": "error", "errorType": "bad_data", "error": "invalid range"}
    if (end - start) / step > 11000:
        return {"status": "error", "errorType": "bad_data", "error": "exceeded maximum resolution of 11,000 points"}
    # Per-step results are memoised while no series was pushed (same rule as
    # query()): a window that slides by one step re-evaluates one step. A real
    # Prometheus evaluates the whole window in milliseconds; evaluating it
    # point by point in Python would otherwise dominate the fake's latency.
    memo = db._range_cache.get(q)
    if memo is None or memo[0] != _MUTATIONS[0]:
        memo = db._range_cache[q] = (_MUTATIONS[0], {})
    steps = memo[1]
    try:
        node = parse(q)
        ev = Evaluator(db)
        series: Dict[tuple, Tuple[Labels, List[str]]] = {}
        n = int(math.floor((end - start) / step))
        for i in range(n + 1):
            t = start + i * step
            rows = steps.get(t)
            if rows is None:
                typ, val = ev.instant(node, t)
                if typ == "scalar":
                    val = [({}, val)]
                tsr = repr(float(t))
                rows = [(tuple(sorted(labels.items())), labels, "[" + tsr + ',"' + _fmt(v) + '"]') for labels, v in val]
                steps[t] = rows
            for k, labels, cell in rows:
                ent = series.get(k)
                if ent is None:
                    ent = series[k] = (labels, [])
                ent[1].append(cell)
        if len(steps) > 4 * (n + 1) + 64:  # keep the memo bounded to about the live window
            for t in sorted(steps)[: len(steps) - 2 * (n + 1)]:
                del steps[t]
    except PromQLError as e:
        return {"status": "error", "errorType": "bad_data", "error": str(e)}
    parts = ['{"metric":' + db.label_json(l) + ',"values":[' + ",".join(vs) + "]}" for l, vs in series.values()]
    return RawJSON('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(parts) + "]}}")
