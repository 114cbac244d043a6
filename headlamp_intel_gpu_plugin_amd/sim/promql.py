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

Storage is :mod:`.tsdb` (series on a scrape grid or pushed samples, 5-minute
lookback); the lexer / parser is :mod:`.promql_parse`. Both are re-exported
here, the module the fake control plane and the tests import.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional, Tuple

from .promql_parse import (AGGREGATIONS, BIN_PREC, RANGE_FUNCS, RANK_AGGREGATIONS, SET_OPS, Matcher,  # noqa: F401
                           PromQLError, parse)
from .tsdb import _MUTATIONS, LOOKBACK_S, Labels, Series, TSDB, changes_since  # noqa: F401


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
        counting = op == "count"  # a function-backed series always has a sample: no value needed
        # A count's partials hold 1.0 per series, not its values: they are kept apart from the value partials.
        key = (sig, byt, wt, math.floor(t / iv), counting)
        hit = db._agg_cache.get(key)
        if hit is None:
            parts: Dict[tuple, list] = {}
            pushed = []
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
        if op == "unless" and matching and matching[0] == "on" and not matching[1]:
            # `x unless on() <non-empty>` is empty whatever x is (every row
            # matches on no labels): answered without evaluating x, as `and`
            # above — the client's first query appends node-exporter's page
            # and totals this way, to be dropped where the exporter reports.
            rt, rv = self.instant(rhs, t)
            if rt == "vector" and rv:
                return ("vector", [])
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


def _fmt_ts(t: float) -> str:
    """A sample timestamp as Prometheus's JSON writes it: seconds, then the milliseconds (3 digits) unless zero."""
    ms = int(round(float(t) * 1000.0))
    sec, frac = divmod(ms, 1000)
    return f"{sec}.{frac:03d}" if frac else str(sec)


class RawJSON(str):
    """A pre-encoded JSON response body (served as-is by the fake apiserver)."""


def cache_stamp(db: TSDB, t: float):
    """What an instant answer at ``t`` depends on: the function-backed series' sample-grid bucket and the TSDB's
    mutation count (pushes). Two evaluations with the same stamp give the same answer; None when the TSDB mixes
    sample intervals (no stamp is cheap to compute)."""
    if len(db._fn_intervals) > 1:
        return None
    iv = next(iter(db._fn_intervals)) if db._fn_intervals else 1.0
    return (math.floor(t / iv), _MUTATIONS[0])


def query(db: TSDB, q: str, t: float):
    """Prometheus ``/api/v1/query`` response body (dict on error/scalar, RawJSON for vectors).

    Function-backed series only change at their sample interval and pushed
    series only on push, so a vector result is reused for repeated queries
    within one interval bucket while nothing was pushed — the evaluation
    cost of a Python TSDB would otherwise dominate the fake's latency, where
    a real Prometheus answers such a selector in well under a millisecond.
    """
    stamp = cache_stamp(db, t)
    cacheable = stamp is not None
    if cacheable:
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
    ts = _fmt_ts(t)
    parts = ['{"metric":' + lj + ',"value":[' + ts + ',"' + fv + '"]}' for lj, fv in rows]
    return RawJSON('{"status":"success","data":{"resultType":"vector","result":[' + ",".join(parts) + "]}}")


def query_range(db: TSDB, q: str, start: float, end: float, step: float):
    """Prometheus ``/api/v1/query_range`` response body."""
    if step <= 0 or end < start:
        return {"status": "error", "errorType": "bad_data", "error": "invalid range"}
    if (end - start) / step > 11000:
        return {"status": "error", "errorType": "bad_data", "error": "exceeded maximum resolution of 11,000 points"}
    # Per-step results are memoised: a window that slides by one step
    # re-evaluates one step, and samples pushed since (tsdb.changes_since)
    # drop only the steps they can change — the ones at or after the pushed
    # sample, not the whole window. A real Prometheus evaluates the whole
    # window in milliseconds; evaluating it point by point in Python would
    # otherwise dominate the fake's latency.
    memo = db._range_cache.get(q)
    if memo is not None and memo[0] != _MUTATIONS[0]:
        changed = changes_since(memo[0])
        if changed is None:
            memo = None
        else:
            steps = memo[1]
            # Changes are (T, inf): a sample pushed at T; (-inf, X): samples
            # dropped, seen up to X; (-inf, inf): a new series.
            lo = min((c[0] for c in changed if c[1] == math.inf), default=math.inf)
            hi = max((c[1] for c in changed if c[1] != math.inf), default=-math.inf)
            for t in [t for t in steps if t >= lo or t <= hi]:
                del steps[t]
            memo = db._range_cache[q] = (_MUTATIONS[0], steps)
    if memo is None:
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
                tsr = _fmt_ts(t)
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
