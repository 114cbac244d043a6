"""Lexer and parser of the PromQL subset :mod:`.promql` evaluates.

``parse(q)`` returns the expression tree the evaluator walks (tuples tagged by
node kind); :class:`Matcher` is a label matcher (``= != =~ !~``) the TSDB's
selector index applies.
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

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
