"""Fake kube-apiserver + Prometheus-behind-the-service-proxy.

Serves exactly the HTTP surface the plugin touches (SURVEY.md §2.3 call sites
M1–M11, AMD equivalents):

* ``GET /api/v1/nodes``, ``GET /api/v1/pods`` (``labelSelector`` with
  equality and set-based terms, ``fieldSelector=spec.nodeName=…``),
  ``GET /api/v1/namespaces/{ns}/pods``;
* ``GET /apis/amd.com/v1alpha1/deviceconfigs`` (404 when the CRD is "not
  installed", to exercise graceful degradation);
* ``GET /api/v1/namespaces/{ns}/services/{svc}:{port}/proxy/api/v1/query``
  and ``…/query_range`` backed by :mod:`..sim.promql` — only the services in
  ``prometheus_up`` answer, the rest return a 503 ``Status``.

Every response is delayed by an injected round-trip latency
(``latency_ms``), identical for every client, so the plugin's request
schedule and the reference's replayed schedule are compared on equal terms
(BASELINE.md "How the comparison will be made"). List bodies are
serialised once per cluster version and cached, like a watch cache.

Runs on its own asyncio loop in a daemon thread (:class:`ServerThread`).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import random
import json
import re
import threading
import time
from typing import Dict, Iterable, List, Optional, Tuple
from urllib.parse import unquote

from aiohttp import web

from ..models.cluster import SyntheticCluster
from . import promql

DEFAULT_PROM_SERVICE = ("monitoring", "kube-prometheus-stack-prometheus", "9090")


# ---------------------------------------------------------------------------
# Label / field selectors
# ---------------------------------------------------------------------------

_SET_RE = re.compile(r"^\s*([A-Za-z0-9_./-]+)\s+(in|notin)\s+\(([^)]*)\)\s*$")


def _split_terms(sel: str) -> List[str]:
    terms, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            terms.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        terms.append(cur)
    return [t.strip() for t in terms if t.strip()]


def parse_label_selector(sel: str):
    """Returns a predicate over a labels dict. Raises ValueError on bad syntax."""
    preds = []
    for term in _split_terms(sel or ""):
        m = _SET_RE.match(term)
        if m:
            key, op, vals = m.group(1), m.group(2), {v.strip() for v in m.group(3).split(",") if v.strip()}
            if op == "in":
                preds.append(lambda l, k=key, vs=vals: l.get(k) in vs)
            else:
                preds.append(lambda l, k=key, vs=vals: l.get(k) not in vs)
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            preds.append(lambda l, k=k.strip(), v=v.strip(): l.get(k) != v)
        elif "==" in term or "=" in term:
            k, v = term.split("==", 1) if "==" in term else term.split("=", 1)
            preds.append(lambda l, k=k.strip(), v=v.strip(): l.get(k) == v)
        elif term.startswith("!"):
            preds.append(lambda l, k=term[1:].strip(): k not in l)
        elif re.match(r"^[A-Za-z0-9_./-]+$", term):
            preds.append(lambda l, k=term: k in l)
        else:
            raise ValueError(f"unable to parse requirement: {term!r}")
    return lambda labels: all(p(labels) for p in preds)


def parse_field_selector(sel: str):
    preds = []
    for term in _split_terms(sel or ""):
        neg = "!=" in term
        k, v = term.split("!=" if neg else ("==" if "==" in term else "="), 1)
        path = k.strip().split(".")

        def get(obj, path=path):
            for p in path:
                obj = obj.get(p) if isinstance(obj, dict) else None
            return "" if obj is None else str(obj)

        preds.append((lambda o, g=get, v=v.strip(): g(o) != v) if neg else (lambda o, g=get, v=v.strip(): g(o) == v))
    return lambda obj: all(p(obj) for p in preds)


# ---------------------------------------------------------------------------
# Server
# ---------------------------------------------------------------------------

class FakeCluster:
    """State + behaviour knobs of the fake control plane."""

    def __init__(self, cluster: SyntheticCluster, db: Optional[promql.TSDB] = None, *, latency_ms: float = 20.0,
                 crd_installed: bool = True, prometheus_up: Iterable[Tuple[str, str, str]] = (DEFAULT_PROM_SERVICE,),
                 per_kb_us: float = 0.0, now=time.time, fail_rate: float = 0.0, hang_rate: float = 0.0,
                 seed: int = 0):
        self.cluster = cluster
        # Fault injection: each request independently fails with a 503 Status
        # (fail_rate) or never answers within the client's 2 s budget
        # (hang_rate, held 3 s) — seeded, so a failing run reproduces.
        self.fail_rate = fail_rate
        self.hang_rate = hang_rate
        self._rng = random.Random(seed)
        self.faults = {"failed": 0, "hung": 0}
        self.db = db if db is not None else promql.TSDB()
        self.latency_ms = latency_ms
        self.per_kb_us = per_kb_us
        self.crd_installed = crd_installed
        self.prometheus_up = {tuple(s) for s in prometheus_up}
        self.now = now
        self.version = 1
        self._cache: Dict[str, bytes] = {}
        self.requests: List[Tuple[str, float]] = []  # (path, server-side seconds)
        self.lock = threading.Lock()

    def bump(self) -> None:
        """Invalidate cached list bodies after mutating ``cluster``."""
        self.version += 1
        self._cache.clear()

    def reset_stats(self) -> None:
        with self.lock:
            self.requests = []

    def stats(self) -> Dict[str, int]:
        with self.lock:
            out: Dict[str, int] = {}
            for p, _ in self.requests:
                kind = "prometheus" if "/proxy/" in p else "apiserver"
                out[kind] = out.get(kind, 0) + 1
            out["total"] = len(self.requests)
            return out

    # -- bodies ---------------------------------------------------------
    def _list(self, kind: str, items: list) -> bytes:
        return json.dumps({"kind": kind, "apiVersion": "v1", "metadata": {"resourceVersion": str(self.version)},
                           "items": items}, separators=(",", ":")).encode()

    def _cached(self, key: str, build) -> bytes:
        b = self._cache.get(key)
        if b is None:
            b = build()
            self._cache[key] = b
        return b

    def pods_body(self, ns: Optional[str], label_sel: str, field_sel: str) -> bytes:
        key = f"pods|{ns}|{label_sel}|{field_sel}"

        def build():
            lp = parse_label_selector(label_sel)
            fp = parse_field_selector(field_sel)
            items = [p for p in self.cluster.pods
                     if (ns is None or p["metadata"]["namespace"] == ns) and lp(p["metadata"].get("labels", {})) and fp(p)]
            return self._list("PodList", items)

        return self._cached(key, build)

    def nodes_body(self, label_sel: str) -> bytes:
        def build():
            lp = parse_label_selector(label_sel)
            return self._list("NodeList", [n for n in self.cluster.nodes if lp(n["metadata"].get("labels", {}))])

        return self._cached(f"nodes|{label_sel}", build)

    def deviceconfigs_body(self, ns: Optional[str]) -> bytes:
        def build():
            items = [d for d in self.cluster.device_configs if ns is None or d["metadata"]["namespace"] == ns]
            return json.dumps({"apiVersion": "amd.com/v1alpha1", "kind": "DeviceConfigList",
                               "metadata": {"resourceVersion": str(self.version)}, "items": items}).encode()

        return self._cached(f"dc|{ns}", build)


def _status(code: int, reason: str, message: str) -> web.Response:
    body = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": message, "reason": reason, "code": code}
    return web.json_response(body, status=code)


def build_app(fc: FakeCluster) -> web.Application:
    @web.middleware
    async def latency(request: web.Request, handler):
        t0 = time.perf_counter()
        if fc.fail_rate or fc.hang_rate:
            x = fc._rng.random()
            if x < fc.hang_rate:
                fc.faults["hung"] += 1
                await asyncio.sleep(3.0)
            elif x < fc.hang_rate + fc.fail_rate:
                fc.faults["failed"] += 1
                await asyncio.sleep(fc.latency_ms / 1000.0)
                return web.json_response({"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                          "message": "injected fault", "reason": "ServiceUnavailable", "code": 503},
                                         status=503)
        resp = await handler(request)
        work = time.perf_counter() - t0
        delay = fc.latency_ms / 1000.0
        if fc.per_kb_us and getattr(resp, "body", None) is not None:
            delay += len(resp.body) / 1024.0 * fc.per_kb_us / 1e6
        if delay > 0:
            await asyncio.sleep(delay)
        with fc.lock:
            fc.requests.append((request.path_qs, work))
        return resp

    def raw(body: bytes) -> web.Response:
        return web.Response(body=body, content_type="application/json")

    async def nodes(req):
        try:
            return raw(fc.nodes_body(req.query.get("labelSelector", "")))
        except ValueError as e:
            return _status(400, "BadRequest", str(e))

    async def pods(req):
        ns = req.match_info.get("ns")
        try:
            return raw(fc.pods_body(ns, req.query.get("labelSelector", ""), req.query.get("fieldSelector", "")))
        except ValueError as e:
            return _status(400, "BadRequest", str(e))

    async def deviceconfigs(req):
        if not fc.crd_installed:
            return _status(404, "NotFound", "the server could not find the requested resource")
        return raw(fc.deviceconfigs_body(req.match_info.get("ns")))

    async def proxy(req):
        ns = req.match_info["ns"]
        svc, _, port = req.match_info["svc"].partition(":")
        if (ns, svc, port) not in fc.prometheus_up:
            return _status(503, "ServiceUnavailable", f'no endpoints available for service "{svc}"')
        sub = req.match_info["sub"]
        q = req.query.get("query")
        if q is None:
            return web.json_response({"status": "error", "errorType": "bad_data", "error": "missing query"}, status=400)
        now = fc.now()
        loop = asyncio.get_running_loop()
        # Prometheus is its own server: its evaluation runs on its own thread,
        # so a slow (Python) evaluation does not hold the apiserver's list
        # responses on this event loop.
        if sub == "api/v1/query":
            t = float(req.query.get("time", now))
            body = await loop.run_in_executor(prom_pool, promql.query, fc.db, q, t)
        elif sub == "api/v1/query_range":
            try:
                rng = float(req.query["start"]), float(req.query["end"]), float(req.query["step"])
            except (KeyError, ValueError):
                rng = None
            if rng is None:
                body = {"status": "error", "errorType": "bad_data", "error": "bad range parameters"}
            else:
                body = await loop.run_in_executor(prom_pool, promql.query_range, fc.db, q, *rng)
        else:
            return _status(404, "NotFound", sub)
        if isinstance(body, promql.RawJSON):
            return web.Response(text=body, content_type="application/json")
        return web.json_response(body, status=200 if body["status"] == "success" else 400)

    # One evaluation thread: the TSDB's lazily built indexes and caches are not
    # shared between concurrent evaluations.
    prom_pool = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="fake-prometheus")

    async def stop_pool(_app):
        prom_pool.shutdown(wait=False)

    app = web.Application(middlewares=[latency])
    app.on_cleanup.append(stop_pool)
    app.router.add_get("/api/v1/nodes", nodes)
    app.router.add_get("/api/v1/pods", pods)
    app.router.add_get("/api/v1/namespaces/{ns}/pods", pods)
    app.router.add_get("/apis/amd.com/v1alpha1/deviceconfigs", deviceconfigs)
    app.router.add_get("/apis/amd.com/v1alpha1/namespaces/{ns}/deviceconfigs", deviceconfigs)
    app.router.add_get("/api/v1/namespaces/{ns}/services/{svc}/proxy/{sub:.*}", proxy)
    return app


class ServerThread:
    """Run the fake control plane on 127.0.0.1 in a background thread."""

    def __init__(self, fc: FakeCluster, host: str = "127.0.0.1", port: int = 0):
        self.fc = fc
        self.host = host
        self.port = port
        self._loop = asyncio.new_event_loop()
        self._runner: Optional[web.AppRunner] = None
        self._thread = threading.Thread(target=self._run, daemon=True, name="fake-apiserver")
        self._ready = threading.Event()
        self._error: Optional[BaseException] = None

    def _run(self) -> None:
        asyncio.set_event_loop(self._loop)
        try:
            self._loop.run_until_complete(self._start())
        except BaseException as e:  # surfaced by start()
            self._error = e
            self._ready.set()
            return
        self._ready.set()
        self._loop.run_forever()

    async def _start(self) -> None:
        self._runner = web.AppRunner(build_app(self.fc), access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port, backlog=256)
        await site.start()
        self.port = self._runner.addresses[0][1]

    def start(self) -> "ServerThread":
        self._thread.start()
        self._ready.wait(30)
        if self._error:
            raise self._error
        return self

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def stop(self) -> None:
        if self._runner is None:
            return

        async def _stop():
            await self._runner.cleanup()

        fut = asyncio.run_coroutine_threadsafe(_stop(), self._loop)
        try:
            fut.result(10)
        finally:
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(10)
            self._runner = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def make_fake(nodes: int, *, source: str = "amd-exporter", latency_ms: float = 20.0, crd_installed: bool = True,
              prometheus_up=(DEFAULT_PROM_SERVICE,), live=None, preset: Optional[str] = None,
              fail_rate: float = 0.0, hang_rate: float = 0.0, seed: int = 0) -> FakeCluster:
    """Convenience: synthetic cluster of ``nodes`` × 8 MI355X (or a BASELINE ``preset``) + telemetry + fake control plane."""
    import copy

    from ..models.cluster import PRESETS, SyntheticCluster, spec_for_nodes
    from ..models.telemetry import populate

    cluster = SyntheticCluster(copy.deepcopy(PRESETS[preset]) if preset else spec_for_nodes(nodes))
    db = promql.TSDB()
    # "both": a kube-prometheus-stack cluster scrapes node-exporter AND the AMD exporter.
    for src in (("amd-exporter", "node-exporter") if source == "both" else (source,)):
        populate(db, cluster, source=src, live=live)
    return FakeCluster(cluster, db, latency_ms=latency_ms, crd_installed=crd_installed, prometheus_up=prometheus_up,
                       fail_rate=fail_rate, hang_rate=hang_rate, seed=seed)


__all__ = ["FakeCluster", "ServerThread", "build_app", "make_fake", "parse_label_selector", "parse_field_selector",
           "DEFAULT_PROM_SERVICE", "unquote"]
