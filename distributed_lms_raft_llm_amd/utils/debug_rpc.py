"""Internal debug/health RPCs, served next to the public services on every process
(``lmsinternal.Debug/<Method>``, JSON bodies, generic handlers -- lms.proto stays untouched):

  Health   {"ok": bool, ...}           liveness + readiness (tutor: engine alive, slots in use)
  Status   component status            (LMS: Raft role/term/leader/commit/applied)
  Metrics  METRICS.snapshot()          counters + latency histograms
  Trace    {"events": [...]}           the tracer ring (utils/trace.py), optionally cleared

The reference has no health or metrics surface at all.
"""
from __future__ import annotations

import json

import grpc

from .metrics import METRICS
from .trace import TRACER

SERVICE = "lmsinternal.Debug"


def debug_handler(health=None, status=None):
    """``health``/``status``: zero-argument callables returning JSON-able dicts."""

    def _wrap(fn):
        def h(body: bytes, context) -> bytes:
            req = json.loads(body) if body else {}
            return json.dumps(fn(req), default=str).encode()

        return grpc.unary_unary_rpc_method_handler(h)

    def _health(req):
        out = {"ok": True}
        if health is not None:
            out.update(health())
        return out

    def _trace(req):
        ev = TRACER.events()
        if req.get("clear"):
            TRACER.clear()
        return {"enabled": TRACER.enabled, "events": ev}

    return grpc.method_handlers_generic_handler(SERVICE, {
        "Health": _wrap(_health),
        "Status": _wrap(lambda req: status() if status is not None else {}),
        "Metrics": _wrap(lambda req: METRICS.snapshot()),
        "Trace": _wrap(_trace),
    })


def debug_call(channel_or_addr, method: str, request: dict | None = None, timeout: float = 5.0) -> dict:
    from .. import wire

    ch = wire.channel(channel_or_addr) if isinstance(channel_or_addr, str) else channel_or_addr
    fn = ch.unary_unary(f"/{SERVICE}/{method}", request_serializer=None, response_deserializer=None)
    try:
        return json.loads(fn(json.dumps(request or {}).encode(), timeout=timeout))
    finally:
        if isinstance(channel_or_addr, str):
            ch.close()
