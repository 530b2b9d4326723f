"""Structured event tracing: the reference's only trace is ``print`` on every Raft
step; here Raft transitions (role/term/leader/commit) and the request lifecycle (LMS RPC, gate,
tutor queue, prefill, decode chunks) are recorded as Chrome-trace events ("X" spans, "i"
instants) in a bounded in-memory ring, dumped as JSON lines or a ``chrome://tracing`` /
Perfetto file.  Enabled by ``DLMS_TRACE=<path>`` (dumped at exit) or ``TRACER.enable()``.

GPU side: ``roctx_range(name)`` pushes a roctx range (``libroctx64``) so ``rocprofv3
--marker-trace`` lines the host phases up with the kernel timeline; it is a no-op unless
``DLMS_ROCTX=1`` (the library is loaded lazily and never required).
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import json
import os
import threading
import time
from collections import deque


class Tracer:
    def __init__(self, cap: int = 200_000):
        self.enabled = False
        self._ev: deque = deque(maxlen=cap)
        self._lock = threading.Lock()
        self._t0 = time.perf_counter()
        self._pid = os.getpid()

    def enable(self, on: bool = True):
        self.enabled = on

    def _us(self, t: float | None = None) -> float:
        return ((time.perf_counter() if t is None else t) - self._t0) * 1e6

    def instant(self, name: str, cat: str = "dlms", **args):
        if not self.enabled:
            return
        ev = {"name": name, "cat": cat, "ph": "i", "s": "t", "ts": self._us(), "pid": self._pid,
              "tid": threading.get_ident(), "args": args}
        with self._lock:
            self._ev.append(ev)

    def complete(self, name: str, t_start: float, t_end: float | None = None, cat: str = "dlms", **args):
        """Record a span from perf_counter timestamps (for spans measured elsewhere)."""
        if not self.enabled:
            return
        ts = self._us(t_start)
        ev = {"name": name, "cat": cat, "ph": "X", "ts": ts, "dur": self._us(t_end) - ts, "pid": self._pid,
              "tid": threading.get_ident(), "args": args}
        with self._lock:
            self._ev.append(ev)

    @contextlib.contextmanager
    def span(self, name: str, cat: str = "dlms", **args):
        if not self.enabled:
            yield
            return
        t = time.perf_counter()
        try:
            yield
        finally:
            self.complete(name, t, cat=cat, **args)

    def events(self) -> list[dict]:
        with self._lock:
            return list(self._ev)

    def clear(self):
        with self._lock:
            self._ev.clear()

    def dump(self, path: str):
        """``*.jsonl``: one event per line; anything else: a Chrome/Perfetto trace file."""
        evs = self.events()
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            if path.endswith(".jsonl"):
                for e in evs:
                    f.write(json.dumps(e) + "\n")
            else:
                json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
        os.replace(tmp, path)


TRACER = Tracer()

_env_path = os.environ.get("DLMS_TRACE")
if _env_path:
    TRACER.enable()
    atexit.register(lambda: TRACER.dump(_env_path.replace("{pid}", str(os.getpid()))))


# ---------------------------------------------------------------------- roctx
_roctx = None
_roctx_on = os.environ.get("DLMS_ROCTX") == "1"


def _lib():
    global _roctx, _roctx_on
    if _roctx is None:
        try:
            _roctx = ctypes.CDLL("libroctx64.so")
            _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _roctx.roctxMarkA.argtypes = [ctypes.c_char_p]
        except OSError:
            _roctx_on = False
            _roctx = False
    return _roctx


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _lib() if _roctx_on else None
    if not lib:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def roctx_mark(name: str):
    lib = _lib() if _roctx_on else None
    if lib:
        lib.roctxMarkA(name.encode())
