"""Process-wide counters and latency histograms: Raft elections and commit
latency, gate/LLM latency, tokens/s, batch sizes, queue depth.  Exported as JSON (``snapshot()``)
for the bench scripts and the ``/metrics``-style debug RPC; the reference only ``print``s.
"""
from __future__ import annotations

import bisect
import json
import threading
import time


class Histogram:
    def __init__(self, cap: int = 4096):
        self.cap = cap
        self.values: list[float] = []
        self.count = 0
        self.total = 0.0

    def add(self, v: float):
        self.count += 1
        self.total += v
        if len(self.values) >= self.cap:
            self.values.pop(0)
        self.values.append(v)

    def quantile(self, q: float) -> float:
        if not self.values:
            return 0.0
        s = sorted(self.values)
        return s[min(len(s) - 1, int(q * (len(s) - 1) + 0.5))]

    def summary(self) -> dict:
        return {"count": self.count, "mean": self.total / self.count if self.count else 0.0,
                "p50": self.quantile(0.5), "p90": self.quantile(0.9), "p99": self.quantile(0.99),
                "max": max(self.values) if self.values else 0.0}


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: dict[str, float] = {}
        self.gauges: dict[str, float] = {}
        self.hists: dict[str, Histogram] = {}
        self.t0 = time.time()

    def inc(self, name: str, v: float = 1.0):
        with self._lock:
            self.counters[name] = self.counters.get(name, 0.0) + v

    def set(self, name: str, v: float):
        with self._lock:
            self.gauges[name] = v

    def observe(self, name: str, v: float):
        with self._lock:
            h = self.hists.get(name)
            if h is None:
                h = self.hists[name] = Histogram()
            h.add(float(v))

    def snapshot(self) -> dict:
        with self._lock:
            return {"uptime_s": time.time() - self.t0, "counters": dict(self.counters), "gauges": dict(self.gauges),
                    "histograms": {k: h.summary() for k, h in self.hists.items()}}

    def to_json(self) -> str:
        return json.dumps(self.snapshot())

    def reset(self):
        with self._lock:
            self.counters.clear()
            self.gauges.clear()
            self.hists.clear()


METRICS = Metrics()


class Timer:
    def __init__(self, name: str, metrics: Metrics = METRICS):
        self.name, self.m = name, metrics

    def __enter__(self):
        self.t = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.ms = (time.perf_counter() - self.t) * 1e3
        self.m.observe(self.name, self.ms)
