"""Continuous (in-flight) batching scheduler for the tutoring decode engine.

The reference serves one ``model.generate`` per request (SURVEY.md §3.3,
reference ``tutoring_server.py``: GetLLMAnswer -> tokenizer -> generate(max_length=150)),
so concurrent students queue behind each other.  Here one scheduler thread owns the engine's
KV-cache slots: a request is prefilled into the lowest free slot as soon as one exists (packed
varlen prefill, ``HipGPT2Engine.admit``), every live sequence advances together in graph-replayed
decode chunks over the smallest batch bucket covering the occupied slots, and a finished
sequence frees its slot at the next chunk boundary -- so a late request never waits for an
earlier batch to drain.

The loop is PIPELINED one chunk deep: chunk k+1 is enqueued before the host reads chunk k's stop
flags (a pinned copy behind chunk k, ``flags_async``), and finished sequences are gathered by a
copy enqueued behind chunk k+1 (``collect_async``: a finished row never changes), so the GPU
always has the next chunk queued while the host retires requests and prepares admissions (the
admission's host->device copies go through pinned memory and never block on the stream).  A
finished slot is reusable at once: its re-admission is stream-ordered behind the gather.

Engine protocol (``HipGPT2Engine`` implements it; tests use a CPU fake):
    max_batch, max_length, cfg.eos_token_id
    admit(prompts, slots, repetition_penalty)   prefill + first token into those slots
    decode(B, steps, repetition_penalty)        ``steps`` decode steps over slots [0, B)
    finished_flags(B) -> list[int]              per-slot stop flags
    collect(slots) -> list[list[int]]           prompt + generated tokens
    flags_async(B), collect_async(slots)        optional: the same as handles with .result()
"""
from __future__ import annotations

import heapq
import os
import threading
import time
from collections import deque
from concurrent.futures import Future
from dataclasses import dataclass, field

import torch

from ..utils.metrics import METRICS
from ..utils.trace import TRACER, roctx_range
from .gpt2_engine import _bucket


class _Ready:
    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


def flags_async(eng, B: int):
    f = getattr(eng, "flags_async", None)
    return f(B) if f is not None else _Ready(eng.finished_flags(B))


def health_async(eng):
    f = getattr(eng, "health_async", None)
    return f() if f is not None else None


def dataflow_status_async(eng):
    f = getattr(eng, "dataflow_status_async", None)
    return f() if f is not None else None


class PeerStalled(RuntimeError):
    """A tensor-parallel peer never reached a collective: the affected chunk's tokens are garbage."""


def collect_async(eng, slots: list[int]):
    f = getattr(eng, "collect_async", None)
    return f(slots) if f is not None else _Ready(eng.collect(slots))


@dataclass
class _Req:
    prompt: list[int]
    future: Future
    t_submit: float = field(default_factory=time.perf_counter)
    t_first: float = 0.0
    steps_left: int = 0  # decode steps until max_length (an upper bound: EOS may come first)


class Overloaded(RuntimeError):
    """``submit`` refused a query: the admission queue already holds ``max_queue`` queries (the
    servers answer RESOURCE_EXHAUSTED at once, so an overloaded replica sheds load in
    microseconds instead of queueing queries until their client deadlines expire)."""


class ContinuousBatcher:
    def __init__(self, engine, repetition_penalty: float = 1.2, chunk: int = 8, max_admit: int | None = None,
                 name: str = "tutor", stream_priority: int | None = None, max_queue: int = 0):
        """``max_queue``: queries allowed to wait for a free KV slot before ``submit`` raises
        ``Overloaded`` (0 = unbounded; the tutoring servers default to one batch of slots)."""
        self.engine = engine
        self.max_queue = int(max_queue or 0)
        self.rejected = 0
        env_prio = os.environ.get("DLMS_BATCHER_STREAM_PRIORITY")
        self.stream_priority = int(env_prio) if env_prio else stream_priority
        self.penalty = float(repetition_penalty)
        self.chunk = max(1, int(chunk))
        self.max_admit = max_admit or engine.max_batch
        self.name = name
        self._queue: deque[_Req] = deque()
        self._cv = threading.Condition()
        self._free = list(range(engine.max_batch))
        heapq.heapify(self._free)
        self._active: dict[int, _Req] = {}
        self._stop = False
        self._error: BaseException | None = None
        self.steps = 0
        self.completed = 0
        # side work run on this thread between decode chunks (gate/service.py GateWorker: the relevance
        # gate's encoder passes go on the decode stream right behind a chunk, never interleaved
        # kernel by kernel with it): work(idle) is called once per loop iteration, pending() says
        # whether it has anything queued or in flight (so an idle batcher does not sleep on it)
        self._side_work = None
        self._side_pending = None
        self._thread = threading.Thread(target=self._run, name=f"{name}-batcher", daemon=True)
        self._thread.start()

    def attach_side_work(self, work, pending):
        with self._cv:
            self._side_work, self._side_pending = work, pending
            self._cv.notify()

    def kick(self):
        """Wake the scheduler thread (new side work arrived)."""
        with self._cv:
            self._cv.notify()

    # ------------------------------------------------------------------ client side
    def submit(self, prompt: list[int]) -> Future:
        fut: Future = Future()
        eos, T = self.engine.cfg.eos_token_id, self.engine.max_length
        p = list(prompt) if len(prompt) else [eos]
        if len(p) >= T:  # nothing to generate (generate() pass-through semantics)
            fut.set_result(p)
            return fut
        with self._cv:
            if self._stop:
                raise RuntimeError("batcher stopped")
            if self._error is not None:
                raise RuntimeError("batcher failed") from self._error
            if self.max_queue and len(self._queue) >= self.max_queue:
                self.rejected += 1
                METRICS.inc(f"{self.name}_rejected_total")
                raise Overloaded(f"{len(self._queue)} queries already waiting for a KV slot")
            self._queue.append(_Req(p, fut))
            self._cv.notify()
        return fut

    @property
    def failed(self) -> BaseException | None:
        """The error that stopped the batcher (None while it serves)."""
        return self._error

    def generate(self, prompts: list[list[int]], timeout: float | None = None) -> list[list[int]]:
        futs = [self.submit(p) for p in prompts]
        return [f.result(timeout) for f in futs]

    def stop(self, timeout: float = 10.0):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout)

    @property
    def active(self) -> int:
        return len(self._active)

    # ------------------------------------------------------------------ scheduler thread
    def _run(self):
        try:
            dev = getattr(self.engine, "device", None)
            if dev is not None and getattr(dev, "type", None) == "cuda" and dev.index is not None:
                torch.cuda.set_device(dev)
            if self.stream_priority is not None and dev is not None and getattr(dev, "type", None) == "cuda":
                # serving beside other GPU processes on the same device (the LMS nodes' relevance
                # gates): the decode chunks go on a stream of this priority (lower = higher; the
                # graphs are replayed on it).  LMS path at 3.5 k q/s, 3 Raft nodes + BERT gates:
                # p50 863 -> 614 ms, p99 1189 -> 927, same tok/s (profiles/r4_serving_grpc.jsonl)
                torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=int(self.stream_priority)))
            with torch.no_grad():
                self._loop()
        except BaseException as e:  # fail every waiter loudly instead of hanging them
            # (the engine's device state is suspect after this -- e.g. a PeerStalled chunk left
            # garbage in the KV cache and the xGMI error word set -- so the batcher does not try
            # to continue: callers see `failed`, and the serving process exits for its supervisor
            # to restart it fresh; tutor/server.py)
            with self._cv:
                self._error = e
                waiters = list(self._active.values()) + list(self._queue)
                self._active.clear()
                self._queue.clear()
            for r in waiters:
                if not r.future.done():
                    r.future.set_exception(e)

    def _loop(self):
        eng = self.engine
        prev = None  # (flags handle, {slot: request} live when that chunk was enqueued) of the last chunk
        retiring = None  # (requests, collect handle) of sequences found finished
        while True:
            with self._cv:
                while not self._stop and not self._queue and not self._active and prev is None and retiring is None \
                        and not (self._side_pending is not None and self._side_pending()):
                    self._cv.wait()
                if self._stop:
                    waiters = list(self._queue) + list(self._active.values()) + \
                        ([r for _, r in retiring[0]] if retiring else [])
                    self._queue.clear()
                    self._active.clear()
                    for r in waiters:
                        if not r.future.done():
                            r.future.set_exception(RuntimeError("batcher stopped"))
                    return
                admits: list[tuple[int, _Req]] = []
                while self._queue and self._free and len(admits) < self.max_admit:
                    r = self._queue.popleft()
                    # RUNNING from here on: a caller's cancel() (a gRPC deadline, asyncio.wait_for
                    # timing out on a wrap_future) can no longer race the result; a request
                    # cancelled while it queued is dropped
                    if r.future.set_running_or_notify_cancel():
                        admits.append((heapq.heappop(self._free), r))
            if admits:
                ta = time.perf_counter()
                with roctx_range("prefill"):
                    eng.admit([r.prompt for _, r in admits], [s for s, _ in admits], self.penalty)
                TRACER.complete("tutor.admit", ta, cat="tutor", n=len(admits),
                                tokens=sum(len(r.prompt) for _, r in admits))
                t_first = time.perf_counter()  # prefill (first token included) is enqueued
                for s, r in admits:
                    self._active[s] = r
                    r.t_first = t_first
                    r.steps_left = max(0, eng.max_length - len(r.prompt) - 1)  # prefill made token 1
                    METRICS.observe(f"{self.name}_queue_ms", (ta - r.t_submit) * 1e3)
                    METRICS.observe(f"{self.name}_ttft_ms", (t_first - r.t_submit) * 1e3)
            cur = None
            # never decode far past the point where every live sequence has hit max_length: the last
            # chunk is cut to the longest remaining budget, and once every budget is spent only a
            # single step runs while the in-flight flags retire them (one step, not a whole no-op
            # chunk, on every query's latency at low load; at least one step keeps the loop making
            # progress even if a sequence's flag were late)
            steps = 0
            if self._active:
                steps = max(1, min(self.chunk, max(r.steps_left for r in self._active.values())))
            if steps > 0:
                B = min(_bucket(max(self._active) + 1), eng.max_batch)
                td = time.perf_counter()
                # the budget each live request actually gives up to this chunk (a request near its
                # max_length gives less than `steps`): an aborted chunk refunds exactly that
                taken = {}
                for s, r in self._active.items():
                    taken[s] = min(steps, r.steps_left)
                    r.steps_left -= taken[s]
                with roctx_range("decode_chunk"):
                    eng.decode(B, steps, self.penalty)
                    cur = (flags_async(eng, B), dict(self._active), health_async(eng), dataflow_status_async(eng),
                           taken)
                self.steps += steps
                TRACER.complete("tutor.decode_chunk", td, cat="tutor", bucket=B, live=len(self._active),
                                steps=steps)
            if self._side_work is not None:  # behind the chunk just enqueued, before the next one
                self._side_work(cur is None and prev is None)
            if retiring is not None:  # gathered behind the chunk before `cur`: ready or nearly
                self._retire(*retiring)
                retiring = None
            if prev is not None:  # chunk k's flags while chunk k+1 runs
                flags = prev[0].result()
                if prev[2] is not None and prev[2].result():
                    # fail every live request (the _run handler) rather than return wrong tokens
                    METRICS.inc(f"{self.name}_peer_stalls")
                    raise PeerStalled("a tensor-parallel peer timed out in an xGMI collective")
                if prev[3] is not None and prev[3].result():
                    # the persistent dataflow kernel aborted that chunk before committing anything:
                    # no row advanced (the engine serves launch-per-op for a while); give the
                    # requests their step budget back so later chunks are not cut short
                    METRICS.inc(f"{self.name}_dataflow_aborts")
                    for s, r in prev[1].items():
                        if self._active.get(s) is r:
                            r.steps_left += prev[4].get(s, 0)
                # by identity: a slot retired one chunk earlier may already hold a new request
                done = [s for s, r in prev[1].items() if s < len(flags) and flags[s] and self._active.get(s) is r]
                if done:
                    handle = collect_async(eng, done)
                    with self._cv:
                        reqs = [(s, self._active.pop(s)) for s in done]
                        for s in done:
                            heapq.heappush(self._free, s)
                    retiring = (reqs, handle)
                    METRICS.set(f"{self.name}_active", len(self._active))
                    METRICS.set(f"{self.name}_kv_slot_occupancy", len(self._active) / eng.max_batch)
            prev = cur

    def _retire(self, reqs, handle):
        outs = handle.result()
        now = time.perf_counter()
        for (s, r), out in zip(reqs, outs):
            self.completed += 1
            n_new = len(out) - len(r.prompt)
            METRICS.observe(f"{self.name}_request_ms", (now - r.t_submit) * 1e3)
            if n_new > 1:  # time per output token after the first
                METRICS.observe(f"{self.name}_tpot_ms", (now - r.t_first) * 1e3 / (n_new - 1))
            METRICS.inc(f"{self.name}_tokens", n_new)
            if not r.future.done():
                r.future.set_result(out)
