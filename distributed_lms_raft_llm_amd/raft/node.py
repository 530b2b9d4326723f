"""A live Raft node: the pure ``RaftCore`` driven by a clock thread, a transport and an apply
thread.

Threading model (the reference has none: its gRPC pool and its 10 ms driver thread mutate
``term``/``log``/``state`` concurrently, ``lms_server.py:1575,1595``):

* every access to the core happens under one lock (``self._lock``), so the core stays
  single-threaded; RPC handler threads hand their message in and get the reply back;
* outgoing messages go to the transport, which sends asynchronously (never under the lock);
* committed entries are applied in log order by a dedicated apply thread; a client proposal
  blocks on a future resolved when ITS entry (same index, same term) has been applied -- so the
  LMS replies after commit, unlike the reference which acknowledges before replication.
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from concurrent.futures import Future

from ..utils.metrics import METRICS
from ..utils.trace import TRACER
from .core import LEADER, REQUESTS, NotLeader, RaftConfig, RaftCore

log = logging.getLogger("dlms.raft")


class RaftNode:
    def __init__(self, node_id: int, peers: dict[int, str], storage, state_machine, transport=None,
                 config: RaftConfig | None = None, tick: float = 0.01, snapshot_every: int = 2000):
        """``state_machine`` provides ``apply(index, command)``, ``snapshot() -> str``,
        ``restore(str)``; ``peers`` maps peer id -> address (self excluded)."""
        self.id = node_id
        self.peer_addresses = dict(peers)
        self.sm = state_machine
        self.transport = transport
        self.tick_dt = tick
        self.snapshot_every = snapshot_every
        self._lock = threading.RLock()
        self._t0 = time.monotonic()
        self.core = RaftCore(node_id, sorted(peers), storage, config, now=self._now())
        self._waiters: dict[int, tuple[int, Future]] = {}
        self._apply_q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.applied_index = self.core.last_applied
        self._applied_cv = threading.Condition()
        self._seen = (self.core.role, self.core.current_term, self.core.leader_id)
        snap = storage.snapshot_data()
        if snap:
            state_machine.restore(snap)

    def _now(self) -> float:
        return time.monotonic() - self._t0

    # ------------------------------------------------------------------ lifecycle
    def start(self):
        for fn, name in ((self._tick_loop, "raft-tick"), (self._apply_loop, "raft-apply")):
            t = threading.Thread(target=fn, name=f"{name}-{self.id}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self):
        self._stop.set()
        self._apply_q.put(None)
        for t in self._threads:
            t.join(timeout=2)
        with self._lock:
            for _, (_, fut) in list(self._waiters.items()):
                if not fut.done():
                    fut.set_exception(NotLeader(None))
            self._waiters.clear()

    # ------------------------------------------------------------------ event plumbing
    def _dispatch(self, msgs, reply_to=None):
        """Send msgs (not under the lock); return the reply addressed to ``reply_to`` if any."""
        reply = None
        for m in msgs:
            if reply_to is not None and reply is None and m.dst == reply_to.src and not isinstance(m, REQUESTS):
                reply = m
            elif self.transport is not None:
                self.transport.send(m)
        return reply

    def _collect(self):
        """Move committed entries to the apply queue and record role/term/leader transitions
        (caller holds the lock)."""
        if self.core.pending_restore is not None:
            self._apply_q.put(("restore", self.core.last_applied, self.core.pending_restore))
            self.core.pending_restore = None
            TRACER.instant("raft.install_snapshot", cat="raft", node=self.id, index=self.core.last_applied)
        committed = self.core.take_committed()
        for idx, e in committed:
            self._apply_q.put(("entry", idx, e))
        if committed:
            TRACER.instant("raft.commit", cat="raft", node=self.id, first=committed[0][0], last=committed[-1][0])
        cur = (self.core.role, self.core.current_term, self.core.leader_id)
        if cur != self._seen:
            role, term, leader = cur
            if term != self._seen[1]:
                METRICS.set(f"raft_term_n{self.id}", term)
            if role != self._seen[0]:
                if role == LEADER:
                    METRICS.inc("raft_leaderships_won")
                    log.info("node %d became leader for term %d", self.id, term)
                elif role == "candidate":
                    METRICS.inc("raft_elections_started")
            TRACER.instant("raft.transition", cat="raft", node=self.id, role=role, term=term, leader=leader)
            self._seen = cur

    def _tick_loop(self):
        while not self._stop.is_set():
            with self._lock:
                out = self.core.tick(self._now())
                self._collect()
                self._fail_stale_waiters()
            self._dispatch(out)
            self._stop.wait(self.tick_dt)

    def _fail_stale_waiters(self):
        if self.core.role == LEADER or not self._waiters:
            return
        # keep waiting: the new leader may still commit these entries; the apply loop
        # resolves them either way (success if the term matches, NotLeader otherwise)

    def handle(self, msg):
        """Process an incoming RPC request message and return the response message."""
        with self._lock:
            out = self.core.step(msg, self._now())
            self._collect()
        return self._dispatch(out, reply_to=msg)

    def deliver(self, msg):
        """Process a response message arriving from the transport."""
        with self._lock:
            out = self.core.step(msg, self._now())
            self._collect()
        self._dispatch(out)

    # ------------------------------------------------------------------ apply
    def _apply_loop(self):
        while True:
            item = self._apply_q.get()
            if item is None:
                return
            kind, idx, payload = item
            if kind == "restore":
                self.sm.restore(payload)
                result, term = None, None
            else:
                try:
                    result = self.sm.apply(idx, payload.command)
                except Exception as e:  # a bad entry must not kill replication
                    log.exception("apply failed at %d: %s", idx, e)
                    result = None
                term = payload.term
            with self._lock:
                w = self._waiters.pop(idx, None) if kind == "entry" else None
                if kind == "restore":
                    for i in [i for i in self._waiters if i <= idx]:
                        _, fut = self._waiters.pop(i)
                        fut.set_exception(NotLeader(self.core.leader_id))
            if w is not None:
                wterm, fut = w
                if wterm == term:
                    fut.set_result(result)
                else:
                    fut.set_exception(NotLeader(self.core.leader_id))
            with self._applied_cv:
                self.applied_index = idx
                self._applied_cv.notify_all()
            if self._apply_q.empty():
                export = getattr(self.sm, "export", None)
                if export is not None:
                    try:
                        export()
                    except Exception:
                        log.exception("state export failed")
                self._maybe_snapshot()

    def _maybe_snapshot(self):
        with self._lock:
            snap_index = self.core.storage.snapshot_meta()[0]
            applied = self.applied_index
            if applied - snap_index < self.snapshot_every or applied > self.core.last_applied:
                return
        data = self.sm.snapshot()
        with self._lock:
            if applied > self.core.storage.snapshot_meta()[0]:
                self.core.compact(applied, data)

    # ------------------------------------------------------------------ client API
    def submit(self, command: str) -> Future:
        with self._lock:
            idx = self.core.propose(command, self._now())  # raises NotLeader
            fut: Future = Future()
            self._waiters[idx] = (self.core.current_term, fut)
            out = self.core.flush(self._now())
            self._collect()
        self._dispatch(out)
        return fut

    def propose(self, command: str, timeout: float = 5.0):
        """Replicate ``command`` and return the state machine's apply result once committed."""
        return self.submit(command).result(timeout=timeout)

    def wait_applied(self, index: int, timeout: float = 5.0) -> bool:
        end = time.monotonic() + timeout
        with self._applied_cv:
            while self.applied_index < index:
                rem = end - time.monotonic()
                if rem <= 0:
                    return False
                self._applied_cv.wait(rem)
        return True

    def read_ready(self) -> bool:
        """Non-blocking ``read_barrier``: True when this node leads and has already applied
        everything committed up to the first entry of its own term (local reads are fenced)."""
        with self._lock:
            if self.core.role != LEADER:
                return False
            target = self.core.commit_index
            if self.core.storage.term_at(target) != self.core.current_term:
                return False
        return self.applied_index >= target

    def read_barrier(self, timeout: float = 5.0) -> bool:
        """Leader-side read fence: wait until this leader has applied everything committed up to
        the first entry of its own term (so local reads reflect every acknowledged write)."""
        end = time.monotonic() + timeout
        while True:
            with self._lock:
                if self.core.role != LEADER:
                    return False
                target = self.core.commit_index
                ready = self.core.storage.term_at(target) == self.core.current_term
            if ready:
                return self.wait_applied(target, max(0.0, end - time.monotonic()))
            if time.monotonic() >= end:
                return False
            time.sleep(0.002)

    # ------------------------------------------------------------------ introspection
    @property
    def leader_id(self) -> int | None:
        with self._lock:
            return self.core.leader_id

    @property
    def is_leader(self) -> bool:
        with self._lock:
            return self.core.role == LEADER

    def status(self) -> dict:
        with self._lock:
            st = self.core.status()
        st["applied_index"] = self.applied_index
        return st
