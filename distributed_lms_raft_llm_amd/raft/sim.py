"""Deterministic discrete-event simulator for ``RaftCore`` clusters (the test harness's
FakeTransport): simulated clock, per-message latency, drop probability,
network partitions, crash/restart with durable storage, and the Raft safety invariants.
"""
from __future__ import annotations

import heapq
import random
from dataclasses import dataclass, field

from .core import LEADER, RaftConfig, RaftCore
from .storage import MemoryStorage


@dataclass
class SimNode:
    core: RaftCore | None
    storage: object
    applied: list = field(default_factory=list)  # (index, term, command)
    up: bool = True


class SimCluster:
    def __init__(self, n: int, seed: int = 0, config: RaftConfig | None = None, latency=(0.001, 0.010),
                 drop: float = 0.0, tick: float = 0.01, storage_factory=None):
        self.rng = random.Random(seed)
        self.cfg = config or RaftConfig()
        self.latency = latency
        self.drop = drop
        self.tick_dt = tick
        self.now = 0.0
        self.ids = list(range(1, n + 1))
        self.blocked: set[tuple[int, int]] = set()
        self._q: list = []
        self._seq = 0
        self.storage_factory = storage_factory or (lambda i: MemoryStorage())
        self.nodes: dict[int, SimNode] = {}
        for i in self.ids:
            st = self.storage_factory(i)
            self.nodes[i] = SimNode(self._make_core(i, st), st)
        self.leaders_by_term: dict[int, set[int]] = {}
        self._next_tick = 0.0

    def _make_core(self, i: int, storage) -> RaftCore:
        return RaftCore(i, [p for p in self.ids if p != i], storage, self.cfg,
                        rng=random.Random(self.rng.randrange(1 << 30)), now=self.now)

    # ------------------------------------------------------------------ faults
    def partition(self, *groups):
        """Only nodes inside the same group can talk."""
        self.blocked.clear()
        where = {n: gi for gi, g in enumerate(groups) for n in g}
        for a in self.ids:
            for b in self.ids:
                if a != b and where.get(a, -1) != where.get(b, -2):
                    self.blocked.add((a, b))

    def heal(self):
        self.blocked.clear()

    def crash(self, i: int):
        self.nodes[i].up = False
        self.nodes[i].core = None

    def restart(self, i: int):
        node = self.nodes[i]
        node.core = self._make_core(i, node.storage)
        node.up = True
        # the state machine restarts from the snapshot (if any) and re-applies committed entries
        snap_index, _ = node.storage.snapshot_meta()
        node.applied = [a for a in node.applied if a[0] <= snap_index]

    # ------------------------------------------------------------------ event loop
    def _send(self, msgs):
        for m in msgs:
            if (m.src, m.dst) in self.blocked or self.rng.random() < self.drop:
                continue
            self._seq += 1
            heapq.heappush(self._q, (self.now + self.rng.uniform(*self.latency), self._seq, m))

    def _after(self, i: int):
        node = self.nodes[i]
        core = node.core
        if core.pending_restore is not None:
            idx = core.last_applied
            node.applied = [a for a in node.applied if a[0] <= idx]
            core.pending_restore = None
        for idx, e in core.take_committed():
            node.applied.append((idx, e.term, e.command))
        if core.role == LEADER:
            self.leaders_by_term.setdefault(core.current_term, set()).add(i)

    def run(self, duration: float):
        end = self.now + duration
        while True:
            t_msg = self._q[0][0] if self._q else float("inf")
            t = min(t_msg, self._next_tick)
            if t > end:
                self.now = end
                return
            self.now = t
            if t == self._next_tick:
                self._next_tick += self.tick_dt
                for i, node in self.nodes.items():
                    if node.up:
                        self._send(node.core.tick(self.now))
                        self._after(i)
            else:
                _, _, m = heapq.heappop(self._q)
                dst = self.nodes[m.dst]
                if not dst.up or (m.src, m.dst) in self.blocked:
                    continue
                self._send(dst.core.step(m, self.now))
                self._after(m.dst)

    # ------------------------------------------------------------------ client helpers
    def leader(self) -> int | None:
        best = None
        for i, node in self.nodes.items():
            if node.up and node.core.role == LEADER:
                if best is None or node.core.current_term > self.nodes[best].core.current_term:
                    best = i
        return best

    def wait_leader(self, timeout: float = 5.0) -> int:
        t_end = self.now + timeout
        while self.now < t_end:
            self.run(0.01)
            lid = self.leader()
            if lid is not None:
                return lid
        raise TimeoutError("no leader elected")

    def propose(self, command: str) -> tuple[int, int]:
        lid = self.leader()
        if lid is None:
            raise RuntimeError("no leader")
        core = self.nodes[lid].core
        idx = core.propose(command, self.now)
        self._send(core.flush(self.now))
        self._after(lid)
        return lid, idx

    def committed_on(self, i: int) -> list[str]:
        return [c for _, _, c in self.nodes[i].applied]

    # ------------------------------------------------------------------ invariants
    def check_safety(self):
        # election safety: at most one leader per term
        for term, ls in self.leaders_by_term.items():
            assert len(ls) <= 1, f"two leaders in term {term}: {ls}"
        # state-machine safety: every node applied a prefix of one common sequence
        seqs = [n.applied for n in self.nodes.values()]
        longest = max(seqs, key=len)
        by_index = {a[0]: a for a in longest}
        for s in seqs:
            for a in s:
                if a[0] in by_index:
                    assert by_index[a[0]][1:] == a[1:], f"divergent apply at index {a[0]}: {a} vs {by_index[a[0]]}"
        # log matching between live nodes: same (index, term) => same prefix
        live = [n.core for n in self.nodes.values() if n.up]
        for a in live:
            for b in live:
                if a is b:
                    continue
                hi = min(a.last_index(), b.last_index())
                lo = max(a.storage.snapshot_meta()[0], b.storage.snapshot_meta()[0]) + 1
                for i in range(hi, lo - 1, -1):
                    if a.storage.term_at(i) == b.storage.term_at(i):
                        ea = a.storage.entries(lo, i + 1)
                        eb = b.storage.entries(lo, i + 1)
                        assert [(e.term, e.command) for e in ea] == [(e.term, e.command) for e in eb], \
                            f"log matching violated between {a.id} and {b.id} up to {i}"
                        break
