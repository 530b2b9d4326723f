"""Pure Raft consensus core: a deterministic state machine with no I/O, no threads, no clock.

The reference's consensus (``lms_server.py:123-697``, driver ``:1531-1556``) is a hand-rolled,
lock-free Raft with positional peer ids, off-by-one log indices, commits that never reach the
followers on heartbeats, no persistence and writes that crash on followers.
This core re-designs it as textbook Raft:

* 1-based log indices, ``commit_index`` 0 = nothing committed; only current-term entries are
  committed by counting replicas (Raft §5.4.2), with a no-op entry at the start of each term;
* persistent ``current_term`` / ``voted_for`` / log through a ``Storage`` (``raft/storage.py``);
* randomized election timeouts, heartbeats that carry ``leader_commit``;
* one in-flight AppendEntries per follower with fast log back-off (the follower's hint);
* check-quorum: a leader that has not heard from a majority for an election timeout steps
  down, so ``WhoIsLeader`` never points clients at a partitioned ex-leader for long;
* snapshots (log compaction) and InstallSnapshot for followers behind the snapshot.

Callers feed it events -- ``tick(now)``, ``step(msg, now)``, ``propose(cmd, now)`` -- and get
back the messages to send; committed entries are drained with ``take_committed()``.  The same
object runs under the gRPC node (``raft/node.py``) and under the deterministic simulator used by
the tests (``raft/sim.py``).
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field

FOLLOWER, CANDIDATE, LEADER = "follower", "candidate", "leader"

NOOP_COMMAND = '{"operation": "NoOp", "args": []}'


@dataclass
class Entry:
    term: int
    command: str


@dataclass
class VoteRequest:
    src: int
    dst: int
    term: int
    last_log_index: int
    last_log_term: int
    pre: bool = False  # Pre-Vote probe (Raft thesis §9.6): ``term`` is the term it WOULD start


@dataclass
class VoteResponse:
    src: int
    dst: int
    term: int  # pre-vote granted: the probed term; otherwise the responder's current term
    granted: bool
    pre: bool = False


@dataclass
class AppendRequest:
    src: int
    dst: int
    term: int
    prev_index: int
    prev_term: int
    entries: list[Entry]
    leader_commit: int


@dataclass
class AppendResponse:
    src: int
    dst: int
    term: int
    success: bool
    # success: index of the last entry now known to match the leader's log
    # failure: follower's hint -- the leader retries from hint + 1
    index: int


@dataclass
class SnapshotRequest:
    src: int
    dst: int
    term: int
    last_index: int
    last_term: int
    data: str


@dataclass
class SnapshotResponse:
    src: int
    dst: int
    term: int
    last_index: int


REQUESTS = (VoteRequest, AppendRequest, SnapshotRequest)


class NotLeader(Exception):
    def __init__(self, leader_id: int | None):
        super().__init__(f"not the leader (leader={leader_id})")
        self.leader_id = leader_id


@dataclass
class RaftConfig:
    election_timeout: tuple[float, float] = (0.15, 0.30)
    heartbeat_interval: float = 0.05
    rpc_timeout: float = 0.1  # < min election timeout: a lost AppendEntries is retried before followers time out
    max_entries_per_append: int = 256
    max_bytes_per_append: int = 8 << 20
    check_quorum: bool = True
    # Pre-Vote + leader stickiness: a node that was partitioned or restarted (and whose election
    # timer fired) first asks whether it COULD win; nodes that heard from a live leader within
    # the minimum election timeout refuse, so it cannot force a term bump on a healthy cluster.
    pre_vote: bool = True


@dataclass
class _Peer:
    next_index: int = 1
    match_index: int = 0
    inflight: bool = False
    sent_at: float = -1e9
    last_ack: float = -1e9
    snapshot_inflight: bool = False


@dataclass
class Stats:
    elections_started: int = 0
    terms_led: int = 0
    appends_sent: int = 0
    entries_sent: int = 0
    snapshots_sent: int = 0
    commits: int = 0
    step_downs: int = 0
    events: list = field(default_factory=list)


class RaftCore:
    def __init__(self, node_id: int, peer_ids: list[int], storage, config: RaftConfig | None = None,
                 rng: random.Random | None = None, now: float = 0.0):
        if node_id in peer_ids:
            raise ValueError("peer_ids must not contain node_id")
        self.id = node_id
        self.peers = {p: _Peer() for p in sorted(peer_ids)}
        self.storage = storage
        self.cfg = config or RaftConfig()
        self.rng = rng or random.Random(node_id * 7919)
        self.current_term, self.voted_for = storage.load_meta()
        self.role = FOLLOWER
        self.leader_id: int | None = None
        snap_index, _ = storage.snapshot_meta()
        self.commit_index = snap_index
        self.last_applied = snap_index
        self.votes: set[int] = set()
        self.prevotes: set[int] | None = None  # collecting pre-votes (role stays FOLLOWER)
        self._leader_contact = -1e9  # last time a current leader reached us
        self.pending_restore: str | None = None  # snapshot data the state machine must load
        self.stats = Stats()
        self._deadline = 0.0
        self._reset_election_timer(now)

    # ------------------------------------------------------------------ helpers
    @property
    def cluster_size(self) -> int:
        return len(self.peers) + 1

    @property
    def quorum(self) -> int:
        return self.cluster_size // 2 + 1

    def last_index(self) -> int:
        return self.storage.last_index()

    def last_term(self) -> int:
        return self.storage.term_at(self.storage.last_index())

    def _reset_election_timer(self, now: float):
        lo, hi = self.cfg.election_timeout
        self._deadline = now + self.rng.uniform(lo, hi)

    def _event(self, kind: str, **kw):
        ev = {"node": self.id, "event": kind, "term": self.current_term, **kw}
        self.stats.events.append(ev)
        if len(self.stats.events) > 1000:
            del self.stats.events[:500]

    def _set_term(self, term: int, voted_for: int | None):
        self.current_term, self.voted_for = term, voted_for
        self.storage.save_meta(term, voted_for)

    def _become_follower(self, term: int, now: float, leader: int | None = None):
        was_leader = self.role == LEADER
        if term > self.current_term:
            self._set_term(term, None)
        if self.role != FOLLOWER:
            self._event("step_down" if was_leader else "follower")
            if was_leader:
                self.stats.step_downs += 1
        self.role = FOLLOWER
        self.leader_id = leader
        self.votes.clear()
        self.prevotes = None
        self._reset_election_timer(now)

    # ------------------------------------------------------------------ timers
    def tick(self, now: float) -> list:
        out: list = []
        if self.role == LEADER:
            if self.cfg.check_quorum and not self._quorum_recent(now):
                self._event("lost_quorum")
                self._become_follower(self.current_term, now)
                return out
            for pid, p in self.peers.items():
                if p.inflight and now - p.sent_at > self.cfg.rpc_timeout:
                    p.inflight = False
                    p.snapshot_inflight = False
                if not p.inflight and (now - p.sent_at >= self.cfg.heartbeat_interval
                                       or p.next_index <= self.last_index()):
                    out.extend(self._replicate_to(pid, now))
        elif now >= self._deadline:
            if self.cfg.pre_vote and self.role == FOLLOWER:
                out.extend(self._start_pre_vote(now))
            else:
                out.extend(self._start_election(now))
        return out

    def _start_pre_vote(self, now: float) -> list:
        self.prevotes = {self.id}
        self.leader_id = None
        self._event("pre_vote")
        self._reset_election_timer(now)
        if len(self.prevotes) >= self.quorum:
            return self._start_election(now)
        li, lt = self.last_index(), self.last_term()
        return [VoteRequest(self.id, pid, self.current_term + 1, li, lt, pre=True) for pid in self.peers]

    def _in_leader_lease(self, now: float) -> bool:
        return self.role == LEADER or now - self._leader_contact < self.cfg.election_timeout[0]

    def _quorum_recent(self, now: float) -> bool:
        window = self.cfg.election_timeout[1]
        alive = 1 + sum(1 for p in self.peers.values() if now - p.last_ack <= window)
        return alive >= self.quorum

    def _start_election(self, now: float) -> list:
        self.prevotes = None
        self.role = CANDIDATE
        self._set_term(self.current_term + 1, self.id)
        self.leader_id = None
        self.votes = {self.id}
        self.stats.elections_started += 1
        self._event("election")
        self._reset_election_timer(now)
        if len(self.votes) >= self.quorum:
            return self._become_leader(now)
        li, lt = self.last_index(), self.last_term()
        return [VoteRequest(self.id, pid, self.current_term, li, lt) for pid in self.peers]

    def _become_leader(self, now: float) -> list:
        self.role = LEADER
        self.leader_id = self.id
        self.stats.terms_led += 1
        self._event("leader")
        nxt = self.last_index() + 1
        for p in self.peers.values():
            p.next_index, p.match_index, p.inflight, p.sent_at = nxt, 0, False, -1e9
            p.last_ack = now  # grace period for check-quorum
            p.snapshot_inflight = False
        # a no-op in the new term lets entries of earlier terms commit (Raft §5.4.2)
        self.storage.append([Entry(self.current_term, NOOP_COMMAND)])
        self._advance_commit()
        out = []
        for pid in self.peers:
            out.extend(self._replicate_to(pid, now))
        return out

    # ------------------------------------------------------------------ client
    def propose(self, command: str, now: float) -> int:
        if self.role != LEADER:
            raise NotLeader(self.leader_id)
        self.storage.append([Entry(self.current_term, command)])
        self._advance_commit()  # single-node cluster commits immediately
        return self.last_index()

    def flush(self, now: float) -> list:
        """Ship freshly proposed entries now instead of waiting for the next tick."""
        out = []
        if self.role == LEADER:
            for pid, p in self.peers.items():
                if not p.inflight:
                    out.extend(self._replicate_to(pid, now))
        return out

    def take_committed(self) -> list[tuple[int, Entry]]:
        if self.commit_index <= self.last_applied:
            return []
        lo = self.last_applied + 1
        ents = self.storage.entries(lo, self.commit_index + 1)
        self.last_applied = self.commit_index
        return list(zip(range(lo, lo + len(ents)), ents))

    # ------------------------------------------------------------------ replication
    def _replicate_to(self, pid: int, now: float) -> list:
        p = self.peers[pid]
        snap_index, snap_term = self.storage.snapshot_meta()
        p.sent_at = now
        p.inflight = True
        if p.next_index <= snap_index:
            p.snapshot_inflight = True
            self.stats.snapshots_sent += 1
            return [SnapshotRequest(self.id, pid, self.current_term, snap_index, snap_term,
                                    self.storage.snapshot_data())]
        prev = p.next_index - 1
        ents = self.storage.entries(p.next_index, p.next_index + self.cfg.max_entries_per_append,
                                    max_bytes=self.cfg.max_bytes_per_append)
        self.stats.appends_sent += 1
        self.stats.entries_sent += len(ents)
        return [AppendRequest(self.id, pid, self.current_term, prev, self.storage.term_at(prev), ents,
                              self.commit_index)]

    def _advance_commit(self):
        if self.role != LEADER:
            return
        matches = sorted([self.last_index()] + [p.match_index for p in self.peers.values()], reverse=True)
        candidate = matches[self.quorum - 1]
        if candidate > self.commit_index and self.storage.term_at(candidate) == self.current_term:
            self.stats.commits += candidate - self.commit_index
            self.commit_index = candidate

    # ------------------------------------------------------------------ message handling
    def step(self, msg, now: float) -> list:
        term = msg.term
        if isinstance(msg, VoteRequest) and msg.pre:
            return [self._on_pre_vote_request(msg, now)]
        if isinstance(msg, VoteResponse) and msg.pre and msg.granted:
            return self._on_pre_vote_response(msg, now)  # carries the probed term: never adopt it
        if isinstance(msg, VoteRequest) and self.cfg.check_quorum and term > self.current_term \
                and self._in_leader_lease(now):
            # leader stickiness: ignore (do not even adopt the term of) a disruptive candidate
            return [VoteResponse(self.id, msg.src, self.current_term, False)]
        if term > self.current_term:
            leader = msg.src if isinstance(msg, (AppendRequest, SnapshotRequest)) else None
            self._become_follower(term, now, leader)
        if isinstance(msg, (AppendRequest, SnapshotRequest)) and term == self.current_term:
            self._leader_contact = now
            self.prevotes = None
        if isinstance(msg, VoteResponse) and msg.pre:
            return []  # refused pre-vote (a higher term was adopted above)
        if isinstance(msg, VoteRequest):
            return [self._on_vote_request(msg, now)]
        if isinstance(msg, VoteResponse):
            return self._on_vote_response(msg, now)
        if isinstance(msg, AppendRequest):
            return [self._on_append(msg, now)]
        if isinstance(msg, AppendResponse):
            return self._on_append_response(msg, now)
        if isinstance(msg, SnapshotRequest):
            return [self._on_snapshot(msg, now)]
        if isinstance(msg, SnapshotResponse):
            return self._on_snapshot_response(msg, now)
        raise TypeError(f"unknown message {type(msg)}")

    def _log_up_to_date(self, last_index: int, last_term: int) -> bool:
        mt = self.last_term()
        return last_term > mt or (last_term == mt and last_index >= self.last_index())

    def _on_vote_request(self, m: VoteRequest, now: float) -> VoteResponse:
        granted = False
        if m.term == self.current_term and self.voted_for in (None, m.src) and self._log_up_to_date(
                m.last_log_index, m.last_log_term) and self.role != LEADER:
            granted = True
            if self.voted_for != m.src:
                self._set_term(self.current_term, m.src)
            self._reset_election_timer(now)
        return VoteResponse(self.id, m.src, self.current_term, granted)

    def _on_pre_vote_request(self, m: VoteRequest, now: float) -> VoteResponse:
        """Grant iff a real vote at ``m.term`` could be granted and no live leader is known.
        Changes no state: no term adoption, no vote recorded, no timer reset."""
        granted = (m.term > self.current_term and not self._in_leader_lease(now)
                   and self._log_up_to_date(m.last_log_index, m.last_log_term))
        return VoteResponse(self.id, m.src, m.term if granted else self.current_term, granted, pre=True)

    def _on_pre_vote_response(self, m: VoteResponse, now: float) -> list:
        if self.prevotes is None or self.role != FOLLOWER or m.term != self.current_term + 1:
            return []
        self.prevotes.add(m.src)
        if len(self.prevotes) >= self.quorum:
            return self._start_election(now)
        return []

    def _on_vote_response(self, m: VoteResponse, now: float) -> list:
        if self.role != CANDIDATE or m.term != self.current_term or not m.granted:
            return []
        self.votes.add(m.src)
        if len(self.votes) >= self.quorum:
            return self._become_leader(now)
        return []

    def _on_append(self, m: AppendRequest, now: float) -> AppendResponse:
        if m.term < self.current_term:
            return AppendResponse(self.id, m.src, self.current_term, False, self.last_index())
        if self.role != FOLLOWER or self.leader_id != m.src:
            self._become_follower(m.term, now, m.src)
        self.leader_id = m.src
        self._reset_election_timer(now)
        snap_index, _ = self.storage.snapshot_meta()
        prev, ents = m.prev_index, list(m.entries)
        if prev < snap_index:
            # the prefix up to our snapshot is committed, hence identical to the leader's: drop it
            skip = snap_index - prev
            if skip >= len(ents):
                return AppendResponse(self.id, m.src, self.current_term, True, snap_index)
            ents = ents[skip:]
            prev = snap_index
        else:
            if prev > self.last_index():
                return AppendResponse(self.id, m.src, self.current_term, False, self.last_index())
            if self.storage.term_at(prev) != m.prev_term:
                # conflicting term at prev: hint the index before that term's first entry here
                bad = self.storage.term_at(prev)
                i = prev
                while i > snap_index + 1 and self.storage.term_at(i - 1) == bad:
                    i -= 1
                return AppendResponse(self.id, m.src, self.current_term, False, max(i - 1, snap_index))
        # append, truncating only on a real conflict (a stale duplicate must not truncate)
        for k, e in enumerate(ents):
            idx = prev + 1 + k
            if idx <= self.last_index():
                if self.storage.term_at(idx) == e.term:
                    continue
                self.storage.truncate_from(idx)
            self.storage.append(ents[k:])
            break
        last_new = prev + len(ents)
        if m.leader_commit > self.commit_index:
            # monotone: a stale / duplicate AppendEntries with a short ``last_new`` must never move
            # the commit index backwards (status(), read fences and a later election read it)
            self.commit_index = max(self.commit_index, min(m.leader_commit, last_new))
        return AppendResponse(self.id, m.src, self.current_term, True, last_new)

    def _on_append_response(self, m: AppendResponse, now: float) -> list:
        if self.role != LEADER or m.term != self.current_term or m.src not in self.peers:
            return []
        p = self.peers[m.src]
        p.inflight = False
        p.last_ack = now
        if m.success:
            if m.index > p.match_index:
                p.match_index = m.index
            p.next_index = max(p.next_index, p.match_index + 1)
            self._advance_commit()
        else:
            p.next_index = max(1, min(p.next_index - 1, m.index + 1))
        if p.next_index <= self.last_index():
            return self._replicate_to(m.src, now)
        return []

    def _on_snapshot(self, m: SnapshotRequest, now: float) -> SnapshotResponse:
        if m.term < self.current_term:
            return SnapshotResponse(self.id, m.src, self.current_term, 0)
        if self.role != FOLLOWER or self.leader_id != m.src:
            self._become_follower(m.term, now, m.src)
        self.leader_id = m.src
        self._reset_election_timer(now)
        snap_index, _ = self.storage.snapshot_meta()
        if m.last_index > snap_index:
            self.storage.install_snapshot(m.last_index, m.last_term, m.data)
            self.commit_index = max(self.commit_index, m.last_index)
            if self.last_applied < m.last_index:
                # the state machine must be replaced by the snapshot before applying further entries
                self.last_applied = m.last_index
                self.pending_restore = m.data
            self._event("snapshot_installed", index=m.last_index)
        return SnapshotResponse(self.id, m.src, self.current_term, m.last_index)

    def _on_snapshot_response(self, m: SnapshotResponse, now: float) -> list:
        if self.role != LEADER or m.term != self.current_term or m.src not in self.peers:
            return []
        p = self.peers[m.src]
        p.inflight = False
        p.snapshot_inflight = False
        p.last_ack = now
        p.match_index = max(p.match_index, m.last_index)
        p.next_index = p.match_index + 1
        self._advance_commit()
        if p.next_index <= self.last_index():
            return self._replicate_to(m.src, now)
        return []

    # ------------------------------------------------------------------ compaction
    def compact(self, upto_index: int, state_data: str):
        """Snapshot the applied state at ``upto_index`` and drop the log prefix."""
        if upto_index > self.last_applied:
            raise ValueError("cannot snapshot beyond last_applied")
        self.storage.compact(upto_index, self.storage.term_at(upto_index), state_data)

    def status(self) -> dict:
        return {"id": self.id, "role": self.role, "term": self.current_term, "leader": self.leader_id,
                "commit_index": self.commit_index, "last_applied": self.last_applied,
                "last_index": self.last_index(), "snapshot_index": self.storage.snapshot_meta()[0]}
