"""gRPC transport for Raft: the control plane stays on the reference's ``RaftService`` RPCs.

Core messages map onto ``lms.proto``:

==================  ================================================================================
VoteRequest         RequestVoteRequest{candidate: TermCandIDPair{term, candidateID}, lastLogIndex,
                    lastLogTerm}
VoteResponse        RequestVoteResponse{result: TermResultPair{term, verdict}}
AppendRequest       AppendEntriesRequest{leader: TermLeaderIDPair{leaderID, term}, prevLogIndex,
                    prevLogTerm, entries: [LogEntry{term, command}], leaderCommit}
AppendResponse      AppendEntriesResponse{result: {term, verdict}, success, term}: ``result.term`` is
                    the responder's current term; the spare ``term`` field (the reference never
                    fills it) carries the match index on success / the back-off hint on failure
==================  ================================================================================

InstallSnapshot has no RPC in ``lms.proto`` (which stays byte-for-byte), so it is served on an
internal generic client-streaming method ``/lmsinternal.Raft/InstallSnapshotStream``: a JSON header
then the snapshot in 1 MiB pieces (the unary ``InstallSnapshot`` of round 1 is still served).

Differences from the reference's call pattern (``lms_server.py:442-650``): one persistent channel
per peer instead of a new channel per RPC, deadlines on every RPC, and a per-peer sender thread
with a BOUNDED, coalescing mailbox -- at most one pending message per kind (vote, append,
snapshot); a newer AppendEntries replaces an unsent older one (the core re-sends from its own
next_index after ``rpc_timeout`` anyway), so a stalled follower can never grow a queue of stale
RPCs that replays when it resumes.
"""
from __future__ import annotations

import json
import logging
import threading

import grpc

from .. import wire
from ..wire import pb
from .core import (AppendRequest, AppendResponse, Entry, SnapshotRequest, SnapshotResponse, VoteRequest,
                   VoteResponse)

log = logging.getLogger("dlms.raft.transport")

SNAPSHOT_METHOD = "/lmsinternal.Raft/InstallSnapshot"
SNAPSHOT_STREAM_METHOD = "/lmsinternal.Raft/InstallSnapshotStream"
SNAPSHOT_CHUNK = 1 << 20


def to_proto(m):
    if isinstance(m, VoteRequest):
        return pb.RequestVoteRequest(candidate=pb.TermCandIDPair(term=m.term, candidateID=m.src),
                                     lastLogIndex=m.last_log_index, lastLogTerm=m.last_log_term)
    if isinstance(m, VoteResponse):
        return pb.RequestVoteResponse(result=pb.TermResultPair(term=m.term, verdict=m.granted))
    if isinstance(m, AppendRequest):
        return pb.AppendEntriesRequest(leader=pb.TermLeaderIDPair(leaderID=m.src, term=m.term),
                                       prevLogIndex=m.prev_index, prevLogTerm=m.prev_term,
                                       entries=[pb.LogEntry(term=e.term, command=e.command) for e in m.entries],
                                       leaderCommit=m.leader_commit)
    if isinstance(m, AppendResponse):
        return pb.AppendEntriesResponse(result=pb.TermResultPair(term=m.term, verdict=m.success), term=m.index,
                                        success=m.success)
    raise TypeError(type(m))


PREVOTE_HEADER = "x-dlms-prevote"  # lms.proto has no pre-vote flag: it rides in call metadata


def vote_request_from(p, dst: int, pre: bool = False) -> VoteRequest:
    return VoteRequest(p.candidate.candidateID, dst, p.candidate.term, p.lastLogIndex, p.lastLogTerm, pre=pre)


def append_request_from(p, dst: int) -> AppendRequest:
    return AppendRequest(p.leader.leaderID, dst, p.leader.term, p.prevLogIndex, p.prevLogTerm,
                         [Entry(e.term, e.command) for e in p.entries], p.leaderCommit)


class _Mailbox:
    """Per-peer pending sends: one slot per message kind, newest wins."""

    KINDS = (VoteRequest, SnapshotRequest, AppendRequest)

    def __init__(self):
        self.cv = threading.Condition()
        self.slots: dict[type, object] = {}
        self.superseded = 0

    def put(self, m) -> None:
        with self.cv:
            if type(m) in self.slots:
                self.superseded += 1
            self.slots[type(m)] = m
            self.cv.notify()

    def take(self, stop: threading.Event, timeout: float = 0.1):
        with self.cv:
            while not self.slots:
                if stop.is_set():
                    return None
                self.cv.wait(timeout)
            for k in self.KINDS:  # votes first: an election must not wait behind a big append
                if k in self.slots:
                    return self.slots.pop(k)
            return self.slots.popitem()[1]

    def __len__(self):
        with self.cv:
            return len(self.slots)


class GrpcTransport:
    def __init__(self, self_id: int, peers: dict[int, str], rpc_timeout: float = 0.5,
                 snapshot_timeout: float = 30.0):
        self.id = self_id
        self.node = None
        self.rpc_timeout = rpc_timeout
        self.snapshot_timeout = snapshot_timeout
        # fast reconnect: a restarted peer must hear heartbeats well within an election timeout
        # (gRPC's default reconnect backoff grows to 120 s)
        self._channels = {pid: wire.channel(addr, reconnect_ms=(50, 500)) for pid, addr in peers.items()}
        self._stubs = {pid: wire.Stub("RaftService", ch) for pid, ch in self._channels.items()}
        self._snap = {pid: ch.stream_unary(SNAPSHOT_STREAM_METHOD) for pid, ch in self._channels.items()}
        self._boxes = {pid: _Mailbox() for pid in peers}
        self._stop = threading.Event()
        self._threads = []
        for pid in peers:
            t = threading.Thread(target=self._sender, args=(pid,), name=f"raft-send-{pid}", daemon=True)
            t.start()
            self._threads.append(t)
        self.blocked: set[int] = set()  # fault injection: peers we pretend not to reach
        self.closed = False

    def attach(self, node):
        self.node = node

    def send(self, m):
        if self.closed or m.dst not in self._boxes or m.dst in self.blocked:
            return
        self._boxes[m.dst].put(m)

    def pending(self) -> dict:
        """Per-peer pending sends (bounded by the number of message kinds) and superseded count."""
        return {pid: {"pending": len(b), "superseded": b.superseded} for pid, b in self._boxes.items()}

    def _sender(self, pid: int):
        box = self._boxes[pid]
        while not self._stop.is_set():
            m = box.take(self._stop)
            if m is None:
                return
            self._send_sync(m)

    @staticmethod
    def _snapshot_pieces(m):
        yield json.dumps({"src": m.src, "term": m.term, "last_index": m.last_index, "last_term": m.last_term,
                          "size": len(m.data)}).encode()
        data = m.data.encode()
        for i in range(0, len(data), SNAPSHOT_CHUNK):
            yield data[i:i + SNAPSHOT_CHUNK]

    def _send_sync(self, m):
        try:
            if isinstance(m, VoteRequest):
                md = ((PREVOTE_HEADER, "1"),) if m.pre else None
                r = self._stubs[m.dst].RequestVote(to_proto(m), timeout=self.rpc_timeout, metadata=md)
                resp = VoteResponse(m.dst, self.id, r.result.term, r.result.verdict, pre=m.pre)
            elif isinstance(m, AppendRequest):
                r = self._stubs[m.dst].AppendEntries(to_proto(m), timeout=self.rpc_timeout)
                resp = AppendResponse(m.dst, self.id, r.result.term, r.result.verdict, r.term)
            elif isinstance(m, SnapshotRequest):
                r = json.loads(self._snap[m.dst](self._snapshot_pieces(m), timeout=self.snapshot_timeout))
                resp = SnapshotResponse(m.dst, self.id, r["term"], r["last_index"])
            else:
                return
        except grpc.RpcError:
            return  # the core's in-flight timeout retries
        except Exception:
            log.exception("raft send to %s failed", m.dst)
            return
        if self.node is not None and not self.closed and m.dst not in self.blocked:
            self.node.deliver(resp)

    def close(self):
        self.closed = True
        self._stop.set()
        for b in self._boxes.values():
            with b.cv:
                b.cv.notify_all()
        for ch in self._channels.values():
            ch.close()


class RaftServicer:
    """Server side of ``lms.RaftService`` (registered through ``wire.register``)."""

    def __init__(self, node, address_of=None, blocked=None):
        self.node = node
        self.address_of = address_of or {}
        self.blocked = blocked if blocked is not None else set()

    def _check(self, src, context):
        if src in self.blocked:
            context.abort(grpc.StatusCode.UNAVAILABLE, "partitioned (fault injection)")

    def RequestVote(self, request, context):
        self._check(request.candidate.candidateID, context)
        pre = dict(context.invocation_metadata() or ()).get(PREVOTE_HEADER) == "1"
        r = self.node.handle(vote_request_from(request, self.node.id, pre=pre))
        return to_proto(r)

    def AppendEntries(self, request, context):
        self._check(request.leader.leaderID, context)
        r = self.node.handle(append_request_from(request, self.node.id))
        return to_proto(r)

    def WhoIsLeader(self, request, context):
        lid = self.node.leader_id
        return pb.LeaderResponse(leader_id=lid if lid is not None else -1)

    def GetLeader(self, request, context):
        lid = self.node.leader_id
        if lid is None:
            return pb.GetLeaderResponse(nodeId=-1, nodeAddress="")
        return pb.GetLeaderResponse(nodeId=lid, nodeAddress=self.address_of.get(lid, ""))

    def SetVal(self, request, context):
        from ..lms import commands

        try:
            self.node.propose(commands.encode("SetVal", [request.key, request.value]))
            return pb.SetValResponse(verdict=True)
        except Exception:
            return pb.SetValResponse(verdict=False)

    def GetVal(self, request, context):
        kv = getattr(self.node.sm, "kv", {})
        if request.key in kv:
            return pb.GetValResponse(verdict=True, value=kv[request.key])
        return pb.GetValResponse(verdict=False, value="")


def snapshot_handler(node):
    def install(body: bytes, context) -> bytes:
        obj = json.loads(body)
        r = node.handle(SnapshotRequest(obj["src"], node.id, obj["term"], obj["last_index"], obj["last_term"],
                                        obj["data"]))
        return json.dumps({"term": r.term, "last_index": r.last_index}).encode()

    def install_stream(pieces, context) -> bytes:
        it = iter(pieces)
        hdr = json.loads(next(it))
        data = b"".join(it)
        if len(data) != hdr["size"]:
            context.abort(grpc.StatusCode.DATA_LOSS, "truncated snapshot stream")
        r = node.handle(SnapshotRequest(hdr["src"], node.id, hdr["term"], hdr["last_index"], hdr["last_term"],
                                        data.decode()))
        return json.dumps({"term": r.term, "last_index": r.last_index}).encode()

    return grpc.method_handlers_generic_handler("lmsinternal.Raft", {
        "InstallSnapshot": grpc.unary_unary_rpc_method_handler(install),
        "InstallSnapshotStream": grpc.stream_unary_rpc_method_handler(install_stream)})
