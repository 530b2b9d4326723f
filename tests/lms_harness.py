"""Helpers for in-process LMS clusters on localhost (real gRPC, real Raft nodes)."""
from __future__ import annotations

import socket
import time
from concurrent import futures

import grpc

from distributed_lms_raft_llm_amd import wire
from distributed_lms_raft_llm_amd.lms.server import LMSServer
from distributed_lms_raft_llm_amd.raft.core import RaftConfig
from distributed_lms_raft_llm_amd.wire import pb


def free_ports(n: int) -> list[int]:
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


class EchoTutor:
    """Stand-in tutoring service: echoes the prompt template like GPT-2's generate() does."""

    def __init__(self):
        self.calls = []

    def GetLLMAnswer(self, request, context):
        self.calls.append(request.query)
        return pb.QueryResponse(success=True, response=f"Question: {request.query}\nAnswer: synthetic")


def start_tutor(servicer=None):
    servicer = servicer or EchoTutor()
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
    wire.register(srv, "Tutoring", servicer)
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    return srv, port, servicer


class SyncKeywordGate:
    """Deterministic gate for service tests: relevant iff the query shares a word with the text.
    (No ``check_async``: GetLLMAnswer runs the worker-pool prelude.)"""

    def check(self, query: str, text: str):
        q = set(query.lower().split())
        t = set(text.lower().split())
        sim = len(q & t) / max(1, len(q))
        return sim > 0, sim


class KeywordGate(SyncKeywordGate):
    """The same gate with the aio front end's thread-free path (service.py ``_llm_prelude_fast``)."""

    def __init__(self):
        self.async_calls = 0

    async def check_async(self, query: str, text: str):
        self.async_calls += 1
        return self.check(query, text)


class Cluster:
    def __init__(self, n: int, tmp_path, tutor_address=None, gate=None, fsync=False, snapshot_every: int = 2000,
                 raft_config: RaftConfig | None = None):
        self.raft_config = raft_config
        self.ports = free_ports(n)
        self.addrs = {i + 1: f"127.0.0.1:{p}" for i, p in enumerate(self.ports)}
        self.tmp = tmp_path
        self.tutor_address = tutor_address
        self.gate = gate
        self.fsync = fsync
        self.snapshot_every = snapshot_every
        self.servers: dict[int, LMSServer] = {}
        for i in self.addrs:
            self.start(i)

    def start(self, i: int):
        peers = {j: a for j, a in self.addrs.items() if j != i}
        srv = LMSServer(i, self.ports[i - 1], peers, str(self.tmp / f"node{i}"), host="127.0.0.1",
                        advertise=self.addrs[i], tutor_address=self.tutor_address, gate=self.gate,
                        raft_config=self.raft_config or RaftConfig(), fsync=self.fsync, workers=16,
                        snapshot_every=self.snapshot_every)
        self.servers[i] = srv.start()
        return srv

    def stop(self, i: int):
        srv = self.servers.pop(i, None)
        if srv is not None:
            srv.stop(grace=0)

    def close(self):
        for i in list(self.servers):
            self.stop(i)

    def who_is_leader(self, i: int, timeout=1.0) -> int:
        with grpc.insecure_channel(self.addrs[i]) as ch:
            return wire.Stub("RaftService", ch).WhoIsLeader(pb.Empty(), timeout=timeout).leader_id

    def wait_leader(self, timeout: float = 10.0) -> int:
        end = time.time() + timeout
        while time.time() < end:
            ids = set()
            for i in self.servers:
                try:
                    ids.add(self.who_is_leader(i))
                except grpc.RpcError:
                    pass
            ids.discard(-1)
            if len(ids) == 1:
                lid = ids.pop()
                if lid in self.servers and self.servers[lid].node.is_leader:
                    return lid
            time.sleep(0.05)
        raise TimeoutError("no leader")

    def stub(self, i: int):
        return wire.Stub("LMS", wire.channel(self.addrs[i]))
