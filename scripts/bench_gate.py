#!/usr/bin/env python3
"""Relevance gate under concurrency: ``--clients`` concurrent ``GetLLMAnswer``
calls through a real single-node LMS gRPC server whose gate is the HIP BERT encoder
(bert-base-uncased, random init -- no checkpoint on this box), against an assignment text that
fills the 512-token window.  Reports p50/p99 per-call latency and gate passes per mode as JSON lines:

* ``batched``   -- the gate's batcher packs concurrent queries into one varlen encoder pass;
* ``serial``    -- ``max_batch=1``: one encoder pass per query (what a per-request gate does).

Clients run in ``--client-procs`` separate processes (100 threads in the server's own interpreter
would compete with it for the GIL); ``--tutor echo`` isolates the LMS + gate path (the tutoring call is an in-process echo);
``--tutor gpt2`` runs the real continuous-batching GPT-2 tutoring server on the same GPU.
The reference's gate re-loads BERT from disk per query (~563 ms) on CPU.
"""
import argparse
import json
import os
import random
import statistics
import sys
import tempfile
import threading
import time
from concurrent import futures

import grpc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_lms_raft_llm_amd import wire  # noqa: E402
from distributed_lms_raft_llm_amd.lms.pdf import make_pdf  # noqa: E402
from distributed_lms_raft_llm_amd.lms.server import LMSServer  # noqa: E402
from distributed_lms_raft_llm_amd.raft.core import RaftConfig  # noqa: E402
from distributed_lms_raft_llm_amd.wire import pb  # noqa: E402

WORDS = ("raft leader election term vote log replication commit index follower candidate heartbeat "
         "snapshot quorum majority state machine consensus partition timeout append entries").split()


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


class EchoTutor:
    def GetLLMAnswer(self, request, context):
        return pb.QueryResponse(success=True, response=f"Question: {request.query}\nAnswer: synthetic")


def _client_proc(conn):
    """Client worker process (spawned before the parent touches the GPU): on each request
    (addr, [(token, query)]) fire all calls at once from threads, reply with latencies (ms)."""
    import grpc as _grpc  # noqa: F401  (fresh interpreter: import here)

    from distributed_lms_raft_llm_amd import wire as _wire
    from distributed_lms_raft_llm_amd.wire import pb as _pb

    stub = None
    while True:
        msg = conn.recv()
        if msg is None:
            return
        addr, calls = msg
        if stub is None:
            stub = _wire.Stub("LMS", _wire.channel(addr))
        lat = [0.0] * len(calls)
        barrier = threading.Barrier(len(calls))

        def one(i):
            barrier.wait()
            t = time.perf_counter()
            r = stub.GetLLMAnswer(_pb.QueryRequest(token=calls[i][0], query=calls[i][1]), timeout=120)
            lat[i] = (time.perf_counter() - t) * 1e3 if (r.success and r.response) else -1.0

        ths = [threading.Thread(target=one, args=(i,)) for i in range(len(calls))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        conn.send(lat)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5, help="bursts of --clients concurrent calls per mode")
    ap.add_argument("--modes", default="batched,serial")
    ap.add_argument("--tutor", choices=["echo", "gpt2"], default="echo")
    ap.add_argument("--gate-model", default="bert-base-uncased")
    ap.add_argument("--window-ms", type=float, default=1.0)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--device", default="cuda", help="'cpu' = torch reference encoder (dry run)")
    ap.add_argument("--client-procs", type=int, default=4,
                    help="client processes (0 = client threads inside the server process)")
    args = ap.parse_args()

    # client processes first: spawned before this process initialises the GPU
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    clients = []
    for _ in range(args.client_procs):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_client_proc, args=(b,), daemon=True)
        p.start()
        clients.append((p, a))

    import torch

    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    gate = RelevanceGate.create(args.gate_model, device=args.device, threshold=0.0)  # admit all: tutor path runs
    tutor_srv = grpc.server(futures.ThreadPoolExecutor(max_workers=args.clients + 8))
    if args.tutor == "echo":
        wire.register(tutor_srv, "Tutoring", EchoTutor())
        tport = tutor_srv.add_insecure_port("127.0.0.1:0")
        tutor_srv.start()
        tserver = None
    else:
        from distributed_lms_raft_llm_amd.tutor.server import TutoringServer, make_engine

        eng = make_engine("gpt2", "cuda", max_batch=256, max_length=150)
        tserver = TutoringServer(eng, port=0, host="127.0.0.1", workers=args.clients + 8).start()
        tport = tserver.port
    tmp = tempfile.mkdtemp(prefix="bench_gate_")
    srv = LMSServer(1, 0, {}, tmp, host="127.0.0.1", tutor_address=f"127.0.0.1:{tport}", gate=gate,
                    raft_config=RaftConfig(), fsync=False, workers=args.clients + 16).start()
    addr = f"127.0.0.1:{srv.port}"
    stub = wire.Stub("LMS", wire.channel(addr))
    end = time.time() + 20
    while not srv.node.is_leader and time.time() < end:
        time.sleep(0.05)
    rng = random.Random(0)
    text = " ".join(rng.choice(WORDS) for _ in range(700))  # > 512 WordPiece tokens: truncated
    tokens = []
    for k in range(args.clients):
        u = f"s{k}"
        assert stub.Register(pb.RegisterRequest(username=u, password="pw", role="student"), timeout=10).success
        tok = stub.Login(pb.LoginRequest(username=u, password="pw"), timeout=10).token
        assert stub.Post(pb.PostRequest(token=tok, type="assignment", file=make_pdf(text), filename=f"a{k}.pdf"),
                         timeout=30).success
        tokens.append(tok)
    gate.warm(srv.state.read(lambda d: d["assignments"]["s0"][0]["text"]))
    queries = [" ".join(rng.choice(WORDS) for _ in range(rng.randint(4, 40))) for _ in range(args.clients)]

    def burst():
        if clients:  # fan the calls out over the client processes, all at once
            shares = [[(tokens[i], queries[i]) for i in range(k, args.clients, len(clients))]
                      for k in range(len(clients))]
            for (_, conn), calls in zip(clients, shares):
                conn.send((addr, calls))
            lat = [x for _, conn in clients for x in conn.recv()]
            assert min(lat) >= 0, "a call failed"
            return lat
        lat = [0.0] * args.clients
        barrier = threading.Barrier(args.clients)

        def one(i):
            barrier.wait()
            t = time.perf_counter()
            r = stub.GetLLMAnswer(pb.QueryRequest(token=tokens[i], query=queries[i]), timeout=120)
            lat[i] = (time.perf_counter() - t) * 1e3
            assert r.success and r.response, r

        ths = [threading.Thread(target=one, args=(i,)) for i in range(args.clients)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        return lat

    for mode in args.modes.split(","):
        gate.max_batch = args.max_batch if mode == "batched" else 1
        gate.window_s = args.window_ms / 1e3 if mode == "batched" else 0.0
        burst()  # warm-up (JIT'd buffers, gRPC channels)
        p0, q0 = gate.passes, gate.batched_queries
        lat = []
        t0 = time.perf_counter()
        for _ in range(args.rounds):
            lat += burst()
        wall = time.perf_counter() - t0
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        print(json.dumps({"bench": "gate_concurrency", "mode": mode, "tutor": args.tutor, "clients": args.clients,
                          "client_procs": args.client_procs,
                          "rounds": args.rounds, "gate_model": args.gate_model,
                          "p50_ms": round(statistics.median(lat), 2), "p99_ms": round(pct(lat, 0.99), 2),
                          "max_ms": round(max(lat), 2), "calls_per_s": round(len(lat) / wall, 1),
                          "gate_passes": gate.passes - p0,
                          "queries_per_pass": round((gate.batched_queries - q0) / max(1, gate.passes - p0), 2)}),
              flush=True)
    for _, conn in clients:
        conn.send(None)
    srv.stop(grace=0)
    if tserver is not None:
        tserver.stop()
    tutor_srv.stop(0)


if __name__ == "__main__":
    main()
