#!/usr/bin/env python3
"""Control-plane benchmark: a real N-node LMS cluster (one OS process per server, gRPC on
localhost) measuring the numbers the survey measured on the reference:

* cold start -> stable leader                     (reference: 91 s)
* leader SIGKILL -> new leader                    (reference: 102 s)
* exactly-quorum liveness (kill down to N//2+1)   (reference: no leader within 100 s)
* write latency (Register acknowledged after commit) p50/p99, and writes/s from C client threads

Prints one JSON line.  Usage: python scripts/bench_raft.py [--nodes 5] [--writes 200]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import grpc  # noqa: E402

from distributed_lms_raft_llm_amd import wire  # noqa: E402
from distributed_lms_raft_llm_amd.wire import pb  # noqa: E402


def free_ports(n):
    socks = [socket.socket() for _ in range(n)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def who(addr):
    try:
        with grpc.insecure_channel(addr) as ch:
            return wire.Stub("RaftService", ch).WhoIsLeader(pb.Empty(), timeout=0.3).leader_id
    except grpc.RpcError:
        return None


def wait_leader(addrs, alive, timeout=120.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        seen = {who(addrs[i]) for i in alive}
        seen.discard(None)
        seen.discard(-1)
        if len(seen) == 1:
            lid = seen.pop()
            if lid in alive:
                return lid, time.time() - t0
        time.sleep(0.01)
    return None, timeout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=5)
    ap.add_argument("--writes", type=int, default=200)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--fsync", action="store_true")
    args = ap.parse_args()
    n = args.nodes
    ports = free_ports(n)
    addrs = {i + 1: f"127.0.0.1:{p}" for i, p in enumerate(ports)}
    tmp = tempfile.mkdtemp(prefix="raftbench")
    procs = {}
    env = dict(os.environ, PYTHONPATH=ROOT)

    def start(i):
        peers = [addrs[j] for j in sorted(addrs) if j != i]
        cmd = [sys.executable, os.path.join(ROOT, "lms_server.py"), str(i), str(ports[i - 1]), *peers,
               "--host", "127.0.0.1", "--advertise", addrs[i], "--data-dir", os.path.join(tmp, f"n{i}"),
               "--tutor", "", "--gate", "off", "--log-level", "WARNING"]
        if not args.fsync:
            cmd.append("--no-fsync")
        procs[i] = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)

    res = {"nodes": n}
    try:
        t0 = time.time()
        for i in addrs:
            start(i)
        lid, _ = wait_leader(addrs, set(addrs))
        res["cold_start_to_leader_s"] = round(time.time() - t0, 3)  # includes Python/gRPC process start-up
        # write latency
        stub = wire.Stub("LMS", wire.channel(addrs[lid]))
        lat = []
        for k in range(args.writes):
            ts = time.perf_counter()
            r = stub.Register(pb.RegisterRequest(username=f"u{k}", password="p", role="student"), timeout=10)
            lat.append((time.perf_counter() - ts) * 1e3)
            assert r.success
        res["write_ms_p50"] = round(statistics.median(lat), 3)
        res["write_ms_p99"] = round(sorted(lat)[int(0.99 * (len(lat) - 1))], 3)
        # throughput with concurrent clients
        count = [0]
        stop = time.time() + 3.0

        def client(c):
            st = wire.Stub("LMS", wire.channel(addrs[lid]))
            k = 0
            while time.time() < stop:
                st.Register(pb.RegisterRequest(username=f"c{c}_{k}", password="p", role="student"), timeout=10)
                k += 1
            count[0] += k

        ts = [threading.Thread(target=client, args=(c,)) for c in range(args.clients)]
        t1 = time.time()
        [t.start() for t in ts]
        [t.join() for t in ts]
        res["writes_per_s"] = round(count[0] / (time.time() - t1), 1)
        # failover: SIGKILL the leader
        alive = set(addrs)
        procs[lid].send_signal(signal.SIGKILL)
        procs[lid].wait()
        alive.discard(lid)
        tk = time.time()
        new, _ = wait_leader(addrs, alive, timeout=60)
        res["failover_s"] = round(time.time() - tk, 3)
        # exactly quorum
        while len(alive) > n // 2 + 1:
            victim = new if new in alive else next(iter(alive))
            procs[victim].send_signal(signal.SIGKILL)
            procs[victim].wait()
            alive.discard(victim)
        tq = time.time()
        new, _ = wait_leader(addrs, alive, timeout=60)
        res["quorum_only_leader_s"] = round(time.time() - tq, 3) if new else None
        if new:
            st = wire.Stub("LMS", wire.channel(addrs[new]))
            ok = st.Register(pb.RegisterRequest(username="after_quorum", password="p", role="student"), timeout=10)
            res["quorum_only_write_ok"] = bool(ok.success)
        res["reference"] = {"cold_start_to_leader_s": 91, "failover_s": 102, "quorum_only_leader_s": None}
        print(json.dumps(res), flush=True)
    finally:
        for p in procs.values():
            if p.poll() is None:
                p.kill()
                p.wait()


if __name__ == "__main__":
    main()
