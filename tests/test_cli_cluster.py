"""Real multi-process cluster through the CLI (SURVEY.md §4.3 "Integration: cluster"): three
``lms_server.py --config cluster.yaml <id>`` processes, writes through the client library, leader
SIGKILL -> re-election and no lost committed write, restart of the killed node from its durable
log/snapshot, and the exactly-quorum case."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import grpc
import pytest
import yaml

from distributed_lms_raft_llm_amd import wire
from distributed_lms_raft_llm_amd.client import LMSClient
from distributed_lms_raft_llm_amd.utils.debug_rpc import debug_call
from distributed_lms_raft_llm_amd.wire import pb

pytestmark = pytest.mark.timeout(180)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


class Proc:
    def __init__(self, tmp, cfg_path, i):
        self.i = i
        self.log = open(tmp / f"node{i}.log", "a")
        env = dict(os.environ, PYTHONPATH=ROOT)
        self.p = subprocess.Popen([sys.executable, os.path.join(ROOT, "lms_server.py"), "--config", str(cfg_path),
                                   str(i)], stdout=self.log, stderr=subprocess.STDOUT, env=env, cwd=str(tmp),
                                  start_new_session=True)

    def kill(self, sig=signal.SIGKILL):
        if self.p.poll() is None:
            os.killpg(self.p.pid, sig)
        self.p.wait(timeout=20)


def _leader(addrs, alive, timeout=15.0):
    end = time.time() + timeout
    while time.time() < end:
        seen = set()
        for i in alive:
            try:
                with grpc.insecure_channel(addrs[i]) as ch:
                    seen.add(wire.Stub("RaftService", ch).WhoIsLeader(pb.Empty(), timeout=0.5).leader_id)
            except grpc.RpcError:
                seen.add(None)
        if len(seen) == 1 and next(iter(seen)) in alive:
            return next(iter(seen))
        time.sleep(0.05)
    raise TimeoutError("no leader")


def test_cli_cluster_failover_and_restart(tmp_path):
    ports = _ports(3)
    addrs = {i + 1: f"127.0.0.1:{p}" for i, p in enumerate(ports)}
    cfg = {"servers": addrs, "host": "127.0.0.1", "gate": "off", "tutor": "", "no_fsync": True,
           "log_level": "WARNING"}
    cfg_path = tmp_path / "cluster.yaml"
    cfg_path.write_text(yaml.safe_dump(cfg))
    for i in addrs:
        (tmp_path / f"d{i}").mkdir()
    procs = {}
    try:
        for i in addrs:
            cfg_i = dict(cfg, data_dir=str(tmp_path / f"d{i}"))
            (tmp_path / f"cluster{i}.yaml").write_text(yaml.safe_dump(cfg_i))
            procs[i] = Proc(tmp_path, tmp_path / f"cluster{i}.yaml", i)
        lid = _leader(addrs, set(addrs), timeout=60)  # first start pays the interpreter/import cost
        cl = LMSClient(list(addrs.values()), timeout=5)
        assert cl.register("alice", "pw", "student").success
        assert cl.register("bob", "pw", "instructor").success
        assert cl.login("alice", "pw")
        assert cl.post_assignment(data=b"raft consensus", filename="a.txt")

        t0 = time.time()
        procs[lid].kill()
        alive = set(addrs) - {lid}
        new = _leader(addrs, alive, timeout=10)
        failover = time.time() - t0
        assert new != lid and failover < 5.0, failover
        # committed writes survived and the replicated session still works on the new leader
        assert cl.grade().startswith(("Grade not yet assigned", "No grade"))
        assert cl.register("carol", "pw", "student").success  # exactly-quorum (2 of 3) still commits

        procs[lid] = Proc(tmp_path, tmp_path / f"cluster{lid}.yaml", lid)  # restart from its data dir
        target = debug_call(addrs[new], "Status")["commit_index"]
        end = time.time() + 60
        st = {}
        while time.time() < end:
            try:
                st = debug_call(addrs[lid], "Status", timeout=1)
                if st["applied_index"] >= target and st["leader"] == new:
                    break
            except grpc.RpcError:
                pass
            time.sleep(0.2)
        else:
            raise AssertionError(f"restarted node never caught up: {st} vs commit {target}")
        users = json.load(open(tmp_path / f"d{lid}" / "lms_data.json"))["users"]
        assert {"alice", "bob", "carol"} <= set(users)
        cl.close()
    finally:
        for p in procs.values():
            p.kill()


def test_sigstopped_follower_bounded_queue_and_catch_up(tmp_path):
    """A follower frozen with SIGSTOP for 10 s while the leader keeps committing (2 of 3): the
    leader's per-peer send mailbox stays bounded (one pending message per kind, newer appends
    supersede older ones) and, after SIGCONT, the follower catches up cleanly."""
    ports = _ports(3)
    addrs = {i + 1: f"127.0.0.1:{p}" for i, p in enumerate(ports)}
    cfg = {"servers": addrs, "host": "127.0.0.1", "gate": "off", "tutor": "", "no_fsync": True,
           "log_level": "WARNING"}
    procs = {}
    try:
        for i in addrs:
            (tmp_path / f"d{i}").mkdir()
            cfg_i = dict(cfg, data_dir=str(tmp_path / f"d{i}"))
            (tmp_path / f"cluster{i}.yaml").write_text(yaml.safe_dump(cfg_i))
            procs[i] = Proc(tmp_path, tmp_path / f"cluster{i}.yaml", i)
        lid = _leader(addrs, set(addrs), timeout=60)
        victim = next(i for i in addrs if i != lid)
        cl = LMSClient(list(addrs.values()), timeout=5)
        os.killpg(procs[victim].p.pid, signal.SIGSTOP)
        worst = 0
        t_end = time.time() + 10
        n = 0
        while time.time() < t_end:
            assert cl.register(f"u{n}", "pw", "student").success
            n += 1
            st = debug_call(addrs[lid], "Status")
            worst = max(worst, st["transport_pending"][str(victim)]["pending"])
        assert worst <= 3, worst
        st = debug_call(addrs[lid], "Status")
        assert st["role"] == "leader" and st["transport_pending"][str(victim)]["superseded"] > 0
        target = st["commit_index"]
        os.killpg(procs[victim].p.pid, signal.SIGCONT)
        end = time.time() + 30
        while time.time() < end:
            s2 = debug_call(addrs[victim], "Status", timeout=2)
            if s2["applied_index"] >= target:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"resumed follower never caught up: {s2} vs {target}")
        assert s2["leader"] == lid  # no disruptive election after resuming (pre-vote)
        users = json.load(open(tmp_path / f"d{victim}" / "lms_data.json"))["users"]
        assert {f"u{k}" for k in range(n)} <= set(users)
        cl.close()
    finally:
        for p in procs.values():
            try:
                os.killpg(p.p.pid, signal.SIGCONT)
            except ProcessLookupError:
                pass
            p.kill()
