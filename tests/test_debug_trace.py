"""Tracing (utils/trace.py), the internal debug RPCs (utils/debug_rpc.py) on a live cluster and a
tutoring server, and multi-replica tutoring failover (TutoringClient)."""
import json

import pytest

from distributed_lms_raft_llm_amd.utils.debug_rpc import debug_call
from distributed_lms_raft_llm_amd.utils.trace import TRACER, Tracer

pytestmark = pytest.mark.timeout(120)


def test_tracer_spans_and_dump(tmp_path):
    t = Tracer(cap=10)
    t.instant("dropped")  # disabled: nothing recorded
    t.enable()
    with t.span("outer", k=1):
        t.instant("inside", x=2)
    for i in range(20):
        t.instant("spam", i=i)
    ev = t.events()
    assert len(ev) == 10 and ev[-1]["args"]["i"] == 19  # bounded ring keeps the newest
    t.clear()
    with t.span("s"):
        pass
    t.dump(str(tmp_path / "t.json"))
    doc = json.load(open(tmp_path / "t.json"))
    assert doc["traceEvents"][0]["ph"] == "X" and doc["traceEvents"][0]["dur"] >= 0
    t.dump(str(tmp_path / "t.jsonl"))
    assert json.loads(open(tmp_path / "t.jsonl").readline())["name"] == "s"


def test_cluster_debug_rpcs_and_raft_trace(tmp_path):
    from lms_harness import Cluster

    TRACER.enable()
    TRACER.clear()
    c = Cluster(3, tmp_path)
    try:
        lid = c.wait_leader()
        addr = c.addrs[lid]
        h = debug_call(addr, "Health")
        assert h["ok"] and h["role"] == "leader" and h["leader"] == lid
        st = debug_call(addr, "Status")
        assert st["role"] == "leader" and st["commit_index"] >= 1
        m = debug_call(addr, "Metrics")
        assert m["counters"].get("raft_leaderships_won", 0) >= 1
        tr = debug_call(addr, "Trace")
        names = {e["name"] for e in tr["events"]}
        assert "raft.transition" in names and "raft.commit" in names
    finally:
        c.close()
        TRACER.enable(False)


def test_tutoring_client_fails_over_between_replicas():
    from lms_harness import start_tutor

    from distributed_lms_raft_llm_amd.lms.service import TutoringClient

    sa, pa, ea = start_tutor()
    sb, pb_, eb = start_tutor()
    dead = "127.0.0.1:1"  # nothing listens there
    cl = TutoringClient(f"{dead},127.0.0.1:{pa},127.0.0.1:{pb_}", timeout=10)
    try:
        for _ in range(4):
            assert cl.ask("tok", "what is raft").success
        assert cl._down_until[0] > 0  # the dead replica was marked down
        assert ea.calls and len(ea.calls) + len(eb.calls) == 4
        sa.stop(0).wait()
        for _ in range(3):
            assert cl.ask("tok", "again").success  # b still answers
        assert len(eb.calls) >= 3
    finally:
        cl.close()
        sb.stop(0)


def test_tutoring_server_health_rpc():
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import TorchGPT2Engine
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights
    from distributed_lms_raft_llm_amd.tutor.server import TutoringServer

    cfg = gpt2_config("gpt2-tiny")
    srv = TutoringServer(TorchGPT2Engine(cfg, init_gpt2_weights(cfg, seed=0), max_length=120), port=0,
                         host="127.0.0.1", max_length=120).start()
    try:
        h = debug_call(f"127.0.0.1:{srv.port}", "Health")
        assert h["ok"] and h["batching"] == "window" and h["engine"] == "TorchGPT2Engine"
        assert "counters" in debug_call(f"127.0.0.1:{srv.port}", "Metrics")
    finally:
        srv.stop()
