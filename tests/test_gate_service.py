"""The relevance gate as a GPU-tier service (gate/service.py): one batched encoder behind an internal
gRPC service, LMS nodes calling it through ``RemoteGate`` (CPU here: bert-tiny torch encoder)."""
import os
import signal
import subprocess
import sys
import time

import grpc
import pytest

from distributed_lms_raft_llm_amd import wire
from distributed_lms_raft_llm_amd.wire import pb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.timeout(300)


def _gate():
    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    return RelevanceGate.create("bert-tiny", device="cpu", threshold=0.6)


@pytest.fixture
def gate_server():
    from distributed_lms_raft_llm_amd.gate.service import GateServer

    srv = GateServer(_gate(), 0, "127.0.0.1").start()
    yield srv
    srv.stop()


def test_remote_gate_equals_local_gate(gate_server):
    """Same encoder weights: the service's similarity is the local gate's, through the key-only
    request, the text-on-miss retry and the Embed warm-up; the threshold is the caller's."""
    from distributed_lms_raft_llm_amd.gate.service import RemoteGate

    local = _gate()
    remote = RemoteGate([f"127.0.0.1:{gate_server.port}"], threshold=0.6)
    text = "raft leader election and log replication across five servers"
    s = remote.similarity("how does the leader get elected", text)
    assert abs(s - local.similarity("how does the leader get elected", text)) < 1e-5
    assert gate_server.missing == 1 and gate_server.scored == 1  # first call: text sent once
    remote.similarity("what is a term", text)
    assert gate_server.missing == 1  # cached by key from then on
    other = "consistent hashing ring with virtual nodes"
    remote.warm(other)
    remote.similarity("virtual nodes", other)
    assert gate_server.missing == 1
    ok, s2 = remote.check("raft", text)
    assert ok == (s2 >= 0.6)
    remote.threshold = 1.01
    assert remote.check("raft", text)[0] is False
    remote.close()


def test_remote_gate_async_and_failover(gate_server):
    """check_async on an event loop; a dead first address is skipped; with every server down the
    local fallback decides (or, without one, the query is admitted)."""
    import asyncio
    import socket

    from distributed_lms_raft_llm_amd.gate.service import RemoteGate

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    dead = f"127.0.0.1:{s.getsockname()[1]}"
    s.close()
    text = "paxos and raft comparison"
    remote = RemoteGate([dead, f"127.0.0.1:{gate_server.port}"], threshold=0.6, timeout=2.0)
    ok, sim = asyncio.run(remote.check_async("raft vs paxos", text))
    assert remote.remote_calls == 1 and remote.fallbacks == 0
    assert abs(sim - _gate().similarity("raft vs paxos", text)) < 1e-5
    only_dead = RemoteGate([dead], threshold=0.6, timeout=2.0, fallback_factory=_gate)
    ok2, sim2 = only_dead.check("raft vs paxos", text)
    assert only_dead.fallbacks == 1 and abs(sim2 - sim) < 1e-5
    admit = RemoteGate([dead], threshold=0.6, timeout=2.0)
    assert admit.check("anything", text) == (True, 1.0)


def _wait_port(addr, timeout=120):
    end = time.time() + timeout
    while time.time() < end:
        try:
            with grpc.insecure_channel(addr) as ch:
                grpc.channel_ready_future(ch).result(timeout=1)
                return
        except grpc.FutureTimeoutError:
            time.sleep(0.2)
    raise TimeoutError(addr)


def test_gpu_less_lms_node_gates_on_the_gate_tier(gate_server, tmp_path):
    """An LMS node started with no visible GPU (``--gate remote``) sends GetLLMAnswer's relevance
    check to the gate server, and the admitted query reaches the tutoring tier."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from lms_harness import free_ports, start_tutor

    from distributed_lms_raft_llm_amd.lms.pdf import make_pdf

    tsrv, tport, tutor = start_tutor()
    port = free_ports(1)[0]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "distributed_lms_raft_llm_amd.lms.server", "1", str(port), "--host", "127.0.0.1",
           "--data-dir", str(tmp_path / "n1"), "--tutor", f"127.0.0.1:{tport}", "--gate", "remote",
           "--gate-addr", f"127.0.0.1:{gate_server.port}", "--gate-fallback", "off", "--gate-threshold", "-1",
           "--log-level", "WARNING", "--no-fsync"]
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         start_new_session=True)
    try:
        addr = f"127.0.0.1:{port}"
        _wait_port(addr)
        st = wire.Stub("LMS", wire.channel(addr))
        end = time.time() + 60
        while True:  # single-node Raft: wait for its own election
            r = st.Register(pb.RegisterRequest(username="s1", password="pw", role="student"), timeout=10)
            if r.success or time.time() > end:
                break
            time.sleep(0.2)
        tok = st.Login(pb.LoginRequest(username="s1", password="pw"), timeout=10).token
        assert tok
        assert st.Post(pb.PostRequest(token=tok, type="assignment", file=make_pdf("raft consensus homework"),
                                      filename="hw.pdf"), timeout=30).success
        r = st.GetLLMAnswer(pb.QueryRequest(token=tok, query="explain raft"), timeout=60)
        assert r.success and r.response.startswith("Question: explain raft"), r.response
        assert gate_server.scored >= 1  # the relevance check ran on the gate tier
        assert tutor.calls == ["explain raft"]
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
        tsrv.stop(0)


def test_tutor_front_ends_serve_the_gate_between_decode_chunks():
    """--serve-gate: the tutor's front-end processes answer lmsinternal.Gate on the tutoring port
    (tokenizing with BERT WordPiece), the engine process scores between decode chunks (GateWorker on
    the batcher thread) -- same similarities as the local gate, tutoring unaffected."""
    import asyncio

    from distributed_lms_raft_llm_amd.gate.service import GateWorker, RemoteGate
    from distributed_lms_raft_llm_amd.models.bert import BertReference, init_bert_weights
    from distributed_lms_raft_llm_amd.models.config import bert_config, gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights
    from distributed_lms_raft_llm_amd.parallel.tp import TorchSlotEngine
    from distributed_lms_raft_llm_amd.tutor.frontend import FrontendPool
    from distributed_lms_raft_llm_amd.tutor.server import PooledTutoringServer

    bc = bert_config("bert-tiny")
    cfg = gpt2_config("gpt2-tiny")
    pool = FrontendPool(1, 0, "127.0.0.1", eos=cfg.eos_token_id,
                        gate=dict(vocab=None, vocab_size=bc.vocab_size, max_length=bc.max_position))
    eng = TorchSlotEngine(cfg, init_gpt2_weights(cfg, seed=0), max_batch=4, max_length=40)
    srv = PooledTutoringServer(eng, pool, max_length=40, chunk=2)
    pool.gate_worker = GateWorker(BertReference(bc, init_bert_weights(bc, seed=0)))
    pool.gate_worker.attach(srv.batcher)
    srv.start()
    try:
        addr = f"127.0.0.1:{srv.port}"
        remote = RemoteGate([addr], threshold=0.6)
        local = _gate()
        text = "raft leader election and log replication"
        s_sync = remote.similarity("who is the leader", text)  # Score: key miss, then the text
        assert abs(s_sync - local.similarity("who is the leader", text)) < 1e-4
        ok, s_async = asyncio.run(remote.check_async("what is a term", text))  # ScoreBatch, cached key
        assert abs(s_async - local.similarity("what is a term", text)) < 1e-4
        remote.warm("virtual nodes on a hash ring")  # Embed
        assert pool.gate_worker.passes >= 3 and pool.gate_worker.scored == 2
        st = wire.Stub("Tutoring", wire.channel(addr))
        r = st.GetLLMAnswer(pb.QueryRequest(token="t", query="hello"), timeout=60)
        assert r.success
    finally:
        srv.stop()


def test_gate_worker_splits_oversized_requests():
    """A ScoreBatch larger than one encoder pass is split across passes and answered in order."""
    from distributed_lms_raft_llm_amd.gate.service import GateWorker
    from distributed_lms_raft_llm_amd.models.bert import BertReference, init_bert_weights
    from distributed_lms_raft_llm_amd.models.config import bert_config
    from distributed_lms_raft_llm_amd.tokenizer import BertWordPiece

    bc = bert_config("bert-tiny")
    w = GateWorker(BertReference(bc, init_bert_weights(bc, seed=0)), max_seqs=8)
    tok = BertWordPiece(None, vocab_size=bc.vocab_size, max_length=bc.max_position)
    text = "raft leader election"
    items = [(tok.encode(f"query number {i}"), "k", tok.encode(text) if i == 0 else None) for i in range(21)]
    out = []
    w.submit(items, out.append)
    while w.pending():
        w.work(True)
    assert len(out) == 1 and len(out[0]) == 21 and all(isinstance(x, float) for x in out[0])
    local = _gate()
    assert abs(out[0][5] - local.similarity("query number 5", text)) < 1e-4
    assert w.passes >= 3


def test_gate_worker_fills_passes_across_requests():
    """Passes are packed full: the request that no longer fits is split so its head fills the pass
    (two 40-query requests, 64 sequences per pass -> 2 passes, not 3), and both callers get every
    result in item order."""
    from distributed_lms_raft_llm_amd.gate.service import GateWorker
    from distributed_lms_raft_llm_amd.models.bert import BertReference, init_bert_weights
    from distributed_lms_raft_llm_amd.models.config import bert_config
    from distributed_lms_raft_llm_amd.tokenizer import BertWordPiece

    bc = bert_config("bert-tiny")
    w = GateWorker(BertReference(bc, init_bert_weights(bc, seed=0)), max_seqs=64)
    tok = BertWordPiece(None, vocab_size=bc.vocab_size, max_length=bc.max_position)
    text = "consensus with a replicated log"
    w.submit([(None, "k", tok.encode(text))], lambda r: None)  # embed the assignment first
    while w.pending():
        w.work(True)
    assert w.passes == 1
    outs = [[], []]
    for r in range(2):
        w.submit([(tok.encode(f"request {r} query {i}"), "k", None) for i in range(40)], outs[r].append)
    while w.pending():
        w.work(True)
    assert w.passes == 1 + 2
    assert [len(o) for o in outs] == [1, 1] and len(outs[0][0]) == 40 and len(outs[1][0]) == 40
    local = _gate()
    assert abs(outs[1][0][33] - local.similarity("request 1 query 33", text)) < 1e-4
