"""Tutoring service end to end on CPU (BASELINE config 1: GPT-2 decode via gRPC, no GPU) and
the full LMS -> gate -> tutoring path through a Raft cluster."""
import threading

import pytest
import torch

from distributed_lms_raft_llm_amd import wire
from distributed_lms_raft_llm_amd.engine.gpt2_engine import TorchGPT2Engine
from distributed_lms_raft_llm_amd.models.config import gpt2_config
from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, init_gpt2_weights, reference_generate
from distributed_lms_raft_llm_amd.tokenizer import GPT2BPE
from distributed_lms_raft_llm_amd.tutor.server import PROMPT_TEMPLATE, TutoringServer, build_prompt
from distributed_lms_raft_llm_amd.wire import pb

pytestmark = pytest.mark.timeout(300)


@pytest.fixture(scope="module")
def tiny():
    cfg = gpt2_config("gpt2-tiny")
    w = init_gpt2_weights(cfg, seed=3)
    return cfg, w


def test_prompt_template_verbatim():
    assert build_prompt("what is raft?") == (
        "You are an intelligent assistant. Answer the following question in detail:\nQuestion: what is raft?\nAnswer:")
    assert PROMPT_TEMPLATE.count("{query}") == 1


def test_tutoring_grpc_batched_matches_unbatched_reference(tiny):
    cfg, w = tiny
    eng = TorchGPT2Engine(cfg, w, max_length=160)
    tok = GPT2BPE(eos_token_id=cfg.eos_token_id)
    srv = TutoringServer(eng, port=0, host="127.0.0.1", max_batch=8, window_ms=50, max_length=160,
                         tokenizer=tok).start()
    try:
        stub = wire.Stub("Tutoring", wire.channel(f"127.0.0.1:{srv.port}"))
        queries = ["what is a quorum?", "explain log matching", "why randomize election timeouts?"]
        results = {}

        def ask(q):
            results[q] = stub.GetLLMAnswer(pb.QueryRequest(token="t", query=q), timeout=120)

        ts = [threading.Thread(target=ask, args=(q,)) for q in queries]
        [t.start() for t in ts]
        [t.join() for t in ts]
        model = GPT2Reference(cfg, w)
        for q in queries:
            r = results[q]
            assert r.success
            prompt = build_prompt(q)
            assert r.response.startswith(prompt)  # generate() echoes the prompt
            ids = tok.encode(prompt)
            ref = reference_generate(model, [ids], max_length=160)[0]
            assert r.response == tok.decode(ref)
    finally:
        srv.stop()


def test_llm_answer_through_cluster_with_bert_gate(tiny, tmp_path):
    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate
    from lms_harness import Cluster

    cfg, w = tiny
    srv = TutoringServer(TorchGPT2Engine(cfg, w, max_length=140), port=0, host="127.0.0.1", max_length=140,
                         window_ms=1).start()
    gate = RelevanceGate.create("bert-tiny", device="cpu", threshold=0.0)
    c = Cluster(3, tmp_path, tutor_address=f"127.0.0.1:{srv.port}", gate=gate)
    try:
        lid = c.wait_leader()
        st = c.stub(lid)
        st.Register(pb.RegisterRequest(username="s", password="p", role="student"), timeout=10)
        tok = st.Login(pb.LoginRequest(username="s", password="p"), timeout=10).token
        st.Post(pb.PostRequest(token=tok, type="assignment", file=b"consensus protocols", filename="a.txt"),
                timeout=10)
        r = st.GetLLMAnswer(pb.QueryRequest(token=tok, query="what is consensus"), timeout=120)
        assert r.success and r.response.startswith(build_prompt("what is consensus"))
        gate.threshold = 1.5  # nothing can pass: the reference's rejection string comes back
        r = st.GetLLMAnswer(pb.QueryRequest(token=tok, query="what is consensus"), timeout=120)
        assert r.response.startswith("Your query does not relate to your assignment.")
    finally:
        c.close()
        srv.stop()
