"""BERT gate: the torch reference encoder matches HF ``BertModel`` on the same weights (CPU,
fp32, parity pinned against transformers), and the HIP encoder matches the reference (GPU)."""
import time

import pytest
import torch

from distributed_lms_raft_llm_amd.models.bert import BertReference, init_bert_weights
from distributed_lms_raft_llm_amd.models.config import bert_config


def _weights(name, seed=0):
    cfg = bert_config(name)
    w = init_bert_weights(cfg, seed=seed)
    g = torch.Generator().manual_seed(5)
    for k, v in w.items():  # non-trivial LN/bias values
        if k.endswith("bias") or "LayerNorm" in k:
            v.add_(torch.randn(v.shape, generator=g) * 0.05)
    return cfg, w


def test_reference_matches_transformers_bertmodel():
    transformers = pytest.importorskip("transformers")
    cfg, w = _weights("bert-tiny")
    hcfg = transformers.BertConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, num_hidden_layers=cfg.n_layer,
                                   num_attention_heads=cfg.n_head, intermediate_size=cfg.intermediate,
                                   max_position_embeddings=cfg.max_position, layer_norm_eps=cfg.layer_norm_eps,
                                   hidden_act="gelu")
    hf = transformers.BertModel(hcfg, add_pooling_layer=False).eval()
    missing, unexpected = hf.load_state_dict(w, strict=False)
    assert not unexpected and all("position_ids" in m for m in missing)
    ids = [101, 7, 99, 500, 3, 102]
    with torch.no_grad():
        ref = hf(torch.tensor([ids])).last_hidden_state.mean(dim=1)[0]
    ours = BertReference(cfg, w).embed([ids])[0]
    torch.testing.assert_close(ours, ref, atol=1e-5, rtol=1e-5)


def test_gate_semantics_cpu():
    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    gate = RelevanceGate.create("bert-tiny", device="cpu", threshold=0.6)
    s_same = gate.similarity("raft leader election", "raft leader election")
    assert abs(s_same - 1.0) < 1e-5
    ok, s = gate.check("anything", "some assignment text")
    assert ok == (s >= 0.6)
    gate.threshold = 1.01
    assert gate.check("raft", "raft")[0] is False


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bert-tiny", "bert-base-uncased"])
def test_hip_encoder_matches_reference(name):
    from distributed_lms_raft_llm_amd.engine.bert_engine import HipBertEncoder

    cfg, w = _weights(name)
    for k, v in w.items():  # give the oracle the same bf16-rounded matrices
        if v.dim() == 2 and "embeddings" not in k:
            w[k] = v.to(torch.bfloat16).float()
    enc = HipBertEncoder(cfg, w)
    g = torch.Generator().manual_seed(0)
    batch = [torch.randint(110, cfg.vocab_size, (L,), generator=g).tolist()
             for L in (5, 64, 1, min(200, cfg.max_position))]
    got_d = enc.embed(batch)
    got = got_d.cpu()
    ref = BertReference(cfg, w, device="cuda").embed(batch).cpu()
    for b in range(len(batch)):
        cos = torch.nn.functional.cosine_similarity(got[b], ref[b], dim=0).item()
        assert cos > 0.999, (b, cos)
        torch.testing.assert_close(got[b], ref[b], atol=5e-2, rtol=5e-2)
    sim = enc.cosine(got_d, got_d).cpu()
    torch.testing.assert_close(torch.diagonal(sim), torch.ones(len(batch)), atol=1e-5, rtol=1e-5)


def test_gate_batches_concurrent_queries_cpu():
    """concurrent checks share packed encoder passes and score exactly like serial
    single-query passes."""
    from concurrent.futures import ThreadPoolExecutor

    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    gate = RelevanceGate.create("bert-tiny", device="cpu", threshold=0.6)
    gate.window_s = 0.02
    text = "raft replicates a log of commands across a majority of nodes"
    queries = [f"question {k} about " + " ".join(["leader", "term", "vote", "log"][: 1 + k % 4]) for k in range(24)]
    ref = []
    for qtext in queries:  # serial oracle: one encoder pass per query, no batcher
        q = gate.embed([qtext])[0]
        a = gate.embed([text])[0]
        ref.append(torch.nn.functional.cosine_similarity(q[None], a[None]).item())
    with ThreadPoolExecutor(24) as ex:
        got = list(ex.map(lambda qt: gate.check(qt, text)[1], queries))
    for g_, r_ in zip(got, ref):
        assert abs(g_ - r_) < 1e-5
    assert gate.batched_queries == len(queries)
    assert gate.passes < len(queries)  # at least some queries shared a pass


def test_check_async_cache_read_never_waits_on_an_encoder_pass():
    """the aio front end reads the assignment-embedding cache on its event
    loop; an encoder pass in progress (the gate's ``_lock`` held) must not stall that read."""
    import asyncio

    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    gate = RelevanceGate.create("bert-tiny", device="cpu", threshold=0.6)
    text = "raft replicates a log"
    gate.warm(text)
    gate._lock.acquire()  # an encoder pass that takes a long time
    try:
        t0 = time.monotonic()
        a = asyncio.run(asyncio.wait_for(asyncio.to_thread(lambda: gate._cache_get(gate._key(text))), 2.0))
        assert a is not None and time.monotonic() - t0 < 1.0
        # the full check_async: its cache read returns at once; the query itself waits for the pass
        loop = asyncio.new_event_loop()
        task = loop.create_task(gate.check_async("raft", text))
        loop.run_until_complete(asyncio.sleep(0.05))
        assert not task.done()  # parked on its batch, the loop kept running (this sleep returned)
    finally:
        gate._lock.release()
    ok, s = loop.run_until_complete(asyncio.wait_for(task, 10.0))
    loop.close()
    assert ok == (s >= 0.6)


@pytest.mark.gpu
def test_hip_gate_batched_at_512_tokens():
    """Packed varlen passes at the reference's 512-token truncation: every row of a mixed batch
    (1..512 tokens) matches the fp32 torch reference, and the gate's batched scores match it."""
    from concurrent.futures import ThreadPoolExecutor

    from distributed_lms_raft_llm_amd.engine.bert_engine import HipBertEncoder
    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    cfg, w = _weights("bert-base-uncased")
    for k, v in w.items():
        if v.dim() == 2 and "embeddings" not in k:
            w[k] = v.to(torch.bfloat16).float()
    enc = HipBertEncoder(cfg, w)
    g = torch.Generator().manual_seed(1)
    lens = [512, 1, 37, 512, 300, 128, 511, 2]
    batch = [torch.randint(110, cfg.vocab_size, (L,), generator=g).tolist() for L in lens]
    got = enc.embed(batch).float().cpu()
    ref = BertReference(cfg, w, device="cuda").embed(batch).cpu()
    for b in range(len(batch)):
        cos = torch.nn.functional.cosine_similarity(got[b], ref[b], dim=0).item()
        assert cos > 0.999, (lens[b], cos)
    # through the gate's batcher, 32 concurrent queries against one assignment text
    from distributed_lms_raft_llm_amd.tokenizer import BertWordPiece

    gate = RelevanceGate(enc, BertWordPiece(None, vocab_size=cfg.vocab_size, max_length=cfg.max_position), 0.6)
    gate.window_s = 0.005
    text = " ".join(f"w{k}" for k in range(600))  # truncated at 512 tokens
    queries = [" ".join(f"w{j}" for j in range(k, k + 5 + 13 * k)) for k in range(32)]
    with ThreadPoolExecutor(32) as ex:
        got_s = list(ex.map(lambda q: gate.check(q, text)[1], queries))
    a = enc.embed([gate.tok.encode(text)]).float()
    for q, s in zip(queries, got_s):
        qe = enc.embed([gate.tok.encode(q)]).float()
        r = torch.nn.functional.cosine_similarity(qe, a).item()
        assert abs(s - r) < 2e-3, (q[:20], s, r)
    assert gate.passes < len(queries)


@pytest.mark.gpu
def test_hip_encoder_graph_buckets_match_eager():
    """hipGraph-replayed passes (rows padded to a power-of-two bucket by dummy sequences, tile table
    padded by repeating its last tile) == the eager packed pass, across buckets and re-used buckets
    with different length mixes."""
    from distributed_lms_raft_llm_amd.engine.bert_engine import HipBertEncoder

    cfg, w = _weights("bert-base-uncased")
    graphed = HipBertEncoder(cfg, w, use_graph=True)
    eager = HipBertEncoder(cfg, w, use_graph=False)
    g = torch.Generator().manual_seed(7)
    mixes = [(5,), (40, 3, 17), (64,), (33, 31), (1, 1, 1, 1, 1), (512, 7), (300, 250, 100), (12,) * 40]
    for lens in mixes + mixes[:3]:
        batch = [torch.randint(110, cfg.vocab_size, (L,), generator=g).tolist() for L in lens]
        a = graphed.embed(batch).cpu()
        b = eager.embed(batch).cpu()
        assert a.shape == b.shape == (len(lens), cfg.hidden)
        cos = torch.nn.functional.cosine_similarity(a, b, dim=1)
        assert cos.min().item() > 0.9999, (lens, cos)
        torch.testing.assert_close(a, b, atol=2e-2, rtol=2e-2)
    assert len(graphed._gstate) >= 3 and all(st["graph"] is not None for st in graphed._gstate.values())
