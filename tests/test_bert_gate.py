"""BERT gate: the torch reference encoder matches HF ``BertModel`` on the same weights (CPU,
fp32, parity pinned against transformers), and the HIP encoder matches the reference (GPU)."""
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
