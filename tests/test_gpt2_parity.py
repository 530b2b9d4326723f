"""GPT-2 parity pinned against HuggingFace ``transformers`` (SURVEY.md §4.3 "Model E2E"): the
reference's exact call -- ``GPT2LMHeadModel.generate(max_length, repetition_penalty=1.2)``,
greedy (``tutoring_server.py:21-29``; sampling flags unset) -- on the SAME random weights must
produce the same token ids as our fp32 reference decode and our CPU engine.  Also pins every
GPT-2 size's architecture numbers to transformers' published configs."""
import pytest
import torch

from distributed_lms_raft_llm_amd.engine.gpt2_engine import TorchGPT2Engine
from distributed_lms_raft_llm_amd.models.config import GPT2Config, gpt2_config
from distributed_lms_raft_llm_amd.models.gpt2 import (GPT2Reference, init_gpt2_weights, perturb_norms_and_biases,
                                                      reference_generate)

transformers = pytest.importorskip("transformers")
pytestmark = pytest.mark.timeout(300)


def _hf_model(cfg: GPT2Config, w):
    hcfg = transformers.GPT2Config(vocab_size=cfg.vocab_size, n_positions=cfg.n_positions, n_embd=cfg.n_embd,
                                   n_layer=cfg.n_layer, n_head=cfg.n_head, layer_norm_epsilon=cfg.layer_norm_epsilon,
                                   activation_function="gelu_new", bos_token_id=cfg.eos_token_id,
                                   eos_token_id=cfg.eos_token_id, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    m = transformers.GPT2LMHeadModel(hcfg).eval()
    missing, unexpected = m.load_state_dict(w, strict=False)
    assert not unexpected and all("attn.bias" in k or "masked_bias" in k or k == "lm_head.weight" for k in missing)
    m.tie_weights()
    return m


@pytest.mark.parametrize("cfg", [gpt2_config("gpt2-tiny"),
                                 GPT2Config("gpt2-mini", 3, 192, 3, n_positions=128, vocab_size=3000,
                                            eos_token_id=2999)])
def test_greedy_reppen_token_exact_vs_transformers_generate(cfg):
    w = init_gpt2_weights(cfg, seed=4)
    perturb_norms_and_biases(w, scale=0.1)
    hf = _hf_model(cfg, w)
    g = torch.Generator().manual_seed(5)
    T = 60
    prompts = [torch.randint(0, cfg.vocab_size - 1, (n,), generator=g).tolist() for n in (1, 9, 17)]
    ours = reference_generate(GPT2Reference(cfg, w), prompts, max_length=T, repetition_penalty=1.2)
    engine = TorchGPT2Engine(cfg, w, max_length=T).generate(prompts, repetition_penalty=1.2)
    for p, o, e in zip(prompts, ours, engine):
        with torch.no_grad():
            ref = hf.generate(torch.tensor([p]), attention_mask=torch.ones(1, len(p), dtype=torch.long),
                              max_length=T, repetition_penalty=1.2, do_sample=False, num_beams=1,
                              pad_token_id=cfg.eos_token_id)[0].tolist()
        assert o == ref, (p, o, ref)
        assert e == ref


@pytest.mark.parametrize("name,hf_name", [("gpt2", "gpt2"), ("gpt2-medium", "gpt2-medium"),
                                          ("gpt2-large", "gpt2-large"), ("gpt2-xl", "gpt2-xl")])
def test_model_sizes_match_published_configs(name, hf_name):
    # the published GPT-2 family (n_layer, n_embd, n_head); transformers' defaults are GPT-2 small
    published = {"gpt2": (12, 768, 12), "gpt2-medium": (24, 1024, 16), "gpt2-large": (36, 1280, 20),
                 "gpt2-xl": (48, 1600, 25)}
    cfg = gpt2_config(name)
    assert (cfg.n_layer, cfg.n_embd, cfg.n_head) == published[hf_name]
    d = transformers.GPT2Config()
    assert (cfg.vocab_size, cfg.n_positions, cfg.eos_token_id, cfg.layer_norm_epsilon) == \
        (d.vocab_size, d.n_positions, d.eos_token_id, d.layer_norm_epsilon)
    assert cfg.n_inner == 4 * cfg.n_embd and cfg.head_dim == 64


def test_batched_teacher_forced_oracle_equals_per_row():
    """The batched margin oracle (used for the 1024-row production-path test) gives the per-row
    oracle's results, including the mismatches of a corrupted sequence."""
    from distributed_lms_raft_llm_amd.models.gpt2 import (reference_generate, teacher_forced_check,
                                                           teacher_forced_check_batch)

    cfg = gpt2_config("gpt2-tiny")
    m = GPT2Reference(cfg, init_gpt2_weights(cfg, seed=0))
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(0, cfg.vocab_size - 1, (n,), generator=g).tolist() for n in (3, 9, 5, 29)]
    seqs = reference_generate(m, prompts, max_length=30)
    seqs[1][12] = (seqs[1][12] + 1) % cfg.vocab_size
    a = [teacher_forced_check(m, s, len(p)) for s, p in zip(seqs, prompts)]
    b = teacher_forced_check_batch(m, seqs, [len(p) for p in prompts], chunk=3)
    assert a[1]["mismatches"] and not a[0]["mismatches"]
    for x, y in zip(a, b):
        assert (x["positions"], x["decisive"]) == (y["positions"], y["decisive"])
        assert [t[:3] for t in x["mismatches"]] == [t[:3] for t in y["mismatches"]]
        assert abs(x["min_margin"] - y["min_margin"]) < 1e-4
