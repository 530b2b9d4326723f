"""CPU checks of the persistent dataflow decode's work split and packed weight streams
(ops/dataflow.py): every weight row is owned by exactly one CU and sits in that CU's stream in
the order the kernel consumes it."""
import numpy as np
import pytest
import torch

from distributed_lms_raft_llm_amd.models.config import GPT2Config, gpt2_config
from distributed_lms_raft_llm_amd.ops.dataflow import ROW_PAD, assign, block_k, pack_weights


@pytest.mark.parametrize("name,G,GS", [("gpt2", 256, 4), ("gpt2-medium", 256, 4), ("gpt2-xl", 256, 4),
                                       ("gpt2-tiny", 64, 4), ("gpt2", 80, 2)])
def test_assignment_covers_every_row_once(name, G, GS):
    cfg = gpt2_config(name)
    d, H, F, V = cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded
    cus = assign(d, H, F, V, G, GS)
    assert len(cus) == G
    for key, n in (("q", 3 * d), ("f", F), ("v", V)):
        covered = np.zeros(n, dtype=int)
        for cu in cus:
            s, c = getattr(cu, key + "0"), getattr(cu, "n" + key)
            covered[s: s + c] += 1
        assert (covered == 1).all(), key
    # W_o^T rows: head h, dims [ak0, ak0 + nk) -- every (head, dim) exactly once
    cov = np.zeros((H, 64), dtype=int)
    att = [cu for cu in cus if cu.ah >= 0]
    assert len(att) == H * GS
    for cu in att:
        cov[cu.ah, cu.ak0: cu.ak0 + cu.nk] += 1
    assert (cov == 1).all()
    assert max(cu.nq for cu in cus) <= 64


def test_assignment_rejects_bad_split():
    with pytest.raises(ValueError):
        assign(768, 12, 3072, 50304, 16, 4)  # 48 attention CUs on 16
    with pytest.raises(ValueError):
        assign(768, 12, 3072, 50304, 256, 3)  # 3 does not divide 64


def test_packed_stream_matches_sources():
    from distributed_lms_raft_llm_amd.engine.weights import prepare_gpt2_weights
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    cfg = GPT2Config("df-test", n_layer=2, n_embd=128, n_head=2, n_positions=64, vocab_size=300, eos_token_id=299)
    w = prepare_gpt2_weights(cfg, init_gpt2_weights(cfg, seed=3), "cpu")
    G, GS = 16, 4
    cus = assign(cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded, G, GS)
    packed, starts = pack_weights(w, cus, "cpu")
    ko, kf = block_k(cus)
    d, L = cfg.n_embd, cfg.n_layer
    assert packed.numel() == sum(cu.step_elems(L, d, ko, kf) for cu in cus)
    assert starts[0] == 0 and starts[1] == cus[0].step_elems(L, d, ko, kf)

    def rows(o, n):  # n padded rows of d at element offset o
        v = packed[o: o + n * (d + ROW_PAD)].reshape(n, d + ROW_PAD)
        assert not v[:, d:].any()
        return v[:, :d]

    for c, cu in enumerate(cus):  # walk each CU's stream and check every piece
        o = starts[c]
        for l, lw in enumerate(w.layers):
            assert torch.equal(rows(o, cu.nq), lw.w_qkv[cu.q0: cu.q0 + cu.nq])
            o += cu.nq * (d + ROW_PAD)
            if cu.nk:
                blk = packed[o: o + d * ko].reshape(d, ko)  # K-major: [d][ko]
                cols = lw.w_o[:, cu.ah * 64 + cu.ak0: cu.ah * 64 + cu.ak0 + cu.nk]
                assert torch.equal(blk[:, : cu.nk], cols) and not blk[:, cu.nk:].any()
                o += d * ko
            assert torch.equal(rows(o, cu.nf), lw.w_fc[cu.f0: cu.f0 + cu.nf])
            o += cu.nf * (d + ROW_PAD)
            blk = packed[o: o + d * kf].reshape(d, kf)
            assert torch.equal(blk[:, : cu.nf], lw.w_p[:, cu.f0: cu.f0 + cu.nf]) and not blk[:, cu.nf:].any()
            o += d * kf
        assert torch.equal(rows(o, cu.nv), w.wte[cu.v0: cu.v0 + cu.nv])


def _emulate_step(cfg, w, cus, tok, pos, kv):
    """One decode step computed the way the dataflow kernel splits it (per-CU partial sums, in
    float64): returns the final hidden state after ln_f.  ``kv``: per layer (K, V) [H, pos, 64]."""
    d, H = cfg.n_embd, cfg.n_head
    f = lambda t: t.double()  # noqa: E731
    x = f(w.wte[tok]) + f(w.wpe[pos])

    def ln(v, g, b):
        m = v.mean()
        return (v - m) / torch.sqrt(((v - m) ** 2).mean() + cfg.layer_norm_epsilon) * f(g) + f(b)

    for l, lw in enumerate(w.layers):
        h = ln(x, lw.ln1_g, lw.ln1_b)
        qkv = torch.zeros(3 * d, dtype=torch.float64)
        for cu in cus:  # every CU: its W_qkv rows
            for i in range(cu.nq):
                qkv[cu.q0 + i] = f(lw.w_qkv[cu.q0 + i]) @ h + f(lw.b_qkv[cu.q0 + i])
        xa = x.clone() + f(lw.b_o)  # every CU adds the bias to its own residual copy
        for cu in cus:
            if cu.ah < 0:
                continue
            hh = cu.ah
            q = qkv[hh * 64:(hh + 1) * 64]
            K = torch.cat([f(kv[l][0][hh]), qkv[d + hh * 64: d + (hh + 1) * 64][None]])
            V = torch.cat([f(kv[l][1][hh]), qkv[2 * d + hh * 64: 2 * d + (hh + 1) * 64][None]])
            p = torch.softmax(K @ q / 8.0, dim=0)
            o = p @ V
            for k in range(cu.nk):  # axpy of this CU's W_o^T rows
                xa += o[cu.ak0 + k] * f(lw.w_o[:, hh * 64 + cu.ak0 + k])
        h2 = ln(xa, lw.ln2_g, lw.ln2_b)
        xm = xa + f(lw.b_p)
        for cu in cus:
            for i in range(cu.nf):
                j = cu.f0 + i
                a = f(lw.w_fc[j]) @ h2 + f(lw.b_fc[j])
                g = 0.5 * a * (1 + torch.tanh(0.7978845608028654 * (a + 0.044715 * a ** 3)))
                xm += g * f(lw.w_p[:, j])
        x = xm
    return ln(x, w.lnf_g, w.lnf_b)


def test_split_reproduces_the_reference_step():
    """The per-CU decomposition (QKV rows, head-dim slices of W_o, c_fc/c_proj pairs, base adds)
    sums to exactly the reference forward (float64, no rounding)."""
    from distributed_lms_raft_llm_amd.engine.weights import prepare_gpt2_weights
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, KVCache, init_gpt2_weights, perturb_norms_and_biases

    cfg = GPT2Config("df-emul", n_layer=2, n_embd=128, n_head=2, n_positions=32, vocab_size=200, eos_token_id=199)
    raw = init_gpt2_weights(cfg, seed=5)
    perturb_norms_and_biases(raw)
    w = prepare_gpt2_weights(cfg, raw, "cpu", dtype=torch.float32)
    cus = assign(cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded, 8, 2)
    ref = GPT2Reference(cfg, raw, device="cpu", dtype=torch.float64)
    seq = [5, 17, 42, 7]
    cache = KVCache.allocate(cfg, 1, 8, dtype=torch.float64, device="cpu")
    toks = torch.tensor([seq])
    hid = ref.forward(toks, torch.arange(len(seq))[None], cache, torch.zeros(1, dtype=torch.long))[0]
    # K/V of the first 3 positions from the reference cache: [H, 3, 64] per layer
    kv = [(cache.data[l, 0, 0, :, :3], cache.data[l, 1, 0, :, :3]) for l in range(cfg.n_layer)]
    got = _emulate_step(cfg, w, cus, seq[3], 3, kv)
    torch.testing.assert_close(got, hid[-1].double(), atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("name,G,window", [
    ("gpt2", 256, 4 * 16 * 1568),            # the LM head's NC in-flight 16-row groups
    ("gpt2-medium", 256, 4 * 16 * 2080),     # 133 KiB: fits the 144 KiB ring at 1 row only
    ("gpt2-medium", 128, 4 * 16 * 2080),     # ... and its c_fc rows + c_proj block need 132096 B
])
def test_ring_window(name, G, window):
    """The stream window a compute wave needs resident (ops/dataflow.py ring_window): the
    gpt2-medium launches that stalled on the GPU (profiles/r3_df_hang_probe.jsonl) are exactly
    those whose window + one 8 KiB loader batch exceeds the ring."""
    from distributed_lms_raft_llm_amd.ops.dataflow import ring_window

    cfg = gpt2_config(name)
    cus = assign(cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded, G, 4)
    ko, kf = block_k(cus)
    assert ring_window(cus, cfg.n_embd, ko, kf) == window
    if G == 128:  # the r3 loader stall at layer 4: the MLP window alone overflows the old ring
        assert max(cu.nf for cu in cus) * 2080 + cfg.n_embd * kf * 2 + 8192 > 139264
    # the r3 probe: medium at 256 CUs with the old 139264 B ring (hb staged 16 rows) stalls
    assert ring_window(cus, cfg.n_embd, ko, kf) + 8192 > 139264 or name == "gpt2"
