"""CPU checks of the persistent dataflow decode's work split and packed weight streams
(ops/dataflow.py): every weight row is owned by exactly one CU and sits in that CU's stream in
the order the kernel consumes it."""
import numpy as np
import pytest
import torch

from distributed_lms_raft_llm_amd.models.config import GPT2Config, gpt2_config
from distributed_lms_raft_llm_amd.ops.dataflow import ROW_PAD, assign, block_k, pack_weights


@pytest.mark.parametrize("split", ["dims", "outputs"])
@pytest.mark.parametrize("name,G,GS,J", [("gpt2", 256, 4, 1), ("gpt2", 200, 2, 4), ("gpt2-medium", 200, 2, 2),
                                         ("gpt2-xl", 256, 4, 1), ("gpt2-xl", 200, 2, 1), ("gpt2-large", 200, 2, 1),
                                         ("gpt2-tiny", 64, 4, 2), ("gpt2", 80, 2, 1)])
def test_assignment_covers_every_row_once(name, G, GS, J, split):
    """Every W_qkv row and LM-head row on exactly one CU; every (intermediate column, output column)
    pair of c_proj on exactly one CU (the J CUs of a slice split its outputs); every (head, output
    column) of W_o on exactly one attention CU; and the per-copy contribution counts the kernel
    polls for hold for EVERY residual word."""
    from distributed_lms_raft_llm_amd.ops.dataflow import expected_contributions

    cfg = gpt2_config(name)
    d, H, F, V = cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded
    C = 2
    cus = assign(d, H, F, V, G, GS, J, C, split)
    assert len(cus) == G
    for key, n in (("q", 3 * d), ("v", V)):
        covered = np.zeros(n, dtype=int)
        for cu in cus:
            s, c = getattr(cu, key + "0"), getattr(cu, "n" + key)
            covered[s: s + c] += 1
        assert (covered == 1).all(), key
    cp = np.zeros((F, d), dtype=int)
    per_word = np.zeros((C, d), dtype=int)
    for cu in cus:
        cp[cu.f0: cu.f0 + cu.nf, cu.pd0: cu.pd0 + cu.pdn] += 1
        per_word[cu.mcp, cu.pd0: cu.pd0 + cu.pdn] += 1
    assert (cp == 1).all()
    cov = np.zeros((H, 64, d), dtype=int)  # (head, head dim, output column) of W_o
    att_word = np.zeros((C, d), dtype=int)
    att = [cu for cu in cus if cu.ah >= 0]
    assert len(att) == H * GS
    for cu in att:
        cov[cu.ah, cu.ak0: cu.ak0 + cu.akn, cu.ao0: cu.ao0 + cu.aon] += 1
        att_word[cu.acp, cu.ao0: cu.ao0 + cu.aon] += 1
    assert (cov == 1).all()
    exp_att, exp_mlp = expected_contributions(cus, C)
    for c in range(C):
        assert (att_word[c] == exp_att[c]).all() and (per_word[c] == exp_mlp[c]).all()
    assert sum(exp_att) == (H if split == "outputs" else H * GS) and sum(exp_mlp) == G // J
    assert max(cu.nq for cu in cus) <= 64 and max(cu.nf for cu in cus) <= 64


def test_assignment_rejects_bad_split():
    with pytest.raises(ValueError):
        assign(768, 12, 3072, 50304, 16, 4)  # 48 attention CUs on 16
    with pytest.raises(ValueError):
        assign(768, 12, 3072, 50304, 256, 5)  # 5 does not split a head's 64 dims
    with pytest.raises(ValueError):
        assign(768, 12, 3072, 50304, 200, 2, 3)  # J must divide G


def test_packed_stream_matches_sources():
    from distributed_lms_raft_llm_amd.engine.weights import prepare_gpt2_weights
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    cfg = GPT2Config("df-test", n_layer=2, n_embd=128, n_head=2, n_positions=64, vocab_size=300, eos_token_id=299)
    w = prepare_gpt2_weights(cfg, init_gpt2_weights(cfg, seed=3), "cpu")
    G, GS, J = 16, 4, 2
    cus = assign(cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded, G, GS, J)  # (dims split: ko 16)
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
            if cu.ah >= 0:
                blk = packed[o: o + cu.aon * ko].reshape(cu.aon, ko)  # K-major: [outputs][head dims]
                k0 = cu.ah * 64 + cu.ak0
                assert torch.equal(blk[:, : cu.akn], lw.w_o[cu.ao0: cu.ao0 + cu.aon, k0: k0 + cu.akn])
                assert not blk[:, cu.akn:].any()
                o += cu.aon * ko
            assert torch.equal(rows(o, cu.nf), lw.w_fc[cu.f0: cu.f0 + cu.nf])
            o += cu.nf * (d + ROW_PAD)
            blk = packed[o: o + cu.pdn * kf].reshape(cu.pdn, kf)
            want = lw.w_p[cu.pd0: cu.pd0 + cu.pdn, cu.f0: cu.f0 + cu.nf]
            assert torch.equal(blk[:, : cu.nf], want) and not blk[:, cu.nf:].any()
            o += cu.pdn * kf
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
            o = p @ V  # the whole head; this CU adds W_o for its output columns x head dims only
            k0 = hh * 64 + cu.ak0
            xa[cu.ao0: cu.ao0 + cu.aon] += f(lw.w_o[cu.ao0: cu.ao0 + cu.aon, k0: k0 + cu.akn]) @ o[cu.ak0: cu.ak0 + cu.akn]
        h2 = ln(xa, lw.ln2_g, lw.ln2_b)
        xm = xa + f(lw.b_p)
        for cu in cus:
            for i in range(cu.nf):
                j = cu.f0 + i
                a = f(lw.w_fc[j]) @ h2 + f(lw.b_fc[j])
                g = 0.5 * a * (1 + torch.tanh(0.7978845608028654 * (a + 0.044715 * a ** 3)))
                xm[cu.pd0: cu.pd0 + cu.pdn] += g * f(lw.w_p[cu.pd0: cu.pd0 + cu.pdn, j])
        x = xm
    return ln(x, w.lnf_g, w.lnf_b)


@pytest.mark.parametrize("split,J", [("dims", 1), ("dims", 2), ("outputs", 2)])
def test_split_reproduces_the_reference_step(split, J):
    """The per-CU decomposition (QKV rows, head-dim slices of W_o, c_fc/c_proj pairs, base adds)
    sums to exactly the reference forward (float64, no rounding)."""
    from distributed_lms_raft_llm_amd.engine.weights import prepare_gpt2_weights
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, KVCache, init_gpt2_weights, perturb_norms_and_biases

    cfg = GPT2Config("df-emul", n_layer=2, n_embd=128, n_head=2, n_positions=32, vocab_size=200, eos_token_id=199)
    raw = init_gpt2_weights(cfg, seed=5)
    perturb_norms_and_biases(raw)
    w = prepare_gpt2_weights(cfg, raw, "cpu", dtype=torch.float32)
    cus = assign(cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded, 8, 2, J, 2, split)
    ref = GPT2Reference(cfg, raw, device="cpu", dtype=torch.float64)
    seq = [5, 17, 42, 7]
    cache = KVCache.allocate(cfg, 1, 8, dtype=torch.float64, device="cpu")
    toks = torch.tensor([seq])
    hid = ref.forward(toks, torch.arange(len(seq))[None], cache, torch.zeros(1, dtype=torch.long))[0]
    # K/V of the first 3 positions from the reference cache: [H, 3, 64] per layer
    kv = [(cache.data[l, 0, 0, :, :3], cache.data[l, 1, 0, :, :3]) for l in range(cfg.n_layer)]
    got = _emulate_step(cfg, w, cus, seq[3], 3, kv)
    torch.testing.assert_close(got, hid[-1].double(), atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("name,G,GS,window", [
    ("gpt2", 256, 4, 16 * 1568),             # one 16-row LM-head group (waves release ahead of it)
    ("gpt2-medium", 256, 4, 16 * 2080),      # c_fc rows and LM-head group tie
    ("gpt2-medium", 128, 4, 32 * 2080),      # 32 c_fc rows (the c_proj block no longer adds to them)
    ("gpt2-large", 200, 2, 1280 * 32 * 2),   # the W_o / c_proj blocks, K padded to 32
    ("gpt2-xl", 200, 2, 32 * 3232),          # 32 c_fc rows of 3.2 KB
])
def test_ring_window(name, G, GS, window):
    """The stream window a compute wave needs resident (ops/dataflow.py ring_window).  The
    c_fc rows are released before the wait for the c_proj block and each LM-head wave releases
    everything before its next group, so the window is the largest SINGLE piece: GPT-2-large
    and XL now fit the ring (the old "c_fc + c_proj together, NC LM-head groups" rule needed
    150-207 KB there), with the one 8 KiB loader batch of slack every launch needs."""
    from distributed_lms_raft_llm_amd.ops.dataflow import ring_window

    cfg = gpt2_config(name)
    cus = assign(cfg.n_embd, cfg.n_head, cfg.n_inner, cfg.vocab_padded, G, GS)
    ko, kf = block_k(cus)
    assert ring_window(cus, cfg.n_embd, ko, kf) == window
    # 139264 B: the smallest ring any supported width gets at one row (160 KiB minus the fixed
    # LDS areas, rounded down to the 8 KiB loader batch)
    assert ring_window(cus, cfg.n_embd, ko, kf) + 8192 <= 139264
