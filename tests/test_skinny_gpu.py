"""Numerics of the latency-path kernels (ops/csrc/skinny.hip) against plain PyTorch fp32
references: pre-shuffled-weight MFMA GEMMs for M <= 32 rows with their fused LayerNorm prologue
and epilogues, and the split-K flash-decode attention (SURVEY.md §4.3 "Kernel unit")."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from distributed_lms_raft_llm_amd import ops

    ops.lib()
    return ops


def _rand(*shape, scale=1.0, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype).to(DEV)


def _ln_ref(x, g, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[1],), g, b, eps)


@pytest.mark.parametrize("M", [1, 3, 16, 17, 32])
@pytest.mark.parametrize("N,K", [(768, 768), (2304, 768), (3072, 1024), (4800, 1600)])
def test_skinny_ln_bf16(M, N, K):
    ops = _ops()
    x = _rand(M, K, seed=1, dtype=torch.float32) * 3 + 0.5
    g, b = _rand(K, seed=2, dtype=torch.float32), _rand(K, seed=3, dtype=torch.float32)
    w = _rand(N, K, scale=0.05, seed=4)
    bias = _rand(N, seed=5, dtype=torch.float32)
    out = ops.skinny_gemm(x, ops.shuffle_weight(w), ops.EPI_BF16, ln=(g, b, 1e-5), bias=bias)
    h = _ln_ref(x, g, b, 1e-5).to(torch.bfloat16).float()
    ref = h @ w.float().t() + bias
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 8, 32])
def test_skinny_ln_gelu(M):
    ops = _ops()
    N, K = 3072, 768
    x = _rand(M, K, seed=11, dtype=torch.float32)
    g, b = _rand(K, seed=12, dtype=torch.float32), _rand(K, seed=13, dtype=torch.float32)
    w = _rand(N, K, scale=0.05, seed=14)
    bias = _rand(N, seed=15, dtype=torch.float32) * 0.1
    out = ops.skinny_gemm(x, ops.shuffle_weight(w), ops.EPI_GELU_TANH, ln=(g, b, 1e-5), bias=bias)
    h = _ln_ref(x, g, b, 1e-5).to(torch.bfloat16).float()
    ref = torch.nn.functional.gelu(h @ w.float().t() + bias, approximate="tanh")
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 7, 16, 29])
@pytest.mark.parametrize("N,K", [(768, 768), (768, 3072), (1024, 4096), (1600, 6400)])
def test_skinny_residual_inplace(M, N, K):
    ops = _ops()
    a = _rand(M, K, seed=21)
    w = _rand(N, K, scale=0.02, seed=22)
    bias = _rand(N, seed=23, dtype=torch.float32)
    x = _rand(M, N, seed=24, dtype=torch.float32)
    ref = x + a.float() @ w.float().t() + bias
    ops.skinny_gemm(a, ops.shuffle_weight(w), ops.EPI_F32, bias=bias, out=x)
    torch.testing.assert_close(x, ref, atol=1e-2, rtol=1e-3)


def test_skinny_partial():
    ops = _ops()
    M, N, K = 4, 768, 3072
    a, w = _rand(M, K, seed=31), _rand(N, K, scale=0.02, seed=32)
    out = ops.skinny_gemm(a, ops.shuffle_weight(w), ops.EPI_PARTIAL)
    torch.testing.assert_close(out, a.float() @ w.float().t(), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("M", [1, 5, 32])
def test_skinny_qkv_scatter(M):
    ops = _ops()
    H, T, S = 12, 40, 40
    D = H * 64
    x = _rand(M, D, seed=41, dtype=torch.float32)
    g, b = _rand(D, seed=42, dtype=torch.float32), _rand(D, seed=43, dtype=torch.float32)
    w = _rand(3 * D, D, scale=0.05, seed=44)
    bias = _rand(3 * D, seed=45, dtype=torch.float32)
    q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    gen = torch.Generator().manual_seed(46)
    slot = torch.randperm(S, generator=gen)[:M].to(torch.int32).to(DEV)
    pos = torch.randint(0, T, (M,), generator=gen).to(torch.int32).to(DEV)
    ops.skinny_gemm(x, ops.shuffle_weight(w), ops.EPI_QKV, ln=(g, b, 1e-5), bias=bias, q_out=q, k_cache=kc,
                    v_cache=vc, row_slot=slot, row_pos=pos)
    h = _ln_ref(x, g, b, 1e-5).to(torch.bfloat16).float()
    z = h @ w.float().t() + bias
    torch.testing.assert_close(q.float(), z[:, :D], atol=3e-2, rtol=2e-2)
    for r in range(M):
        s, p = int(slot[r]), int(pos[r])
        torch.testing.assert_close(kc[s, :, p].float().reshape(-1), z[r, D:2 * D], atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(vc[s, :, p].float().reshape(-1), z[r, 2 * D:], atol=3e-2, rtol=2e-2)
    # nothing else written
    mask = torch.zeros(S, T, dtype=torch.bool, device=DEV)
    mask[slot.long(), pos.long()] = True
    assert kc.permute(0, 2, 1, 3)[~mask].abs().sum() == 0


@pytest.mark.parametrize("M", [1, 6, 32])
def test_skinny_argmax_penalty(M):
    """Keys equal the fp32 argmax of the penalised logits wherever the top-2 margin is clear."""
    ops = _ops()
    V, Vp, K = 3000, 3008 + 64, 768  # padded vocabulary: columns >= V never win
    Vp = (Vp + 63) // 64 * 64
    h = _rand(M, K, seed=51)
    w = _rand(Vp, K, scale=0.05, seed=52)
    words = Vp // 32
    gen = torch.Generator().manual_seed(53)
    seen_ids = [torch.randint(0, V, (20,), generator=gen) for _ in range(M)]
    seen = torch.zeros(M, words, dtype=torch.int32)
    for r, ids in enumerate(seen_ids):
        for t in ids.tolist():
            seen[r, t // 32] |= (1 << (t % 32)) if t % 32 < 31 else -(1 << 31)
    seen = seen.to(DEV)
    keys = torch.zeros(M, Vp // 64, dtype=torch.int64, device=DEV)
    ops.skinny_gemm(h, ops.shuffle_weight(w), ops.EPI_ARGMAX, argmax_out=keys, seen=seen, vocab=V, penalty=1.2)
    tok = ops.argmax_reduce(keys)
    idx = (~(tok & 0xFFFFFFFF)).to(torch.int64) & 0xFFFFFFFF
    logits = h.float() @ w.float().t()
    logits[:, V:] = -float("inf")
    for r, ids in enumerate(seen_ids):
        u = torch.unique(ids).to(DEV)
        v = logits[r, u]
        logits[r, u] = torch.where(v < 0, v * 1.2, v / 1.2)
    top2 = logits.topk(2, dim=1)
    clear = (top2.values[:, 0] - top2.values[:, 1]) > 1e-2
    assert clear.any()
    assert torch.equal(idx[clear].cpu(), top2.indices[clear, 0].cpu())


@pytest.mark.parametrize("M", [1, 5])
def test_skinny_argmax_with_ln_prologue(M):
    """ln_f fused into the skinny LM head: keys == those of the bf16 LN output fed to the same kernel."""
    ops = _ops()
    V, K = 3000, 768
    Vp = (V + 63) // 64 * 64
    x = _rand(M, K, seed=131, dtype=torch.float32) * 2 + 0.3
    g, b = _rand(K, seed=132, dtype=torch.float32), _rand(K, seed=133, dtype=torch.float32)
    w_sh = ops.shuffle_weight(_rand(Vp, K, scale=0.05, seed=134))
    seen = torch.zeros(M, Vp // 32, dtype=torch.int32, device=DEV)
    seen[:, 3] = 0x0F0F0F0F
    k1 = torch.zeros(M, Vp // 64, dtype=torch.int64, device=DEV)
    k2 = torch.zeros_like(k1)
    ops.skinny_gemm(x, w_sh, ops.EPI_ARGMAX, ln=(g, b, 1e-5), argmax_out=k1, seen=seen, vocab=V, penalty=1.2)
    h = _ln_ref(x, g, b, 1e-5).to(torch.bfloat16)
    ops.skinny_gemm(h, w_sh, ops.EPI_ARGMAX, argmax_out=k2, seen=seen, vocab=V, penalty=1.2)
    # the prologue's LN rounds to bf16 like the reference up to last-bit ties, so compare the
    # winning columns per 64-column group (nearly all equal) and the per-row argmax
    cols1, cols2 = (~k1) & 0xFFFFFFFF, (~k2) & 0xFFFFFFFF
    assert (cols1 == cols2).float().mean().item() > 0.97
    assert torch.equal((~ops.argmax_reduce(k1)) & 0xFFFFFFFF, (~ops.argmax_reduce(k2)) & 0xFFFFFFFF)


def _attn_ref(q, kc, vc, slot, kvlen):
    R = q.shape[0]
    H = kc.shape[1]
    out = torch.empty(R, H * 64, device=DEV)
    for r in range(R):
        s, n = int(slot[r]), int(kvlen[r])
        k = kc[s, :, :n].float()  # [H, n, 64]
        v = vc[s, :, :n].float()
        qq = q[r].float().reshape(H, 1, 64)
        p = torch.softmax((qq @ k.transpose(1, 2)) / 8.0, dim=-1)
        out[r] = (p @ v).reshape(-1)
    return out


@pytest.mark.parametrize("B,T", [(1, 1024), (8, 1024), (3, 150), (16, 37)])
@pytest.mark.parametrize("waves", [2, 4, 16])
def test_attention_split(B, T, waves):
    ops = _ops()
    H, S = 12, max(B, 4)
    kc = _rand(S, H, T, 64, seed=61)
    vc = _rand(S, H, T, 64, seed=62)
    q = _rand(B, H * 64, seed=63)
    gen = torch.Generator().manual_seed(64)
    slot = torch.randperm(S, generator=gen)[:B].to(torch.int32).to(DEV)
    kvlen = torch.randint(1, T + 1, (B,), generator=gen)
    kvlen[0] = T
    kvlen = kvlen.to(torch.int32).to(DEV)
    out = ops.attention_split(q, kc, vc, slot, kvlen, waves=waves)
    ref = _attn_ref(q, kc, vc, slot, kvlen)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("B,T", [(1, 1024), (8, 1024), (2, 700), (3, 150)])
@pytest.mark.parametrize("waves,splits", [(4, 3), (4, 8), (2, 16), (8, 64), (4, 0)])
@pytest.mark.parametrize("sync", [0, 2])
def test_attention_split_across_workgroups(B, T, waves, splits, sync):
    """Keys split over several workgroups per (row, head), merged by the last to arrive: matches
    fp32 at T=1024 / B=1 and 8 (splits=0: the engine's geometry); re-running on the same
    workspace (counters re-armed by the kernel) gives bit-identical output."""
    ops = _ops()
    H, S = 12, max(B, 4)
    if splits == 0:
        waves, splits = ops.attention_split_geometry(B * H, T)
    kc = _rand(S, H, T, 64, seed=91)
    vc = _rand(S, H, T, 64, seed=92)
    q = _rand(B, H * 64, seed=93)
    gen = torch.Generator().manual_seed(94)
    slot = torch.randperm(S, generator=gen)[:B].to(torch.int32).to(DEV)
    kvlen = torch.randint(1, T + 1, (B,), generator=gen)
    kvlen[0] = T
    if B > 2:
        kvlen[1] = 1  # most workgroups of this row see no keys
    kvlen = kvlen.to(torch.int32).to(DEV)
    ws = ops.AttnSplitWorkspace(B * H, splits, DEV)
    out = ops.attention_split(q, kc, vc, slot, kvlen, waves=waves, splits=splits, workspace=ws, sync=sync)
    ref = _attn_ref(q, kc, vc, slot, kvlen)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    assert int(ws.counters.abs().sum()) == 0
    for _ in range(3):
        again = ops.attention_split(q, kc, vc, slot, kvlen, waves=waves, splits=splits, workspace=ws, sync=sync)
        assert torch.equal(again, out)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("H,T", [(12, 150), (12, 37), (16, 512), (20, 150), (25, 100)])
def test_attention_oproj(M, H, T):
    """Fused decode attention + out-projection: slab h == fp32 attention of head h -> bf16 ->
    @ W_o[:, head h]^T, and the slabs sum to the full out-projection."""
    ops = _ops()
    N, S = H * 64, 6
    kc, vc = _rand(S, H, T, 64, seed=101), _rand(S, H, T, 64, seed=102)
    q = _rand(M, H * 64, seed=103)
    wo = _rand(N, H * 64, scale=0.05, seed=104)
    gen = torch.Generator().manual_seed(105)
    slot = torch.randperm(S, generator=gen)[:M].to(torch.int32).to(DEV)
    kvlen = torch.randint(1, T + 1, (M,), generator=gen)
    kvlen[0] = T
    kvlen = kvlen.to(torch.int32).to(DEV)
    parts = torch.full((H, 4, N), 7.0, device=DEV)
    ops.attention_oproj(q, kc, vc, slot, kvlen, ops.shuffle_weight(wo), parts)
    o = _attn_ref(q, kc, vc, slot, kvlen).to(torch.bfloat16).float().reshape(M, H, 64)
    for h in range(H):
        ref_h = o[:, h] @ wo.float()[:, 64 * h:64 * h + 64].t()
        torch.testing.assert_close(parts[h, :M], ref_h, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(parts[:, :M].sum(0), o.reshape(M, -1) @ wo.float().t(), atol=5e-2, rtol=2e-2)
    assert torch.all(parts[:, M:] == 7.0)  # rows >= M untouched


@pytest.mark.parametrize("H,hg,tiles", [(12, 3, 3), (12, 3, 1), (16, 4, 4), (16, 4, 2), (12, 4, 3)])
@pytest.mark.parametrize("T", [1, 37, 150])
def test_attention_oproj_grouped(H, hg, tiles, T):
    """One row, heads in groups of hg: slab g == sum over its heads of attn_h(q) -> bf16 -> @ W_o[:, h]^T."""
    ops = _ops()
    N, S = H * 64, 5
    kc, vc = _rand(S, H, T, 64, seed=121), _rand(S, H, T, 64, seed=122)
    q = _rand(1, H * 64, seed=123)
    wo = _rand(N, H * 64, scale=0.05, seed=124)
    slot = torch.tensor([3], dtype=torch.int32, device=DEV)
    kvlen = torch.tensor([T], dtype=torch.int32, device=DEV)
    parts = torch.full((H // hg, 2, N), 7.0, device=DEV)
    ops.attention_oproj_grouped(q, kc, vc, slot, kvlen, ops.shuffle_weight(wo), parts, hg, tiles=tiles)
    o = _attn_ref(q, kc, vc, slot, kvlen).to(torch.bfloat16).float().reshape(H, 64)
    for g in range(H // hg):
        ref = sum(o[h] @ wo.float()[:, 64 * h:64 * h + 64].t() for h in range(g * hg, g * hg + hg))
        torch.testing.assert_close(parts[g, 0], ref, atol=3e-2, rtol=2e-2)
    assert torch.all(parts[:, 1] == 7.0)


@pytest.mark.parametrize("ns", [12, 16])
def test_skinny_addln_many_slabs(ns):
    """The fused add+LN consumes 12 / 16 per-head slabs (fixed order) like 4."""
    ops = _ops()
    M, K, N = 3, 768 if ns == 12 else 1024, 3072
    x = _rand(M, K, seed=111, dtype=torch.float32)
    parts = _rand(ns, M, K, seed=112, dtype=torch.float32) * 0.3
    rb = _rand(K, seed=113, dtype=torch.float32)
    g, b = _rand(K, seed=114, dtype=torch.float32), _rand(K, seed=115, dtype=torch.float32)
    w = _rand(N, K, scale=0.05, seed=116)
    bias = _rand(N, seed=117, dtype=torch.float32) * 0.1
    x_out = torch.zeros_like(x)
    out = ops.skinny_addln_gemm(x, ops.shuffle_weight(w), ops.EPI_GELU_TANH, g, b, 1e-5, x_out=x_out, parts=parts,
                                nsplit=ns, res_bias=rb, bias=bias)
    v = x + rb + parts.sum(0)
    torch.testing.assert_close(x_out, v, atol=1e-5, rtol=1e-5)
    h = _ln_ref(v, g, b, 1e-5).to(torch.bfloat16).float()
    ref = torch.nn.functional.gelu(h @ w.float().t() + bias, approximate="tanh")
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


def test_attention_split_matches_wave_kernel():
    """Split-K and the one-wave-per-(row, head) kernel agree (same online-softmax numerics)."""
    ops = _ops()
    B, H, T = 5, 12, 150
    kc, vc = _rand(B, H, T, 64, seed=71), _rand(B, H, T, 64, seed=72)
    q = _rand(B, H * 64, seed=73)
    slot = torch.arange(B, dtype=torch.int32, device=DEV)
    kvlen = torch.tensor([1, 9, 64, 100, 150], dtype=torch.int32, device=DEV)
    a = ops.attention_split(q, kc, vc, slot, kvlen, waves=8)
    b = ops.row_attention(q, kc, vc, slot, kvlen)
    torch.testing.assert_close(a.float(), b.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("M", [1, 4, 5, 8])
@pytest.mark.parametrize("K", [768, 1024, 1280, 1600])
@pytest.mark.parametrize("nsplit", [0, 1, 4])
def test_skinny_addln_gelu(M, K, nsplit):
    """v = x + res_bias + sum(parts); x_out = v; out = gelu(LN(v) @ W.T + b)."""
    ops = _ops()
    if M > ops.skinny_addln_max_rows(K):
        pytest.skip("row count above this width's fused-kernel limit")
    N = 4 * K
    x = _rand(M, K, seed=81, dtype=torch.float32)
    parts = _rand(4, M, K, seed=82, dtype=torch.float32)
    rb = _rand(K, seed=83, dtype=torch.float32)
    g, b = _rand(K, seed=84, dtype=torch.float32), _rand(K, seed=85, dtype=torch.float32)
    w = _rand(N, K, scale=0.05, seed=86)
    bias = _rand(N, seed=87, dtype=torch.float32) * 0.1
    x_out = torch.full_like(x, 7.0)
    out = ops.skinny_addln_gemm(x, ops.shuffle_weight(w), ops.EPI_GELU_TANH, g, b, 1e-5, x_out=x_out, parts=parts,
                                nsplit=nsplit, res_bias=rb, bias=bias)
    v = x + rb + parts[:nsplit].sum(0)
    torch.testing.assert_close(x_out, v, atol=1e-5, rtol=1e-5)
    h = _ln_ref(v, g, b, 1e-5).to(torch.bfloat16).float()
    ref = torch.nn.functional.gelu(h @ w.float().t() + bias, approximate="tanh")
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 3, 8])
def test_skinny_addln_qkv(M):
    ops = _ops()
    H, T, S = 12, 20, 16
    D = 64 * H
    x = _rand(M, D, seed=91, dtype=torch.float32)
    g, b = _rand(D, seed=92, dtype=torch.float32), _rand(D, seed=93, dtype=torch.float32)
    w = _rand(3 * D, D, scale=0.05, seed=94)
    bias = _rand(3 * D, seed=95, dtype=torch.float32)
    q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    slot = torch.arange(M, dtype=torch.int32, device=DEV) * 2
    pos = torch.arange(M, dtype=torch.int32, device=DEV) + 3
    ops.skinny_addln_gemm(x, ops.shuffle_weight(w), ops.EPI_QKV, g, b, 1e-5, bias=bias, q_out=q, k_cache=kc,
                          v_cache=vc, row_slot=slot, row_pos=pos)
    h = _ln_ref(x, g, b, 1e-5).to(torch.bfloat16).float()
    z = h @ w.float().t() + bias
    torch.testing.assert_close(q.float(), z[:, :D], atol=3e-2, rtol=2e-2)
    for r in range(M):
        s, p = int(slot[r]), int(pos[r])
        torch.testing.assert_close(kc[s, :, p].float().reshape(-1), z[r, D:2 * D], atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(vc[s, :, p].float().reshape(-1), z[r, 2 * D:], atol=3e-2, rtol=2e-2)


def _to_fix(x):
    """f32 [M, K] -> fixed point [fix_copies(), M, K], spread over the copies (readers must sum them)."""
    from distributed_lms_raft_llm_amd import ops

    C = ops.fix_copies()
    total = torch.round(x.double() * ops.FIX_SCALE).to(torch.int64)
    share = total // C
    out = share.unsqueeze(0).repeat(C, 1, 1)
    out[0] += total - share * C
    return out.contiguous()


@pytest.mark.parametrize("M", [1, 2, 5, 8])
@pytest.mark.parametrize("K", [768, 1024, 1280, 1600])
@pytest.mark.parametrize("nsplit,xfix", [(4, False), (4, True), (0, True), (0, False)])
def test_skinny_mlp(M, K, nsplit, xfix, cg=0):
    """Fused MLP: r_out += fix(v + gelu(LN(v) W_fc^T + b_fc) W_p^T + b_p), v = x + res_bias + sum(parts),
    against fp32 (with the same bf16 roundings of LN(v) and h), and bit-identical over repeated launches
    (the workgroups' 64-bit integer atomics commute).  GPT-2 small .. XL widths (r3)."""
    ops = _ops()
    if nsplit and K > 1024:
        pytest.skip("head-group slabs: d <= 1024 only")
    if ops.skinny_mlp_cg(K, M, cg) == 0:
        pytest.skip(f"{M} rows of width {K} do not fit the fused MLP")
    F = 4 * K
    x = _rand(M, K, seed=201, dtype=torch.float32) * 2
    parts = _rand(4, M, K, seed=202, dtype=torch.float32) * 0.5
    rb = _rand(K, seed=203, dtype=torch.float32)
    g, b = _rand(K, seed=204, dtype=torch.float32), _rand(K, seed=205, dtype=torch.float32)
    w_fc = _rand(F, K, scale=0.05, seed=206)
    b_fc = _rand(F, seed=207, dtype=torch.float32) * 0.1
    w_p = _rand(K, F, scale=0.03, seed=208)
    b_p = _rand(K, seed=209, dtype=torch.float32) * 0.1
    x_in = _to_fix(x) if xfix else x
    x_used = ops.fix_to_float(x_in) if xfix else x
    w_fc_sh, w_p_sl = ops.shuffle_weight(w_fc), ops.slice_cproj(w_p)
    outs = []
    for _ in range(3):
        r = torch.zeros(ops.fix_copies(), M, K, dtype=torch.int64, device=DEV)
        ops.skinny_mlp(x_in, g, b, 1e-5, w_fc_sh, b_fc, w_p_sl, b_p, r, parts=parts if nsplit else None,
                       nsplit=nsplit, res_bias=rb, cg=cg)
        outs.append(r)
    assert all(torch.equal(outs[0], o) for o in outs[1:]), "fixed-point accumulation must be order-independent"
    v = x_used + rb + parts[:nsplit].sum(0)
    h = _ln_ref(v, g, b, 1e-5).to(torch.bfloat16).float()
    ff = torch.nn.functional.gelu(h @ w_fc.float().t() + b_fc, approximate="tanh").to(torch.bfloat16).float()
    ref = v + ff @ w_p.float().t() + b_p
    torch.testing.assert_close(ops.fix_to_float(outs[0]), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("K", [768, 1024, 1280, 1600])
@pytest.mark.parametrize("cg", [1, 2, 4])
@pytest.mark.parametrize("M", [1, 6])
def test_skinny_mlp_column_groups(M, K, cg):
    """Every column-group width of the fused MLP (workgroups owning 16, 32 or 64 intermediate
    columns) against the fp32 reference (narrowed to what fits the LDS at this width)."""
    test_skinny_mlp(M, K, 0, False, cg=cg)


def test_skinny_mlp_adds_into_accumulator():
    """r_out is accumulated into, not overwritten: a pre-set value shows up in the result."""
    ops = _ops()
    M, K = 1, 768
    x = _rand(M, K, seed=211, dtype=torch.float32)
    g, b = _rand(K, seed=212, dtype=torch.float32), _rand(K, seed=213, dtype=torch.float32)
    w_fc, w_p = _rand(4 * K, K, scale=0.05, seed=214), _rand(K, 4 * K, scale=0.03, seed=215)
    b_fc, b_p = torch.zeros(4 * K, device=DEV), torch.zeros(K, device=DEV)
    args = (g, b, 1e-5, ops.shuffle_weight(w_fc), b_fc, ops.slice_cproj(w_p), b_p)
    C = ops.fix_copies()
    r0 = torch.zeros(C, M, K, dtype=torch.int64, device=DEV)
    ops.skinny_mlp(x, *args, r0)
    r1 = torch.full((C, M, K), 5 << 32, dtype=torch.int64, device=DEV)
    ops.skinny_mlp(x, *args, r1)
    assert torch.equal(r1.sum(0) - r0.sum(0), torch.full_like(r0[0], C * (5 << 32)))


@pytest.mark.parametrize("M", [1, 3])
def test_skinny_addln_qkv_fixed_point_and_zero(M):
    """QKV from the int64 fixed-point residual (the fused MLP's output) equals QKV from the same
    residual in f32, and the kernel clears the side buffer it is handed."""
    ops = _ops()
    H, T, S = 12, 20, 16
    D = 64 * H
    x = _rand(M, D, seed=221, dtype=torch.float32) * 3
    xf = _to_fix(x)
    x32 = ops.fix_to_float(xf)
    g, b = _rand(D, seed=222, dtype=torch.float32), _rand(D, seed=223, dtype=torch.float32)
    w = ops.shuffle_weight(_rand(3 * D, D, scale=0.05, seed=224))
    bias = _rand(3 * D, seed=225, dtype=torch.float32)
    res = []
    for xin in (x32, xf):
        q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
        kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros_like(kc)
        zero = torch.full((ops.fix_copies(), M, D), 123, dtype=torch.int64, device=DEV)
        slot = torch.arange(M, dtype=torch.int32, device=DEV) * 2
        pos = torch.arange(M, dtype=torch.int32, device=DEV) + 3
        ops.skinny_addln_gemm(xin, w, ops.EPI_QKV, g, b, 1e-5, bias=bias, q_out=q, k_cache=kc, v_cache=vc,
                              row_slot=slot, row_pos=pos, zero=zero)
        assert int(zero.abs().sum()) == 0
        res.append((q, kc, vc))
    for a, c in zip(res[0], res[1]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("M", [1, 2, 5])
def test_skinny_fixed_point_residual_add(M):
    """EPI_F32 into an int64 residual: copy 0 += fix(a W^T + b), column-owning and in place."""
    ops = _ops()
    N, K = 768, 768
    a = _rand(M, K, seed=241)
    w = _rand(N, K, scale=0.05, seed=242)
    bias = _rand(N, seed=243, dtype=torch.float32)
    x = _rand(M, N, seed=244, dtype=torch.float32)
    xf = _to_fix(x)
    ops.skinny_gemm(a, ops.shuffle_weight(w), ops.EPI_F32, bias=bias, out=xf[0])
    ref = x + a.float() @ w.float().t() + bias
    torch.testing.assert_close(ops.fix_to_float(xf), ref, atol=2e-3, rtol=1e-3)


@pytest.mark.parametrize("M,K", [(1, 768), (3, 1024), (2, 1600)])
def test_ln_fix(M, K):
    ops = _ops()
    x = _rand(M, K, seed=231, dtype=torch.float32) * 4 + 1
    xf = _to_fix(x)
    g, b = _rand(K, seed=232, dtype=torch.float32), _rand(K, seed=233, dtype=torch.float32)
    out = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
    ops.ln_fix(xf, g, b, 1e-5, out)
    ref = _ln_ref(ops.fix_to_float(xf), g, b, 1e-5)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=1e-2)


# ---------------------------------------------------------------------------------------------
# gemm_ps: LDS-resident activation panel + pre-shuffled weights (throughput path)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("M", [1, 40, 64, 100, 512])
@pytest.mark.parametrize("geo", [(2, 1, None), (2, 2, None), (4, 2, None), (4, 1, 3)])
def test_gemm_ps_bf16_gelu(M, geo):
    ops = _ops()
    N, K = 1024, 768
    a, w = _rand(M, K, seed=101), _rand(N, K, scale=0.05, seed=102)
    bias = _rand(N, seed=103, dtype=torch.float32) * 0.1
    mt, nt, cw = geo
    cw = cw or -(-(N // (16 * nt)) // 8)
    out = ops.gemm_ps(a, ops.shuffle_weight(w), ops.EPI_GELU_TANH, bias=bias, geometry=(mt, nt, cw))
    ref = torch.nn.functional.gelu(a.float() @ w.float().t() + bias, approximate="tanh")
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,K,split", [(64, 768, 1), (300, 768, 2), (512, 3072, 4), (37, 1024, 1)])
def test_gemm_ps_partial(M, K, split):
    ops = _ops()
    N = 768
    a, w = _rand(M, K, seed=111), _rand(N, K, scale=0.02, seed=112)
    out = ops.gemm_ps(a, ops.shuffle_weight(w), ops.EPI_PARTIAL, split_k=split)
    torch.testing.assert_close(out.sum(0), a.float() @ w.float().t(), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("M", [5, 512])
def test_gemm_ps_qkv(M):
    ops = _ops()
    H, T, S = 12, 8, 600
    D = 64 * H
    a, w = _rand(M, D, seed=121), _rand(3 * D, D, scale=0.05, seed=122)
    bias = _rand(3 * D, seed=123, dtype=torch.float32)
    q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    slot = torch.randperm(S, generator=torch.Generator().manual_seed(1))[:M].to(torch.int32).to(DEV)
    pos = torch.randint(0, T, (M,), generator=torch.Generator().manual_seed(2)).to(torch.int32).to(DEV)
    ops.gemm_ps(a, ops.shuffle_weight(w), ops.EPI_QKV, bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot,
                row_pos=pos)
    z = a.float() @ w.float().t() + bias
    torch.testing.assert_close(q.float(), z[:, :D], atol=3e-2, rtol=2e-2)
    ks = kc[slot.long(), :, pos.long()].float().reshape(M, -1)
    vs = vc[slot.long(), :, pos.long()].float().reshape(M, -1)
    torch.testing.assert_close(ks, z[:, D:2 * D], atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(vs, z[:, 2 * D:], atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,K,mt", [(3, 768, 0), (64, 768, 0), (300, 768, 5), (512, 768, 0), (512, 768, 5),
                                    (512, 1024, 0), (1024, 1024, 0), (256, 1280, 0), (77, 1280, 2)])
def test_gemm_ps_argmax_matches_tiled(M, K, mt):
    """Same keys as the tiled LM head's fused penalty + argmax (identical per-element sums are not
    required: compare the decoded token wherever the fp32 top-2 margin is clear); K > 1008 (GPT-2
    medium and wider) takes 32-row panels so the panel fits in LDS.  64-row panels (K = 768) run
    the 8-k-block register chunks; 80- and 32-row panels the 4-k-block ones."""
    ops = _ops()
    V = 50257
    Vp = 50304
    h = _rand(M, K, seed=131)
    w = _rand(Vp, K, scale=0.05, seed=132)
    seen = torch.randint(-2**31, 2**31 - 1, (M, Vp // 32), generator=torch.Generator().manual_seed(3),
                         dtype=torch.int64).to(torch.int32).to(DEV)
    seen &= 0x01010101  # ~1/8 of the vocabulary penalised
    geo = ops.gemm_ps_geometry(M, Vp, ops.EPI_ARGMAX, K=K)
    if mt:  # the 80-row panel (two seen-bitmap words per lane) / 32-row panels, not the default
        geo = (mt, geo[1], max(1, 256 // -(-M // (16 * mt))))
    keys = torch.zeros(M, 8 * geo[2], dtype=torch.int64, device=DEV)
    ops.gemm_ps(h, ops.shuffle_weight(w), ops.EPI_ARGMAX, argmax_out=keys, seen=seen, vocab=V, penalty=1.2,
                geometry=geo)
    tok = ops.argmax_reduce(keys)
    got = ((~(tok & 0xFFFFFFFF)) & 0xFFFFFFFF).cpu()
    logits = h.float() @ w.float().t()
    bits = ((seen.long().unsqueeze(-1) >> torch.arange(32, device=DEV)) & 1).reshape(M, -1).bool()
    logits = torch.where(bits, torch.where(logits < 0, logits * 1.2, logits / 1.2), logits)
    logits[:, V:] = -float("inf")
    top2 = logits.topk(2, dim=1)
    clear = (top2.values[:, 0] - top2.values[:, 1]) > 1e-2
    assert clear.float().mean() > 0.5
    assert torch.equal(got[clear.cpu()], top2.indices[clear, 0].cpu())


@pytest.mark.parametrize("blocks", [1, 7, 512])
def test_attention_persist_matches_reference(blocks):
    """The persistent low-occupancy decode attention (fixed grid looping over (row, head) pairs)."""
    ops = _ops()
    B, H, T, S = 37, 12, 150, 40
    kc, vc = _rand(S, H, T, 64, seed=141), _rand(S, H, T, 64, seed=142)
    q = _rand(B, H * 64, seed=143)
    gen = torch.Generator().manual_seed(144)
    slot = torch.randperm(S, generator=gen)[:B].to(torch.int32).to(DEV)
    kvlen = torch.randint(1, T + 1, (B,), generator=gen).to(torch.int32).to(DEV)
    out = ops.row_attention(q, kc, vc, slot, kvlen, impl="persist", blocks=blocks)
    torch.testing.assert_close(out.float(), _attn_ref(q, kc, vc, slot, kvlen), atol=2e-2, rtol=2e-2)
