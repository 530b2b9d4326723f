"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op
(SURVEY.md §4.3 "Kernel unit")."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from distributed_lms_raft_llm_amd import ops

    ops.lib()
    return ops


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


@pytest.mark.parametrize("M,N,K", [(1, 64, 64), (7, 192, 128), (16, 768, 768), (33, 2304, 768), (128, 3072, 768),
                                   (130, 768, 3072), (300, 256, 512), (1000, 128, 64)])
def test_gemm_bias_bf16(M, N, K):
    ops = _ops()
    a, w = _bf(M, K, seed=1), _bf(N, K, scale=0.05, seed=2)
    bias = torch.randn(N, device=DEV)
    out = ops.gemm(a, w, ops.EPI_BF16, bias=bias)
    ref = a.float() @ w.float().t() + bias
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


def test_gemm_asymmetric_identity():
    # A = I with an asymmetric B catches a transposed C-write (cdna_hip_programming.md §3).
    ops = _ops()
    K = 64
    a = torch.eye(K, device=DEV).to(torch.bfloat16)
    w = torch.arange(K * 64, device=DEV, dtype=torch.float32).reshape(64, K).remainder(97).to(torch.bfloat16)
    out = ops.gemm(a, w, ops.EPI_BF16)
    torch.testing.assert_close(out.float(), w.float().t(), atol=0, rtol=0)


@pytest.mark.parametrize("epi", ["gelu_tanh", "gelu_erf"])
def test_gemm_gelu(epi):
    ops = _ops()
    M, N, K = 96, 3072, 768
    a, w = _bf(M, K, seed=3), _bf(N, K, scale=0.05, seed=4)
    bias = torch.randn(N, device=DEV) * 0.1
    e = ops.EPI_GELU_TANH if epi == "gelu_tanh" else ops.EPI_GELU_ERF
    out = ops.gemm(a, w, e, bias=bias)
    z = a.float() @ w.float().t() + bias
    ref = torch.nn.functional.gelu(z, approximate="tanh" if epi == "gelu_tanh" else "none")
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


def test_gemm_f32_residual_inplace():
    ops = _ops()
    M, N, K = 64, 768, 3072
    a, w = _bf(M, K, seed=5), _bf(N, K, scale=0.02, seed=6)
    bias = torch.randn(N, device=DEV)
    x = torch.randn(M, N, device=DEV)
    ref = x + a.float() @ w.float().t() + bias
    ops.gemm(a, w, ops.EPI_F32, bias=bias, out=x, resid=x)
    torch.testing.assert_close(x, ref, atol=1e-2, rtol=1e-3)


def test_gemm_qkv_scatter():
    ops = _ops()
    H, T, S = 4, 16, 3
    D = H * 64
    M = 5
    a, w = _bf(M, D, seed=7), _bf(3 * D, D, scale=0.05, seed=8)
    bias = torch.randn(3 * D, device=DEV)
    q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    slot = torch.tensor([0, 2, 2, 1, 0], dtype=torch.int32, device=DEV)
    pos = torch.tensor([3, 0, 7, 15, 4], dtype=torch.int32, device=DEV)
    ops.gemm(a, w, ops.EPI_QKV, bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot, row_pos=pos)
    ref = a.float() @ w.float().t() + bias
    torch.testing.assert_close(q.float(), ref[:, :D], atol=2e-2, rtol=2e-2)
    for m in range(M):
        s, p = int(slot[m]), int(pos[m])
        torch.testing.assert_close(kc[s, :, p].float().reshape(-1), ref[m, D:2 * D], atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(vc[s, :, p].float().reshape(-1), ref[m, 2 * D:], atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [4096, 16384])
@pytest.mark.parametrize("epi", ["bf16", "gelu_tanh", "qkv"])
def test_gemm_256_tiles_large_m(epi, M):
    """Prefill-sized GEMMs: 4096 rows take the 256x256 8-wave tile, the 1024-prompt packed prefill
    size class (>= 16384 rows) the 256x256 8-phase kernel (both counted as 256x256 launches by the
    census): bias/GELU epilogues and the QKV scatter (packed rows over 4 slots), vs fp32."""
    ops = _ops()
    K = 768
    tile = (256, 256)
    ops.gemm_tile_reset()
    if epi == "qkv":
        H, S = 4, 4
        D = H * 64
        T = M // S
        a, w = _bf(M, K if K == D else D, seed=21), _bf(3 * D, D, scale=0.05, seed=22)
        bias = torch.randn(3 * D, device=DEV)
        q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
        kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros_like(kc)
        slot = (torch.arange(M, device=DEV) // T).to(torch.int32)
        pos = (torch.arange(M, device=DEV) % T).to(torch.int32)
        ops.gemm(a, w, ops.EPI_QKV, bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot, row_pos=pos)
        ref = a.float() @ w.float().t() + bias
        torch.testing.assert_close(q.float(), ref[:, :D], atol=2e-2, rtol=2e-2)
        # cache [S][H][T][64] -> [S*T][H*64] rows in packed order
        k_rows = kc.permute(0, 2, 1, 3).reshape(M, D).float()
        v_rows = vc.permute(0, 2, 1, 3).reshape(M, D).float()
        torch.testing.assert_close(k_rows, ref[:, D:2 * D], atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(v_rows, ref[:, 2 * D:], atol=2e-2, rtol=2e-2)
        assert ops.gemm_tile_count(*tile) == 1
        return
    N = 3072
    a, w = _bf(M, K, seed=23), _bf(N, K, scale=0.05, seed=24)
    bias = torch.randn(N, device=DEV) * 0.1
    out = ops.gemm(a, w, ops.EPI_BF16 if epi == "bf16" else ops.EPI_GELU_TANH, bias=bias)
    ref = a.float() @ w.float().t() + bias
    if epi == "gelu_tanh":
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    assert ops.gemm_tile_count(*tile) == 1


@pytest.mark.parametrize("tile", [24, 25, 26])
@pytest.mark.parametrize("epi", ["gelu_tanh", "qkv"])
def test_gemm_big_modes(tile, epi):
    """The big-GEMM main-loop modes (gemm.hip MODE: REGPF = fragments of a whole K-tile in registers,
    DMA two K-tiles ahead; GROUPED = tiles in groups of 4 row tiles) on 128x128 tiles (ids 24: both,
    the prefill default; 25: GROUPED only) and the 8-phase 256x256 kernel (id 26), forced, vs fp32.  M = 4100 leaves a partial last row
    tile and a partial last tile group; the QKV scatter covers the epilogue that the prefill uses."""
    ops = _ops()
    L = ops.lib()
    M, K = 4100, 768
    L.dlms_gemm_force_tile(tile)
    try:
        if epi == "qkv":
            H, S = 4, 5
            D = H * 64
            T = 1024
            a, w = _bf(M, D, seed=61), _bf(3 * D, D, scale=0.05, seed=62)
            bias = torch.randn(3 * D, device=DEV)
            q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
            kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
            vc = torch.zeros_like(kc)
            slot = (torch.arange(M, device=DEV) // T).to(torch.int32)
            pos = (torch.arange(M, device=DEV) % T).to(torch.int32)
            ops.gemm(a, w, ops.EPI_QKV, bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot, row_pos=pos)
            ref = a.float() @ w.float().t() + bias
            torch.testing.assert_close(q.float(), ref[:, :D], atol=2e-2, rtol=2e-2)
            sl, ps = slot.long(), pos.long()
            torch.testing.assert_close(kc[sl, :, ps].reshape(M, D).float(), ref[:, D:2 * D], atol=2e-2, rtol=2e-2)
            torch.testing.assert_close(vc[sl, :, ps].reshape(M, D).float(), ref[:, 2 * D:], atol=2e-2, rtol=2e-2)
        else:
            N = 3072
            a, w = _bf(M, K, seed=63), _bf(N, K, scale=0.05, seed=64)
            bias = torch.randn(N, device=DEV) * 0.1
            out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
            ops.gemm(a, w, ops.EPI_GELU_TANH, bias=bias, out=out)
            ref = torch.nn.functional.gelu(a.float() @ w.float().t() + bias, approximate="tanh")
            torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    finally:
        L.dlms_gemm_force_tile(-1)


@pytest.mark.parametrize("split,K", [(1, 768), (1, 3072), (2, 3072), (4, 3072)])
def test_gemm_8phase_partial_slabs(split, K):
    """The 8-phase kernel's fp32 split-K slabs (out-projection / c_proj of the packed prefill) vs
    fp32, a partial last row tile included."""
    ops = _ops()
    L = ops.lib()
    M, N = 4100, 768
    a, w = _bf(M, K, seed=71), _bf(N, K, scale=0.05, seed=72)
    parts = torch.full((split, M, N), float("nan"), device=DEV)
    L.dlms_gemm_force_tile(26)
    try:
        ops.gemm(a, w, ops.EPI_PARTIAL, out=parts, split_k=split)
    finally:
        L.dlms_gemm_force_tile(-1)
    torch.testing.assert_close(parts.sum(0), a.float() @ w.float().t(), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("N,K,epi", [(2304, 768, "bf16"), (3072, 768, "gelu"), (768, 3072, "partial")])
def test_gemm_8phase_bit_identical_to_128_tiles_at_prefill_size(N, K, epi):
    """At the 1024-prompt prefill size the 8-phase kernel sums every output in the same k order as
    the 128x128 default, so the results are bit-identical -- and identical over repeated launches
    (a screen for a DMA/read race in its half-tile schedule)."""
    ops = _ops()
    L = ops.lib()
    M = 32768
    a, w = _bf(M, K, seed=73), _bf(N, K, scale=0.05, seed=74)
    bias = torch.randn(N, device=DEV) * 0.1

    def run(tile):
        L.dlms_gemm_force_tile(tile)
        try:
            if epi == "partial":
                out = torch.full((1, M, N), float("nan"), device=DEV)
                ops.gemm(a, w, ops.EPI_PARTIAL, out=out, split_k=1)
            else:
                out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
                ops.gemm(a, w, ops.EPI_GELU_TANH if epi == "gelu" else ops.EPI_BF16, bias=bias, out=out)
        finally:
            L.dlms_gemm_force_tile(-1)
        return out

    ref = run(24)
    for _ in range(4):
        got = run(26)
        assert torch.equal(got, ref)


@pytest.mark.parametrize("epi,M,N,K", [("gelu_tanh", 256, 6400, 1600), ("bf16", 300, 4096, 1024),
                                        ("qkv", 256, 3072, 1024)])
def test_gemm_wide_model_tiles(epi, M, N, K):
    """Decode GEMMs of the wider GPT-2 sizes (K >= 1024, <= 256 tiles of 128x64) take the 128x64
    3-stage tile: GELU / bias epilogues (incl. a ragged 300-row tail) and the QKV scatter, vs fp32."""
    ops = _ops()
    a, w = _bf(M, K, seed=31), _bf(N, K, scale=0.03, seed=32)
    bias = torch.randn(N, device=DEV) * 0.1
    ref = a.float() @ w.float().t() + bias
    if epi == "qkv":
        D = K
        H, S = D // 64, 2
        T = M // S
        q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
        kc = torch.zeros(S, H, T, 64, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros_like(kc)
        slot = (torch.arange(M, device=DEV) // T).to(torch.int32)
        pos = (torch.arange(M, device=DEV) % T).to(torch.int32)
        ops.gemm(a, w, ops.EPI_QKV, bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot, row_pos=pos)
        torch.testing.assert_close(q.float(), ref[:, :D], atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(kc.permute(0, 2, 1, 3).reshape(M, D).float(), ref[:, D:2 * D], atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(vc.permute(0, 2, 1, 3).reshape(M, D).float(), ref[:, 2 * D:], atol=3e-2, rtol=2e-2)
        return
    out = ops.gemm(a, w, ops.EPI_BF16 if epi == "bf16" else ops.EPI_GELU_TANH, bias=bias)
    if epi == "gelu_tanh":
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,tile", [(1, -1), (5, -1), (32, -1), (37, -1), (512, -1), (512, 26), (512, 27),
                                    (300, 27), (512, 28)])
def test_gemm_argmax_penalty(M, tile):
    """Fused penalty + argmax epilogue vs fp32.  The key buffer is pre-filled with huge stale keys,
    which a tile wider than 64 columns must zero in every 64-column group it covers (a narrower
    earlier config could have left keys there).  ``tile``: forced LM-head tiles with all rows of
    a decode half in one row tile (512x64, plain and register-staged; 256x64)."""
    ops = _ops()
    if tile >= 0:
        ops.lib().dlms_gemm_force_tile(tile)
        try:
            return _argmax_case(ops, M)
        finally:
            ops.lib().dlms_gemm_force_tile(-1)
    _argmax_case(ops, M)


def _argmax_case(ops, M):
    K, V = 768, 50257
    Vp = (V + 63) // 64 * 64
    a = _bf(M, K, seed=9)
    w = torch.zeros(Vp, K, dtype=torch.bfloat16, device=DEV)
    w[:V] = _bf(V, K, scale=0.05, seed=10)
    seen = torch.zeros(M, Vp // 32, dtype=torch.int32, device=DEV)
    logits = a.float() @ w.float().t()
    # mark the current argmax (and some others) as seen so the penalty must change the answer
    top = logits[:, :V].argmax(1)
    seen_bool = torch.zeros(M, Vp, dtype=torch.bool, device=DEV)
    seen_bool[torch.arange(M), top] = True
    seen_bool[:, :500] = True
    words = torch.zeros(M, Vp // 32, dtype=torch.int64, device=DEV)
    for bit in range(32):
        words |= seen_bool.view(M, Vp // 32, 32)[:, :, bit].long() << bit
    seen.copy_(words.to(torch.int64).where(words < 2**31, words - 2**32).to(torch.int32))
    parts = torch.full((M, Vp // 64), 2**62, dtype=torch.int64, device=DEV)
    ops.gemm(a, w, ops.EPI_ARGMAX, argmax_out=parts, seen=seen, vocab=V, penalty=1.2)
    keys = ops.argmax_reduce(parts)
    pen = torch.where(logits < 0, logits * 1.2, logits / 1.2)
    ref = torch.where(seen_bool, pen, logits)[:, :V]
    got = (~(keys & 0xFFFFFFFF)).bitwise_and(0xFFFFFFFF)
    ref_idx = ref.argmax(1)
    # allow a different index only on a numerical near-tie
    ok = (got == ref_idx) | ((ref.gather(1, got[:, None]).squeeze(1) - ref.max(1).values).abs() < 1e-3)
    assert bool(ok.all()), (got, ref_idx)


@pytest.mark.parametrize("M,D", [(1, 768), (5, 1024), (64, 1280), (33, 1600)])
def test_layernorm(M, D):
    ops = _ops()
    x = torch.randn(M, D, device=DEV) * 3 + 1
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    of = torch.empty(M, D, device=DEV)
    ob = ops.layernorm(x, g, b, 1e-5, out_f32=of)
    ref = torch.nn.functional.layer_norm(x, (D,), g, b, 1e-5)
    torch.testing.assert_close(of, ref, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ob.float(), ref, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("impl", ["wave", "lds", "persist"])
@pytest.mark.parametrize("kvlens", [[1, 5, 150], [64, 63, 65, 1024], [31, 33, 7, 2]])
def test_row_attention(kvlens, impl):
    ops = _ops()
    H, T = 5, 1024  # 5 heads: a partial last group of 4 heads per workgroup
    R = len(kvlens)
    q = _bf(R, H * 64, seed=11)
    kc = _bf(R, H, T, 64, seed=12)
    vc = _bf(R, H, T, 64, seed=13)
    slot = torch.arange(R, dtype=torch.int32, device=DEV).flip(0)
    kvl = torch.tensor(kvlens, dtype=torch.int32, device=DEV)
    out = ops.row_attention(q, kc, vc, slot, kvl, impl=impl)
    for r in range(R):
        s, L = int(slot[r]), kvlens[r]
        qq = q[r].float().view(H, 64)
        K = kc[s, :, :L].float()
        V = vc[s, :, :L].float()
        p = torch.softmax(torch.einsum("hd,htd->ht", qq, K) / 8.0, -1)
        ref = torch.einsum("ht,htd->hd", p, V).reshape(-1)
        torch.testing.assert_close(out[r].float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("lens", [[1, 7, 16, 17, 32, 50], [150, 3], [33]])
def test_tile_attention_matches_fp32(lens, causal):
    """MFMA tile attention (prefill / encoder) on packed variable-length sequences vs an fp32
    torch softmax-attention, with 5 heads (partial last 4-head workgroup) and slots that do not
    follow the packing order."""
    ops = _ops()
    H, T = 5, 160
    R, n = sum(lens), len(lens)
    q = _bf(R, H * 64, seed=21)
    kc = _bf(n + 2, H, T, 64, seed=22)
    vc = _bf(n + 2, H, T, 64, seed=23)
    slots = [(3 * b + 1) % (n + 2) for b in range(n)]
    assert len(set(slots)) == n
    row_slot = torch.tensor([slots[b] for b, L in enumerate(lens) for _ in range(L)], dtype=torch.int32, device=DEV)
    kvl = torch.tensor([(i + 1) if causal else L for L in lens for i in range(L)], dtype=torch.int32, device=DEV)
    tiles = ops.AttnTiles(lens, DEV)
    out = ops.tile_attention(q, kc, vc, row_slot, kvl, tiles)
    row = 0
    for b, L in enumerate(lens):
        s = slots[b]
        K, V = kc[s, :, :L].float(), vc[s, :, :L].float()          # [H, L, 64]
        qq = q[row: row + L].float().view(L, H, 64).transpose(0, 1)  # [H, L, 64]
        sc = torch.einsum("hqd,hkd->hqk", qq, K) / 8.0
        if causal:
            sc = sc.masked_fill(torch.ones(L, L, device=DEV).triu(1).bool(), float("-inf"))
        ref = torch.einsum("hqk,hkd->hqd", torch.softmax(sc, -1), V).transpose(0, 1).reshape(L, H * 64)
        torch.testing.assert_close(out[row: row + L].float(), ref, atol=2e-2, rtol=2e-2)
        row += L


def test_tile_attention_equals_row_attention_on_prefill_rows():
    """Same inputs through both kernels (the row kernel is the decode path): outputs agree to bf16."""
    ops = _ops()
    H, T = 12, 64
    lens = [32] * 9 + [5, 20]
    R, n = sum(lens), len(lens)
    q = _bf(R, H * 64, seed=31)
    kc = _bf(n, H, T, 64, seed=32)
    vc = _bf(n, H, T, 64, seed=33)
    row_slot = torch.tensor([b for b, L in enumerate(lens) for _ in range(L)], dtype=torch.int32, device=DEV)
    kvl = torch.tensor([i + 1 for L in lens for i in range(L)], dtype=torch.int32, device=DEV)
    a = ops.tile_attention(q, kc, vc, row_slot, kvl, ops.AttnTiles(lens, DEV))
    b = ops.row_attention(q, kc, vc, row_slot, kvl)
    torch.testing.assert_close(a.float(), b.float(), atol=1.6e-2, rtol=1.6e-2)


def test_embed_and_decode_update():
    ops = _ops()
    V, P, D, B, T = 1000, 64, 128, 3, 10
    wte, wpe = _bf(V, D, seed=14), _bf(P, D, seed=15)
    tok = torch.tensor([5, 999, 0], dtype=torch.int32, device=DEV)
    pos = torch.tensor([0, 7, 63], dtype=torch.int32, device=DEV)
    x = ops.embed(tok, pos, wte, wpe)
    torch.testing.assert_close(x, wte[tok.long()].float() + wpe[pos.long()].float())

    keys = torch.zeros(B, dtype=torch.int64, device=DEV)
    # row 0 -> token 17, row 1 -> eos (999), row 2 already finished
    def key(v, i):
        u = torch.tensor([v], dtype=torch.float32).view(torch.int32).item() & 0xFFFFFFFF
        o = (~u & 0xFFFFFFFF) if (u & 0x80000000) else (u | 0x80000000)
        k = (o << 32) | (~i & 0xFFFFFFFF)
        return k - (1 << 64) if k >= (1 << 63) else k
    keys.copy_(torch.tensor([key(1.5, 17), key(-2.0, 999), key(0.0, 3)], dtype=torch.int64))
    lens = torch.tensor([4, 9, 10], dtype=torch.int32, device=DEV)
    fin = torch.tensor([0, 0, 1], dtype=torch.int32, device=DEV)
    out = torch.zeros(B, T, dtype=torch.int32, device=DEV)
    out[2, 9] = 42
    seen = torch.zeros(B, 32, dtype=torch.int32, device=DEV)
    ct, cp, ck = (torch.zeros(B, dtype=torch.int32, device=DEV) for _ in range(3))
    xb = torch.zeros(B, D, device=DEV)
    # keys as [B, P] partials with a decoy partial per row (max must win), and as a [P, B].T view
    decoy = torch.tensor([key(-5.0, 1)] * B, dtype=torch.int64, device=DEV)
    parts = torch.stack([decoy, keys], dim=1)
    keys_t = torch.stack([keys, decoy], dim=0).t()
    assert keys_t.stride(0) == 1
    ops.decode_update(parts, lens, fin, out, seen, ct, cp, ck, wte, wpe, xb, eos=999, t_max=T)
    assert lens.tolist() == [5, 10, 10]
    assert fin.tolist() == [0, 1, 1]
    assert out[0, 4].item() == 17 and out[1, 9].item() == 999
    assert ct.tolist() == [17, 999, 42] and cp.tolist() == [4, 9, 9] and ck.tolist() == [5, 10, 10]
    # the transposed (gathered-per-rank) layout decodes the same tokens
    lens2 = torch.tensor([4, 9, 10], dtype=torch.int32, device=DEV)
    fin2 = torch.tensor([0, 0, 1], dtype=torch.int32, device=DEV)
    out2 = torch.zeros(B, T, dtype=torch.int32, device=DEV)
    out2[2, 9] = 42
    ops.decode_update(keys_t, lens2, fin2, out2, torch.zeros_like(seen), ct, cp, ck, wte, wpe, xb, eos=999, t_max=T)
    assert torch.equal(out2, out) and lens2.tolist() == lens.tolist()
    assert (seen[0, 0].item() >> 17) & 1 == 1
    torch.testing.assert_close(xb[0], wte[17].float() + wpe[4].float())


@pytest.mark.parametrize("D", [768, 1024, 1600])
def test_decode_update_fused_ln1_is_bit_identical(D):
    """decode_update's fused layer-0 LN1 (the overlapped step skips that launch on steps 2.. of a
    graph replay) writes exactly what add_layernorm writes from the stored row -- bit for bit, so
    the tokens cannot depend on how many steps a replay holds -- and matches the fp32 LayerNorm."""
    ops = _ops()
    V, P, B, T = 3000, 256, 37, 150
    wte, wpe = _bf(V, D, seed=21), _bf(P, D, seed=22)
    g = torch.randn(D, generator=torch.Generator().manual_seed(23)).to(DEV)
    b = torch.randn(D, generator=torch.Generator().manual_seed(24)).to(DEV)
    gk = torch.Generator().manual_seed(25)
    toks = torch.randint(0, V, (B, 5), generator=gk)
    keys = ((torch.randint(0, 2**30, (B, 5), generator=gk) << 32) | (~toks & 0xFFFFFFFF)).to(DEV)  # valid ids only
    lens = torch.randint(1, T - 1, (B,), generator=torch.Generator().manual_seed(26)).to(torch.int32).to(DEV)
    fin = (torch.arange(B) % 5 == 3).to(torch.int32).to(DEV)
    out = torch.randint(0, V, (B, T), generator=torch.Generator().manual_seed(27)).to(torch.int32).to(DEV)
    seen = torch.zeros(B, (V + 31) // 32, dtype=torch.int32, device=DEV)
    ct, cp, ck = (torch.zeros(B, dtype=torch.int32, device=DEV) for _ in range(3))
    x = torch.zeros(B, D, device=DEV)
    h = torch.full((B, D), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops.decode_update(keys, lens, fin, out, seen, ct, cp, ck, wte, wpe, x, eos=V - 1, t_max=T, ln=(g, b, 1e-5), h=h)
    torch.testing.assert_close(x, wte[ct.long()].float() + wpe[cp.long()].float())
    ref = torch.empty_like(h)
    ops.add_layernorm(x.clone(), g, b, 1e-5, out_bf16=ref)
    assert torch.equal(h.view(torch.int16), ref.view(torch.int16))
    torch.testing.assert_close(h.float(), torch.nn.functional.layer_norm(x, (D,), g, b, 1e-5), atol=3e-2, rtol=2e-2)


def test_bert_embed_pool_cosine():
    ops = _ops()
    V, P, D = 100, 32, 128
    word = torch.randn(V, D, device=DEV)
    pe = torch.randn(P, D, device=DEV)
    t0 = torch.randn(D, device=DEV)
    g, b = torch.randn(D, device=DEV), torch.randn(D, device=DEV)
    ids = torch.tensor([1, 5, 7, 9, 2], dtype=torch.int32, device=DEV)
    pos = torch.tensor([0, 1, 2, 0, 1], dtype=torch.int32, device=DEV)
    xf, xb = ops.bert_embed_ln(ids, pos, word, pe, t0, g, b, 1e-12)
    ref = torch.nn.functional.layer_norm(word[ids.long()] + pe[pos.long()] + t0, (D,), g, b, 1e-12)
    torch.testing.assert_close(xf, ref, atol=1e-4, rtol=1e-4)
    start = torch.tensor([0, 3], dtype=torch.int32, device=DEV)
    ln = torch.tensor([3, 2], dtype=torch.int32, device=DEV)
    pooled = ops.mean_pool(xf, start, ln)
    torch.testing.assert_close(pooled, torch.stack([ref[:3].mean(0), ref[3:].mean(0)]), atol=1e-5, rtol=1e-5)
    sim = ops.cosine(pooled, pooled)
    refsim = torch.nn.functional.cosine_similarity(pooled[:, None], pooled[None], dim=-1)
    torch.testing.assert_close(sim, refsim, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("M,N,K,S", [(256, 768, 3072, 4), (7, 768, 768, 3), (64, 256, 512, 8), (300, 128, 128, 1)])
def test_gemm_split_k_partials_and_add_layernorm(M, N, K, S):
    ops = _ops()
    a, w = _bf(M, K, seed=21), _bf(N, K, scale=0.05, seed=22)
    parts = torch.full((S, M, N), float("nan"), device=DEV)
    ops.gemm(a, w, ops.EPI_PARTIAL, out=parts, split_k=S)
    full = a.float() @ w.float().t()
    torch.testing.assert_close(parts.sum(0), full, atol=2e-3, rtol=1e-3)
    # fused residual update + LayerNorm consumes the slabs
    x = torch.randn(M, N, device=DEV)
    bias = torch.randn(N, device=DEV)
    g, b = torch.randn(N, device=DEV), torch.randn(N, device=DEV)
    ref_x = x + bias + full
    out = ops.add_layernorm(x, g, b, 1e-5, parts=parts, nsplit=S, bias=bias)
    torch.testing.assert_close(x, ref_x, atol=2e-3, rtol=1e-3)
    ref = torch.nn.functional.layer_norm(ref_x, (N,), g, b, 1e-5)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=1e-2)


def test_add_layernorm_no_update():
    ops = _ops()
    x = torch.randn(5, 768, device=DEV)
    x0 = x.clone()
    g, b = torch.randn(768, device=DEV), torch.randn(768, device=DEV)
    out = ops.add_layernorm(x, g, b, 1e-5)
    assert torch.equal(x, x0)
    torch.testing.assert_close(out.float(), torch.nn.functional.layer_norm(x0, (768,), g, b, 1e-5), atol=3e-2,
                               rtol=1e-2)


# ---------------------------------------------------------------------------- fp8 (W8A8, OCP e4m3)
def _deq(q, s):
    return q.float() * s[:, None]


@pytest.mark.parametrize("M,N,K", [(256, 2304, 768), (7, 128, 256), (130, 64, 1024)])
def test_gemm_fp8_matches_dequantized_reference(M, N, K):
    ops = _ops()
    a, w = _bf(M, K, seed=31), _bf(N, K, scale=0.05, seed=32)
    a8, sa = ops.quantize_fp8_rows(a)
    w8, sw = ops.quantize_fp8_weight(w)
    # the kernel quantiser agrees with torch's e4m3fn rounding
    ref8 = (a.float() / sa[:, None]).to(ops.FP8)
    assert (a8.view(torch.uint8) != ref8.view(torch.uint8)).float().mean() < 1e-3
    bias = torch.randn(N, device=DEV)
    out = ops.gemm(a8, w8, ops.EPI_BF16, bias=bias, a_scale=sa, w_scale=sw)
    ref = _deq(a8, sa) @ _deq(w8, sw).t() + bias
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    # and stays close to the bf16 product it approximates
    cos = torch.nn.functional.cosine_similarity(out.float().flatten(), (a.float() @ w.float().t() + bias).flatten(),
                                                dim=0)
    assert cos > 0.995


def test_add_layernorm_fp8_output_and_fp8_argmax():
    ops = _ops()
    M, D, V = 33, 768, 4096
    x = torch.randn(M, D, device=DEV)
    g, b = torch.randn(D, device=DEV), torch.randn(D, device=DEV)
    h8 = torch.empty(M, D, dtype=ops.FP8, device=DEV)
    hs = torch.empty(M, device=DEV)
    out = ops.add_layernorm(x, g, b, 1e-5, out_fp8=h8, out_fp8_scale=hs)
    ref = torch.nn.functional.layer_norm(x, (D,), g, b, 1e-5)
    torch.testing.assert_close(hs, ref.abs().amax(1) / 448, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(_deq(h8, hs), ref, atol=0.08 * ref.abs().amax().item() / 8, rtol=0.07)
    assert out is not None
    # fp8 LM head with the fused penalty + argmax epilogue equals argmax of the dequantised logits
    w8, sw = ops.quantize_fp8_weight(_bf(V, D, scale=0.05, seed=33))
    keys = torch.zeros(M, V // 64, dtype=torch.int64, device=DEV)
    seen = torch.zeros(M, V // 32, dtype=torch.int32, device=DEV)
    ops.gemm(h8, w8, ops.EPI_ARGMAX, argmax_out=keys, seen=seen, vocab=V - 5, penalty=1.2, a_scale=hs, w_scale=sw)
    logits = _deq(h8, hs) @ _deq(w8, sw).t()
    logits[:, V - 5:] = float("-inf")
    red = ops.argmax_reduce(keys)  # unsigned key max on the device
    idx = (~(red & 0xFFFFFFFF)) & 0xFFFFFFFF
    top2 = logits.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3  # ignore near-ties (fp32 summation order)
    assert torch.equal(idx[clear], logits.argmax(1)[clear])


@pytest.mark.parametrize("M", [257, 384, 512])
@pytest.mark.parametrize("epi", ["qkv", "gelu_tanh", "partial_ln"])
def test_gemm96_headline_instantiations(M, epi):
    """The exact 64x96 instantiations every BENCH decode step launches on its 512-row halves
    (gemm.hip: 256 < M <= 512): QKV N 2304 / K 768 with the K/V scatter into a [slots][H][T][64]
    cache, c_fc + GELU-tanh N 3072 / K 768, and c_proj EPI_PARTIAL N 768 / K 3072 split 4 followed
    by the add + LayerNorm that sums its slabs -- each vs fp32, and each asserted to dispatch the
    64x96 tile."""
    ops = _ops()
    D = 768
    ops.gemm_tile_reset()
    if epi == "qkv":
        H, S, T = 12, 4, 150
        a, w = _bf(M, D, seed=41), _bf(3 * D, D, scale=0.05, seed=42)
        bias = torch.randn(3 * D, device=DEV) * 0.1
        q = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
        kc = torch.zeros(S * (M // S + 1), H, T, 64, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros_like(kc)
        # decode-shaped rows: every row its own slot at its own position
        slot = torch.randperm(kc.shape[0], generator=torch.Generator().manual_seed(M))[:M].to(torch.int32).to(DEV)
        pos = (torch.arange(M, device=DEV) * 37 % T).to(torch.int32)
        ops.gemm(a, w, ops.EPI_QKV, bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot, row_pos=pos)
        assert ops.gemm_tile_count(64, 96) == 1
        ref = a.float() @ w.float().t() + bias
        torch.testing.assert_close(q.float(), ref[:, :D], atol=2e-2, rtol=2e-2)
        sl, ps = slot.long(), pos.long()
        k_rows = kc[sl, :, ps].reshape(M, D).float()
        v_rows = vc[sl, :, ps].reshape(M, D).float()
        torch.testing.assert_close(k_rows, ref[:, D:2 * D], atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(v_rows, ref[:, 2 * D:], atol=2e-2, rtol=2e-2)
        assert int((kc != 0).sum()) == M * D  # nothing written outside the rows' (slot, pos)
    elif epi == "gelu_tanh":
        N = 4 * D
        a, w = _bf(M, D, seed=43), _bf(N, D, scale=0.05, seed=44)
        bias = torch.randn(N, device=DEV) * 0.1
        out = ops.gemm(a, w, ops.EPI_GELU_TANH, bias=bias)
        assert ops.gemm_tile_count(64, 96) == 1
        ref = torch.nn.functional.gelu(a.float() @ w.float().t() + bias, approximate="tanh")
        torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    else:
        K = 4 * D
        a, w = _bf(M, K, seed=45), _bf(D, K, scale=0.02, seed=46)
        parts = torch.full((4, M, D), float("nan"), device=DEV)  # every slab element must be written
        ops.gemm(a, w, ops.EPI_PARTIAL, out=parts, split_k=4)
        assert ops.gemm_tile_count(64, 96) == 1
        ref_parts = torch.stack([a[:, s * D:(s + 1) * D].float() @ w[:, s * D:(s + 1) * D].float().t()
                                 for s in range(4)])
        torch.testing.assert_close(parts, ref_parts, atol=1e-2, rtol=1e-3)
        bias = torch.randn(D, device=DEV) * 0.1
        g, b = 1 + 0.1 * torch.randn(D, device=DEV), 0.1 * torch.randn(D, device=DEV)
        x = torch.randn(M, D, device=DEV)
        xr = x + ref_parts.sum(0) + bias
        out = ops.add_layernorm(x, g, b, 1e-5, parts=parts, nsplit=4, bias=bias)
        torch.testing.assert_close(x, xr, atol=1e-2, rtol=1e-3)  # residual updated in place
        ref = torch.nn.functional.layer_norm(xr, (D,), g, b, 1e-5)
        torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)
