"""Convert HF-layout GPT-2 weights into the device layouts the HIP kernels consume, sharded for
Megatron-style tensor parallelism.

Kernel layout: every GEMM weight is stored [N][K] (K contiguous, "TN"), bf16; biases and LN
parameters stay fp32.  TP sharding:

* attention: column-parallel QKV by head (uneven head counts allowed, e.g. GPT-2-XL's 25 heads
  over 8 ranks -> 4,3,3,3,3,3,3,3), row-parallel out-projection;
* MLP: column-parallel c_fc, row-parallel c_proj (64-column granules);
* LM head: vocab-parallel over the tied ``wte`` (shard boundaries on 64-row tiles) with a
  fused local argmax and a cross-rank (value, index) max.

Row-parallel GEMMs emit raw fp32 partials; after the all-reduce every rank applies
``x += bias + sum(partials)`` in the fused add+LayerNorm kernel, so the replicated residual stays
bit-identical across ranks.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..models.config import GPT2Config


def split_even(n: int, parts: int) -> list[int]:
    base, rem = divmod(n, parts)
    return [base + (1 if i < rem else 0) for i in range(parts)]


def shard_range(n: int, parts: int, rank: int) -> tuple[int, int]:
    sizes = split_even(n, parts)
    start = sum(sizes[:rank])
    return start, start + sizes[rank]


@dataclass
class LayerWeights:
    ln1_g: torch.Tensor
    ln1_b: torch.Tensor
    w_qkv: torch.Tensor  # [3*Dl, D]
    b_qkv: torch.Tensor  # [3*Dl]
    w_o: torch.Tensor  # [D, Dl]
    b_o: torch.Tensor  # [D], added once after the reduction
    ln2_g: torch.Tensor
    ln2_b: torch.Tensor
    w_fc: torch.Tensor  # [Fl, D]
    b_fc: torch.Tensor  # [Fl]
    w_p: torch.Tensor  # [D, Fl]
    b_p: torch.Tensor  # [D], added once after the reduction
    # fp8 (W8A8) copies of the LayerNorm-fed GEMMs: e4m3 [N, Kp] (K zero-padded to a multiple of
    # 128) + per-output-channel f32 scales; None for the bf16 engine
    w_qkv8: torch.Tensor | None = None
    s_qkv: torch.Tensor | None = None
    w_fc8: torch.Tensor | None = None
    s_fc: torch.Tensor | None = None
    # MFMA-fragment-order copies (ops.shuffle_weight) of the LN-fed GEMMs for the latency path's
    # skinny kernels; filled by the engine when that path is enabled
    w_qkv_sh: torch.Tensor | None = None
    w_fc_sh: torch.Tensor | None = None
    w_o_sh: torch.Tensor | None = None  # fused attention + out-projection / in-place out-proj
    w_p_sh: torch.Tensor | None = None  # in-place c_proj (latency path, TP=1)
    w_p_sl: torch.Tensor | None = None  # fused batch-1 MLP: c_proj in 16-column slabs (ops.slice_cproj)


@dataclass
class GPT2DeviceWeights:
    cfg: GPT2Config
    tp_rank: int
    tp_size: int
    head_range: tuple[int, int]
    ffn_range: tuple[int, int]
    vocab_range: tuple[int, int]  # padded-vocab rows of the LM head shard
    wte: torch.Tensor  # [Vpad, D] bf16 (full; embedding gather + LM head view)
    wpe: torch.Tensor  # [P, D] bf16
    lnf_g: torch.Tensor
    lnf_b: torch.Tensor
    layers: list[LayerWeights] = field(default_factory=list)
    lm_head8: torch.Tensor | None = None  # fp8 LM-head shard [V1-V0, Kp] + scales
    s_lm: torch.Tensor | None = None

    @property
    def fp8(self) -> bool:
        return self.lm_head8 is not None

    @property
    def k_fp8(self) -> int:
        """K of the fp8 GEMMs: d padded to the fp8 kernel's 128-element ring step."""
        return -(-self.cfg.n_embd // 128) * 128

    @property
    def n_heads_local(self) -> int:
        return self.head_range[1] - self.head_range[0]

    @property
    def d_local(self) -> int:
        return 64 * self.n_heads_local

    @property
    def ffn_local(self) -> int:
        return self.ffn_range[1] - self.ffn_range[0]

    @property
    def lm_head(self) -> torch.Tensor:
        return self.wte[self.vocab_range[0]: self.vocab_range[1]]

    def nbytes(self) -> int:
        n = self.wte.numel() * 2 + self.wpe.numel() * 2
        for lw in self.layers:
            for t in (lw.w_qkv, lw.w_o, lw.w_fc, lw.w_p):
                n += t.numel() * t.element_size()
        return n


def quantize_fp8_padded(w: torch.Tensor, kp: int):
    """[N, K] -> (e4m3 [N, kp] zero-padded, f32 per-row scales): scale = absmax / 448."""
    wf = w.float()
    scale = wf.abs().amax(dim=1).clamp_min(1e-20) / 448.0
    q = torch.zeros(wf.shape[0], kp, dtype=torch.float8_e4m3fn, device=wf.device)
    q[:, : wf.shape[1]] = (wf / scale[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    return q, scale.contiguous()


def prepare_gpt2_weights(cfg: GPT2Config, w: dict[str, torch.Tensor], device, tp_rank: int = 0, tp_size: int = 1,
                         dtype=torch.bfloat16, fp8: bool = False) -> GPT2DeviceWeights:
    """Shard + lay out GPT-2 weights for this TP rank.  ``fp8``: additionally quantise the QKV,
    c_fc and LM-head weights to OCP e4m3 with per-output-channel scales (the W8A8 path; the
    row-parallel out-proj / c_proj, whose inputs have no cheap row scale, stay bf16)."""
    D, H, hd = cfg.n_embd, cfg.n_head, cfg.head_dim
    assert hd == 64, "kernels assume 64-wide heads (all GPT-2 sizes)"
    h0, h1 = shard_range(H, tp_size, tp_rank)
    if h1 <= h0:
        raise ValueError(f"tp_size={tp_size} leaves rank {tp_rank} with no attention heads (H={H})")
    ft = cfg.n_inner // 64
    f0, f1 = (x * 64 for x in shard_range(ft, tp_size, tp_rank))
    vt = cfg.vocab_padded // 64
    v0, v1 = (x * 64 for x in shard_range(vt, tp_size, tp_rank))

    def dev(t, dt=dtype):
        return t.to(device=device, dtype=dt).contiguous()

    f32 = torch.float32
    wte = torch.zeros(cfg.vocab_padded, D, dtype=f32)
    wte[: cfg.vocab_size] = w["transformer.wte.weight"].float()
    out = GPT2DeviceWeights(
        cfg=cfg, tp_rank=tp_rank, tp_size=tp_size, head_range=(h0, h1), ffn_range=(f0, f1), vocab_range=(v0, v1),
        wte=dev(wte), wpe=dev(w["transformer.wpe.weight"]),
        lnf_g=dev(w["transformer.ln_f.weight"], f32), lnf_b=dev(w["transformer.ln_f.bias"], f32),
    )
    cols = slice(h0 * hd, h1 * hd)
    for i in range(cfg.n_layer):
        p = f"transformer.h.{i}."
        wa = w[p + "attn.c_attn.weight"].float()  # [D, 3D]
        ba = w[p + "attn.c_attn.bias"].float()
        q, k, v = wa[:, :D], wa[:, D: 2 * D], wa[:, 2 * D:]
        bq, bk, bv = ba[:D], ba[D: 2 * D], ba[2 * D:]
        w_qkv = torch.cat([q[:, cols], k[:, cols], v[:, cols]], dim=1).t()
        b_qkv = torch.cat([bq[cols], bk[cols], bv[cols]])
        wo = w[p + "attn.c_proj.weight"].float()[cols, :].t()  # [D, Dl]
        wfc = w[p + "mlp.c_fc.weight"].float()[:, f0:f1].t()  # [Fl, D]
        wp = w[p + "mlp.c_proj.weight"].float()[f0:f1, :].t()  # [D, Fl]
        out.layers.append(LayerWeights(
            ln1_g=dev(w[p + "ln_1.weight"], f32), ln1_b=dev(w[p + "ln_1.bias"], f32),
            w_qkv=dev(w_qkv), b_qkv=dev(b_qkv, f32),
            w_o=dev(wo), b_o=dev(w[p + "attn.c_proj.bias"], f32),
            ln2_g=dev(w[p + "ln_2.weight"], f32), ln2_b=dev(w[p + "ln_2.bias"], f32),
            w_fc=dev(wfc), b_fc=dev(w[p + "mlp.c_fc.bias"].float()[f0:f1], f32),
            w_p=dev(wp), b_p=dev(w[p + "mlp.c_proj.bias"], f32),
        ))
    if fp8:
        kp = out.k_fp8
        for lw in out.layers:
            lw.w_qkv8, lw.s_qkv = quantize_fp8_padded(lw.w_qkv, kp)
            lw.w_fc8, lw.s_fc = quantize_fp8_padded(lw.w_fc, kp)
        out.lm_head8, out.s_lm = quantize_fp8_padded(out.lm_head, kp)
    return out
