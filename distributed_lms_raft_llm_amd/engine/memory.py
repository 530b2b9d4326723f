"""KV-cache / slot capacity planning against the GPU's HBM ("KV budget
computed from hipMemGetInfo against the 288 GB HBM").

A decode slot owns its full-length KV cache (``[L][2][H_local][T][64]`` bf16, allocated up front so
the decode graph never reallocates) plus O(d + V/32) bytes of per-sequence state.  The planner
takes the free HBM (``hipMemGetInfo`` via ``torch.cuda.mem_get_info``), keeps a reserve for the
weights (if not yet resident), hipGraph pools, prefill activations and allocator slack, and
returns the largest batch bucket that fits -- capped, because past ~2k live sequences a GPT-2
decode step is compute-bound and more slots only add latency.  GPT-2-small at T=150 needs
~5.6 MB per slot: one MI355X could hold ~45k concurrent sequences; XL at TP=8 ~5.8 MB.
"""
from __future__ import annotations

from ..models.config import GPT2Config
from .weights import shard_range

GIB = 1 << 30
BUCKETS = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768, 1024, 1536, 2048, 3072, 4096, 6144,
           8192, 12288, 16384, 24576, 32768, 49152, 65536)


def slot_bytes(cfg: GPT2Config, max_length: int, tp_size: int = 1, tp_rank: int = 0) -> int:
    """Device bytes one decode slot costs on this rank (KV cache + per-sequence state)."""
    h0, h1 = shard_range(cfg.n_head, tp_size, tp_rank)
    hl = h1 - h0
    dl = hl * cfg.head_dim
    fl = cfg.n_inner // tp_size + 64
    vshard = cfg.vocab_padded // tp_size + 64
    kv = cfg.n_layer * 2 * hl * max_length * cfg.head_dim * 2
    state = (cfg.n_embd * 4            # residual x (f32)
             + 8 * cfg.n_embd * 4      # split-K / TP partial slabs
             + cfg.n_embd * 2 + 2 * dl * 2 + fl * 2   # h, q, att, ff (bf16)
             + vshard // 64 * 8 + 8 + tp_size * 8     # argmax keys
             + 6 * 4 + max_length * 4                 # lens/flags/cur_*, output tokens
             + cfg.vocab_padded // 8)                 # repetition-penalty bitmap
    return kv + state


def weight_bytes(cfg: GPT2Config, tp_size: int = 1) -> int:
    return int(cfg.num_params() * 2 / tp_size) + (cfg.vocab_padded - cfg.vocab_size) * cfg.n_embd * 2


def plan_max_batch(cfg: GPT2Config, max_length: int, tp_size: int = 1, free_bytes: int | None = None,
                   weights_resident: bool = False, reserve_frac: float = 0.08, reserve_bytes: int = 4 * GIB,
                   prefill_tokens: int = 32768, cap: int = 4096, device=None) -> int:
    """Largest batch bucket (<= ``cap``) whose slots fit in the free HBM after the reserve."""
    if free_bytes is None:
        import torch

        free_bytes, _ = torch.cuda.mem_get_info(device)
    budget = free_bytes * (1.0 - reserve_frac) - reserve_bytes
    if not weights_resident:
        budget -= weight_bytes(cfg, tp_size)
    # transient prefill activations for ``prefill_tokens`` packed prompt tokens
    budget -= prefill_tokens * (cfg.n_embd * 4 * 9 + cfg.n_inner // tp_size * 2 + cfg.n_embd * 6)
    per = slot_bytes(cfg, max_length, tp_size)
    fit = int(budget // per) if budget > 0 else 0
    best = 0
    for b in BUCKETS:
        if b <= fit and b <= cap:
            best = b
    if best == 0:
        raise MemoryError(f"not even one decode slot fits: {free_bytes / GIB:.1f} GiB free, {per / 2**20:.1f} MiB/slot")
    return best
