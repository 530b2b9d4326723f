"""Tensor-parallel (Megatron-style) GPT-2 decode: process groups, collectives and a torch
reference of the sharded forward.

Sharding (``engine/weights.py``): QKV column-parallel by head (uneven splits allowed, e.g.
GPT-2-XL's 25 heads over 8 ranks), out-proj row-parallel -> all-reduce; c_fc column-parallel,
c_proj row-parallel -> all-reduce; LM head vocab-parallel with a local fused argmax and an
all-gather of the packed (value, index) keys.  Per token and layer that is 2 all-reduces of a
[B, d] fp32 tensor (latency-bound at decode sizes) plus one 8-byte-per-row
all-gather per step.

``TorchTPGPT2`` runs exactly that dataflow with torch ops, on any device and any backend (gloo
on CPU), so the sharding and the collective placement are testable without GPUs; the HIP engine
(``engine/gpt2_engine.py``) executes the same plan with its kernels inside one hipGraph per step.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

from ..engine.weights import GPT2DeviceWeights, prepare_gpt2_weights
from ..models.config import GPT2Config
from ..models.gpt2 import gelu_new


def init_distributed(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise the default process group from torchrun env vars (one process per GPU)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0"))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device(f"cuda:{local}"))
    else:
        dist.init_process_group(backend)
    return rank, world, local


def tp_groups(tp: int):
    """Split the world into consecutive TP groups of size ``tp`` (DP across groups).
    Returns (my TP group, my DP index, number of DP replicas).  On an 8-GPU node TP groups of
    consecutive local ranks share the fully connected xGMI mesh."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % tp:
        raise ValueError(f"world size {world} is not a multiple of tp={tp}")
    mine = None
    for g in range(world // tp):
        grp = dist.new_group(list(range(g * tp, (g + 1) * tp)))
        if g == rank // tp:
            mine = grp
    return mine, rank // tp, world // tp


def all_gather_rows(local: torch.Tensor, group) -> torch.Tensor:
    """[n] -> [world, n] on every rank (uses the fused tensor API when the backend has it)."""
    world = dist.get_world_size(group)
    out = torch.empty(world, *local.shape, dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out.view(-1), local.contiguous(), group=group)
    else:
        parts = list(out.unbind(0))
        dist.all_gather(parts, local.contiguous(), group=group)
        for i, p in enumerate(parts):
            out[i].copy_(p)
    return out


def pack_keys(values: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """(value, index) -> int64 whose signed order is (value desc, index asc): the same key the
    LM-head kernel's atomicMax uses, reinterpreted as a signed int64 (sign bit flipped)."""
    u = values.float().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ordered = torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    key = (ordered << 32) | ((~index.to(torch.int64)) & 0xFFFFFFFF)
    return key ^ (-(1 << 63))  # unsigned order -> signed order


def unpack_index(keys: torch.Tensor) -> torch.Tensor:
    return (~(keys ^ (-(1 << 63)))) & 0xFFFFFFFF


class TorchTPGPT2:
    """Sharded GPT-2 forward with torch ops (the TP algorithm's executable specification)."""

    def __init__(self, cfg: GPT2Config, weights: dict[str, torch.Tensor], group=None, device="cpu",
                 dtype=torch.float32):
        self.cfg = cfg
        self.group = group
        self.rank = dist.get_rank(group) if group is not None else 0
        self.size = dist.get_world_size(group) if group is not None else 1
        self.w: GPT2DeviceWeights = prepare_gpt2_weights(cfg, weights, device, self.rank, self.size, dtype=dtype)
        self.device = torch.device(device)

    def _ar(self, t):
        if self.size > 1:
            dist.all_reduce(t, group=self.group)
        return t

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, positions: torch.Tensor, cache: list, ln_f: bool = True) -> torch.Tensor:
        """tokens/positions [S] for ONE sequence; ``cache`` is a per-layer list of (K, V) [Hl, T, 64]."""
        cfg, w = self.cfg, self.w
        Hl = w.n_heads_local
        x = (w.wte[tokens] + w.wpe[positions]).float()
        S = tokens.numel()
        for li, lw in enumerate(w.layers):
            h = torch.nn.functional.layer_norm(x, (cfg.n_embd,), lw.ln1_g, lw.ln1_b, cfg.layer_norm_epsilon)
            qkv = h @ lw.w_qkv.float().t() + lw.b_qkv
            q, k, v = qkv.view(S, 3, Hl, 64).unbind(1)
            K, V = cache[li]
            K[:, positions] = k.transpose(0, 1)
            V[:, positions] = v.transpose(0, 1)
            T = int(positions.max()) + 1
            att = torch.einsum("shd,htd->hst", q, K[:, :T]) / math.sqrt(64)
            mask = torch.arange(T, device=x.device)[None, :] <= positions[:, None]
            att = torch.softmax(att.masked_fill(~mask[None], float("-inf")), dim=-1)
            a = torch.einsum("hst,htd->shd", att, V[:, :T]).reshape(S, Hl * 64)
            x = x + self._ar(a @ lw.w_o.float().t()) + lw.b_o
            h = torch.nn.functional.layer_norm(x, (cfg.n_embd,), lw.ln2_g, lw.ln2_b, cfg.layer_norm_epsilon)
            f = gelu_new(h @ lw.w_fc.float().t() + lw.b_fc)
            x = x + self._ar(f @ lw.w_p.float().t()) + lw.b_p
        if ln_f:
            x = torch.nn.functional.layer_norm(x, (cfg.n_embd,), w.lnf_g, w.lnf_b, cfg.layer_norm_epsilon)
        return x

    def new_cache(self, T: int) -> list:
        Hl = self.w.n_heads_local
        return [(torch.zeros(Hl, T, 64, device=self.device), torch.zeros(Hl, T, 64, device=self.device))
                for _ in range(self.cfg.n_layer)]

    @torch.no_grad()
    def next_token(self, hidden_last: torch.Tensor, seen: set[int], penalty: float) -> int:
        """Vocab-parallel greedy step: local penalised argmax, then the cross-rank key max."""
        v0, v1 = self.w.vocab_range
        logits = hidden_last @ self.w.lm_head.float().t()
        ids = torch.arange(v0, v1, device=logits.device)
        valid = ids < self.cfg.vocab_size
        seen_mask = torch.zeros_like(valid)
        loc = [t - v0 for t in seen if v0 <= t < v1]
        if loc:
            seen_mask[torch.tensor(loc, device=logits.device)] = True
        logits = torch.where(seen_mask, torch.where(logits < 0, logits * penalty, logits / penalty), logits)
        logits = torch.where(valid, logits, torch.full_like(logits, float("-inf")))
        j = int(torch.argmax(logits))
        key = pack_keys(logits[j:j + 1], torch.tensor([v0 + j], device=logits.device))
        if self.size > 1:
            key = all_gather_rows(key, self.group).max(dim=0).values
        return int(unpack_index(key)[0])

    @torch.no_grad()
    def generate(self, prompt: list[int], max_length: int, penalty: float = 1.2) -> list[int]:
        cache = self.new_cache(max_length)
        seq = list(prompt)
        seen = set(prompt)
        toks = torch.tensor(seq, device=self.device)
        h = self.forward(toks, torch.arange(len(seq), device=self.device), cache)
        while len(seq) < max_length:
            t = self.next_token(h[-1], seen, penalty)
            seq.append(t)
            seen.add(t)
            if t == self.cfg.eos_token_id or len(seq) >= max_length:
                break
            h = self.forward(torch.tensor([t], device=self.device),
                             torch.tensor([len(seq) - 1], device=self.device), cache)
        return seq


class TorchSlotEngine:
    """The continuous-batching slot protocol (``engine/scheduler.py``) on ``TorchTPGPT2``: any
    device/backend, TP over ``group`` or unsharded.  Every rank of a TP group must receive the
    same admit/decode calls (``engine/tp_serving.py`` mirrors them); the per-slot token state is
    identical on all ranks because the vocab-parallel argmax is all-gathered.  Sequences run one
    after another inside a step (no batching) -- this is the executable specification and the
    CPU serving path, the HIP engine is the fast one."""

    def __init__(self, cfg: GPT2Config, weights: dict[str, torch.Tensor], group=None, max_batch: int = 8,
                 max_length: int = 150, device="cpu"):
        self.m = TorchTPGPT2(cfg, weights, group=group, device=device)
        self.cfg, self.max_batch, self.max_length = cfg, max_batch, max_length
        self.device = torch.device(device)
        eos = cfg.eos_token_id
        self.seqs = [[eos] for _ in range(max_batch)]
        self.fin = [1] * max_batch
        self.seen: list[set] = [set() for _ in range(max_batch)]
        self.caches: list = [None] * max_batch

    def _emit(self, s: int, hidden_last: torch.Tensor, penalty: float):
        t = self.m.next_token(hidden_last, self.seen[s], penalty)
        self.seqs[s].append(t)
        self.seen[s].add(t)
        if t == self.cfg.eos_token_id or len(self.seqs[s]) >= self.max_length:
            self.fin[s] = 1
            self.caches[s] = None

    @torch.no_grad()
    def admit(self, prompts: list[list[int]], slots: list[int], repetition_penalty: float = 1.2):
        for p, s in zip(prompts, slots):
            if not (0 <= s < self.max_batch) or not self.fin[s]:
                raise ValueError(f"slot {s} is not free")
            self.seqs[s], self.seen[s], self.fin[s] = list(p), set(p), 0
            self.caches[s] = self.m.new_cache(self.max_length)
            h = self.m.forward(torch.tensor(p, device=self.device), torch.arange(len(p), device=self.device),
                               self.caches[s])
            self._emit(s, h[-1], repetition_penalty)

    @torch.no_grad()
    def decode(self, B: int, steps: int, repetition_penalty: float = 1.2):
        for _ in range(steps):
            for s in range(B):
                if self.fin[s]:
                    continue
                n = len(self.seqs[s])
                h = self.m.forward(torch.tensor([self.seqs[s][-1]], device=self.device),
                                   torch.tensor([n - 1], device=self.device), self.caches[s])
                self._emit(s, h[-1], repetition_penalty)

    @torch.no_grad()
    def warm_decode_graphs(self, repetition_penalty: float = 1.2, max_batch: int | None = None) -> tuple[int, float]:
        """The HIP engine's start-up warm-up has no graphs to capture here, but it keeps the same
        collective contract: one throw-away decode forward on a scratch cache runs the group's
        all-reduces, so rank 0 calling it alone (not mirrored to the followers) deadlocks exactly
        like an unmirrored graph capture would (tests/test_tp_serving.py, the torchrun CLI test)."""
        import time

        t0 = time.perf_counter()
        eos = self.cfg.eos_token_id
        self.m.forward(torch.tensor([eos], device=self.device), torch.tensor([0], device=self.device),
                       self.m.new_cache(1))
        return 0, time.perf_counter() - t0

    def finished_flags(self, B: int) -> list[int]:
        return list(self.fin[:B])

    def collect(self, slots: list[int]) -> list[list[int]]:
        return [list(self.seqs[s]) for s in slots]
