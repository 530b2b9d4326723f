"""GPT-2 weights + a plain-PyTorch reference implementation.

This module is the CPU path (BASELINE config 1, "plumbing, no GPU") and the fp32
oracle that the HIP engine (``engine/gpt2_engine.py``) is checked against.

Parity target: ``GPT2LMHeadModel.generate(max_length=150, repetition_penalty=1.2)``
with ``do_sample`` unset, i.e. greedy decoding with a CTRL-style penalty
(``tutoring_server.py:21-29``).

Weights are held in the HF ``Conv1D`` layout ([in, out]) under the HF key names so
that ``transformers`` checkpoints (safetensors) load unchanged and the oracle tests
can push the same tensors into ``transformers.GPT2LMHeadModel``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .config import GPT2Config


def gelu_new(x: torch.Tensor) -> torch.Tensor:
    # GPT-2's tanh-approximated GELU ("gelu_new").
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def init_gpt2_weights(cfg: GPT2Config, seed: int = 0, dtype=torch.float32) -> dict[str, torch.Tensor]:
    """Seeded random init with GPT-2's initializer (normal(0, 0.02); residual projections
    scaled by 1/sqrt(2L); LayerNorm = (1, 0)).  Returns HF-named tensors."""
    g = torch.Generator().manual_seed(seed)
    d, L, std = cfg.n_embd, cfg.n_layer, cfg.initializer_range
    proj_std = std / math.sqrt(2 * L)

    def normal(*shape, s=std):
        return (torch.randn(*shape, generator=g) * s).to(dtype)

    w: dict[str, torch.Tensor] = {
        "transformer.wte.weight": normal(cfg.vocab_size, d),
        "transformer.wpe.weight": normal(cfg.n_positions, d, s=0.01),
        "transformer.ln_f.weight": torch.ones(d, dtype=dtype),
        "transformer.ln_f.bias": torch.zeros(d, dtype=dtype),
    }
    for i in range(L):
        p = f"transformer.h.{i}."
        w[p + "ln_1.weight"] = torch.ones(d, dtype=dtype)
        w[p + "ln_1.bias"] = torch.zeros(d, dtype=dtype)
        w[p + "attn.c_attn.weight"] = normal(d, 3 * d)
        w[p + "attn.c_attn.bias"] = torch.zeros(3 * d, dtype=dtype)
        w[p + "attn.c_proj.weight"] = normal(d, d, s=proj_std)
        w[p + "attn.c_proj.bias"] = torch.zeros(d, dtype=dtype)
        w[p + "ln_2.weight"] = torch.ones(d, dtype=dtype)
        w[p + "ln_2.bias"] = torch.zeros(d, dtype=dtype)
        w[p + "mlp.c_fc.weight"] = normal(d, 4 * d)
        w[p + "mlp.c_fc.bias"] = torch.zeros(4 * d, dtype=dtype)
        w[p + "mlp.c_proj.weight"] = normal(4 * d, d, s=proj_std)
        w[p + "mlp.c_proj.bias"] = torch.zeros(d, dtype=dtype)
    return w


def perturb_norms_and_biases(w: dict[str, torch.Tensor], seed: int = 1, scale: float = 0.02) -> None:
    """Give LN gains/biases and linear biases non-trivial values so kernel tests
    exercise the affine/bias paths (an all-ones/zeros init would hide bugs)."""
    g = torch.Generator().manual_seed(seed)
    for k, v in w.items():
        if k.endswith(".bias") or (("ln_" in k) and k.endswith(".weight")):
            v.add_(torch.randn(v.shape, generator=g).to(v.dtype) * scale)


def load_safetensors_weights(path: str) -> dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    raw = load_file(path)
    out = {}
    for k, v in raw.items():
        key = k if k.startswith("transformer.") or k.startswith("lm_head") else "transformer." + k
        out[key] = v.float()
    return out


@dataclass
class KVCache:
    """Contiguous per-slot KV cache for the reference path: [L, 2, B, H, Tmax, hd]."""

    data: torch.Tensor

    @classmethod
    def allocate(cls, cfg: GPT2Config, batch: int, max_len: int, dtype=torch.float32, device="cpu"):
        return cls(torch.zeros(cfg.n_layer, 2, batch, cfg.n_head, max_len, cfg.head_dim, dtype=dtype, device=device))


class GPT2Reference:
    """Plain-torch GPT-2 forward with a KV cache (batch, ragged prompt lengths)."""

    def __init__(self, cfg: GPT2Config, weights: dict[str, torch.Tensor], device="cpu", dtype=torch.float32):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.w = {k: v.to(device=self.device, dtype=dtype) for k, v in weights.items()}

    def _ln(self, x, name):
        return torch.nn.functional.layer_norm(
            x, (self.cfg.n_embd,), self.w[name + ".weight"], self.w[name + ".bias"], self.cfg.layer_norm_epsilon
        )

    def forward(self, tokens: torch.Tensor, positions: torch.Tensor, cache: KVCache, rows: torch.Tensor) -> torch.Tensor:
        """Run ``tokens`` [B, S] at ``positions`` [B, S] for cache rows ``rows`` [B].

        Keys at cache positions ``<= position`` are attended (causal); returns the
        final hidden state after ``ln_f`` as [B, S, d].
        """
        cfg = self.cfg
        B, S = tokens.shape
        H, hd, d = cfg.n_head, cfg.head_dim, cfg.n_embd
        x = self.w["transformer.wte.weight"][tokens] + self.w["transformer.wpe.weight"][positions]
        Tmax = cache.data.shape[4]
        key_pos = torch.arange(Tmax, device=self.device)
        mask = key_pos[None, None, :] <= positions[:, :, None]  # [B, S, Tmax]
        bidx = rows[:, None].expand(B, S)
        for i in range(cfg.n_layer):
            p = f"transformer.h.{i}."
            h = self._ln(x, p + "ln_1")
            qkv = h @ self.w[p + "attn.c_attn.weight"] + self.w[p + "attn.c_attn.bias"]
            q, k, v = qkv.split(d, dim=-1)
            q = q.view(B, S, H, hd)
            k = k.view(B, S, H, hd)
            v = v.view(B, S, H, hd)
            cache.data[i, 0, bidx, :, positions] = k.to(cache.data.dtype)
            cache.data[i, 1, bidx, :, positions] = v.to(cache.data.dtype)
            K = cache.data[i, 0, rows].to(x.dtype)  # [B, H, Tmax, hd]
            V = cache.data[i, 1, rows].to(x.dtype)
            att = torch.einsum("bshd,bhtd->bhst", q, K) / math.sqrt(hd)
            att = att.masked_fill(~mask[:, None, :, :], float("-inf"))
            att = torch.softmax(att, dim=-1)
            a = torch.einsum("bhst,bhtd->bshd", att, V).reshape(B, S, d)
            x = x + a @ self.w[p + "attn.c_proj.weight"] + self.w[p + "attn.c_proj.bias"]
            h = self._ln(x, p + "ln_2")
            f = gelu_new(h @ self.w[p + "mlp.c_fc.weight"] + self.w[p + "mlp.c_fc.bias"])
            x = x + f @ self.w[p + "mlp.c_proj.weight"] + self.w[p + "mlp.c_proj.bias"]
        return self._ln(x, "transformer.ln_f")

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        return hidden @ self.w["transformer.wte.weight"].t()


def apply_repetition_penalty(logits: torch.Tensor, seen: torch.Tensor, penalty: float) -> torch.Tensor:
    """CTRL-style penalty (HF ``RepetitionPenaltyLogitsProcessor``): for every id already
    in the sequence, ``l < 0 ? l * p : l / p``.  ``seen`` is a bool mask [B, V]."""
    if penalty == 1.0:
        return logits
    pen = torch.where(logits < 0, logits * penalty, logits / penalty)
    return torch.where(seen, pen, logits)


@torch.no_grad()
def reference_generate(
    model: GPT2Reference,
    prompts: list[list[int]],
    max_length: int = 150,
    repetition_penalty: float = 1.2,
    eos_token_id: int | None = None,
) -> list[list[int]]:
    """Batched greedy + repetition-penalty decode.  Returns full sequences (prompt
    echoed, as ``generate`` does), each stopping at EOS (inclusive) or ``max_length``."""
    cfg = model.cfg
    eos = cfg.eos_token_id if eos_token_id is None else eos_token_id
    B = len(prompts)
    dev = model.device
    cache = KVCache.allocate(cfg, B, max_length, dtype=model.dtype, device=dev)
    rows = torch.arange(B, device=dev)
    seqs = [list(p) for p in prompts]
    seen = torch.zeros(B, cfg.vocab_size, dtype=torch.bool, device=dev)
    for b, p in enumerate(prompts):
        seen[b, torch.tensor(p, device=dev)] = True
    done = [len(p) >= max_length for p in prompts]
    # prefill each prompt (ragged lengths: run per-length groups padded on the right)
    maxp = max(len(p) for p in prompts)
    toks = torch.zeros(B, maxp, dtype=torch.long, device=dev)
    pos = torch.zeros(B, maxp, dtype=torch.long, device=dev)
    for b, p in enumerate(prompts):
        toks[b, : len(p)] = torch.tensor(p, device=dev)
        # pad positions repeat the last real position so they overwrite it with
        # identical k/v (harmless) instead of polluting later slots
        pos[b, : len(p)] = torch.arange(len(p), device=dev)
        pos[b, len(p):] = len(p) - 1
        toks[b, len(p):] = p[-1]
    hidden = model.forward(toks, pos, cache, rows)
    last = torch.tensor([len(p) - 1 for p in prompts], device=dev)
    h_last = hidden[rows, last]
    while True:
        logits = model.logits(h_last)
        logits = apply_repetition_penalty(logits, seen, repetition_penalty)
        nxt = torch.argmax(logits, dim=-1)
        for b in range(B):
            if done[b]:
                continue
            t = int(nxt[b])
            seqs[b].append(t)
            seen[b, t] = True
            if t == eos or len(seqs[b]) >= max_length:
                done[b] = True
        if all(done):
            break
        cur_pos = torch.tensor([min(len(s) - 1, max_length - 1) for s in seqs], device=dev)
        cur_tok = torch.tensor([s[-1] for s in seqs], device=dev)
        hidden = model.forward(cur_tok[:, None], cur_pos[:, None], cache, rows)
        h_last = hidden[:, 0]
    return seqs


@torch.no_grad()
def teacher_forced_check(model: GPT2Reference, seq: list[int], prompt_len: int, repetition_penalty: float = 1.2,
                         eps: float = 0.05) -> dict:
    """Margin-aware exactness oracle for a generated sequence: run the fp32 reference once over
    ``seq`` (teacher forcing), and at every generated position compare the produced token with the
    reference's greedy choice under the repetition penalty of the prefix.  A position is
    *decisive* when the reference's top-1 minus top-2 penalised logit exceeds ``eps``; at every
    decisive position the token must be the reference's argmax.

    Returns {"positions", "decisive", "mismatches": [(i, got, want, margin)], "min_margin"}."""
    cfg = model.cfg
    dev = model.device
    S = len(seq)
    if S <= prompt_len:
        return {"positions": 0, "decisive": 0, "mismatches": [], "min_margin": float("inf")}
    cache = KVCache.allocate(cfg, 1, S, dtype=model.dtype, device=dev)
    toks = torch.tensor([seq], device=dev)
    pos = torch.arange(S, device=dev)[None]
    hidden = model.forward(toks, pos, cache, torch.zeros(1, dtype=torch.long, device=dev))[0]
    logits = model.logits(hidden[prompt_len - 1: S - 1])  # row j predicts seq[prompt_len + j]
    n = logits.shape[0]
    seen = torch.zeros(n, cfg.vocab_size, dtype=torch.bool, device=dev)
    for j in range(n):
        seen[j, torch.tensor(seq[: prompt_len + j], device=dev)] = True
    logits = apply_repetition_penalty(logits, seen, repetition_penalty)
    top = logits.topk(2, dim=-1)
    margin = (top.values[:, 0] - top.values[:, 1]).tolist()
    want = top.indices[:, 0].tolist()
    out = {"positions": n, "decisive": 0, "mismatches": [], "min_margin": min(margin)}
    for j in range(n):
        got = seq[prompt_len + j]
        if margin[j] > eps:
            out["decisive"] += 1
            if got != want[j]:
                out["mismatches"].append((prompt_len + j, got, want[j], margin[j]))
    return out


@torch.no_grad()
def teacher_forced_check_batch(model: GPT2Reference, seqs: list[list[int]], prompt_lens: list[int],
                               repetition_penalty: float = 1.2, eps: float = 0.05, chunk: int = 16) -> list[dict]:
    """``teacher_forced_check`` for many sequences at once (chunks of ``chunk`` rows, each padded on
    the right: causal attention keeps the padding out of every checked position).  The penalty
    mask of position j of a row is "first occurrence of v < prompt_len + j", built by one
    scatter-min instead of a loop of small launches.  Same result dicts, in order."""
    cfg, dev = model.cfg, model.device
    out: list[dict] = []
    for c0 in range(0, len(seqs), chunk):
        rows = seqs[c0: c0 + chunk]
        pls = prompt_lens[c0: c0 + chunk]
        Bc = len(rows)
        S = max(len(s) for s in rows)
        toks = torch.tensor([s + [s[-1]] * (S - len(s)) for s in rows], device=dev)
        pos = torch.arange(S, device=dev)[None].expand(Bc, S).contiguous()
        cache = KVCache.allocate(cfg, Bc, S, dtype=model.dtype, device=dev)
        hidden = model.forward(toks, pos, cache, torch.arange(Bc, device=dev))
        first = torch.full((Bc, cfg.vocab_size), S + 1, dtype=torch.long, device=dev)
        first.scatter_reduce_(1, toks, pos, reduce="amin")
        for b, (s, pl) in enumerate(zip(rows, pls)):
            n = len(s) - pl
            if n <= 0:
                out.append({"positions": 0, "decisive": 0, "mismatches": [], "min_margin": float("inf")})
                continue
            logits = model.logits(hidden[b, pl - 1: len(s) - 1])
            seen = first[b][None, :] < (pl + torch.arange(n, device=dev))[:, None]
            logits = apply_repetition_penalty(logits, seen, repetition_penalty)
            top = logits.topk(2, dim=-1)
            margin = (top.values[:, 0] - top.values[:, 1]).tolist()
            want = top.indices[:, 0].tolist()
            r = {"positions": n, "decisive": 0, "mismatches": [], "min_margin": min(margin)}
            for j in range(n):
                if margin[j] > eps:
                    r["decisive"] += 1
                    if s[pl + j] != want[j]:
                        r["mismatches"].append((pl + j, s[pl + j], want[j], margin[j]))
            out.append(r)
    return out
