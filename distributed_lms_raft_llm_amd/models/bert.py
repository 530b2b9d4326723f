"""BERT (bert-base-uncased architecture) weights + plain-PyTorch reference encoder.

The reference gate (``lms_server.py:97-104,1257-1270``) embeds the query and the assignment
text with ``BertModel``: ``last_hidden_state.mean(dim=1)`` (all tokens, [CLS]/[SEP] included,
truncation 512) and rejects the query when the cosine similarity is below 0.6.  Weights use the
HF ``BertModel`` key names (``nn.Linear`` = [out, in]) so a local safetensors checkpoint loads
as-is; without one they are seeded random (BERT's normal(0, 0.02) initializer).
"""
from __future__ import annotations

import math

import torch

from .config import BertConfig


def init_bert_weights(cfg: BertConfig, seed: int = 0, dtype=torch.float32) -> dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    H, I, std = cfg.hidden, cfg.intermediate, cfg.initializer_range

    def normal(*shape):
        return (torch.randn(*shape, generator=g) * std).to(dtype)

    w = {
        "embeddings.word_embeddings.weight": normal(cfg.vocab_size, H),
        "embeddings.position_embeddings.weight": normal(cfg.max_position, H),
        "embeddings.token_type_embeddings.weight": normal(cfg.type_vocab_size, H),
        "embeddings.LayerNorm.weight": torch.ones(H, dtype=dtype),
        "embeddings.LayerNorm.bias": torch.zeros(H, dtype=dtype),
    }
    w["embeddings.word_embeddings.weight"][cfg.pad_token_id].zero_()
    for i in range(cfg.n_layer):
        p = f"encoder.layer.{i}."
        for n in ("query", "key", "value"):
            w[p + f"attention.self.{n}.weight"] = normal(H, H)
            w[p + f"attention.self.{n}.bias"] = torch.zeros(H, dtype=dtype)
        w[p + "attention.output.dense.weight"] = normal(H, H)
        w[p + "attention.output.dense.bias"] = torch.zeros(H, dtype=dtype)
        w[p + "attention.output.LayerNorm.weight"] = torch.ones(H, dtype=dtype)
        w[p + "attention.output.LayerNorm.bias"] = torch.zeros(H, dtype=dtype)
        w[p + "intermediate.dense.weight"] = normal(I, H)
        w[p + "intermediate.dense.bias"] = torch.zeros(I, dtype=dtype)
        w[p + "output.dense.weight"] = normal(H, I)
        w[p + "output.dense.bias"] = torch.zeros(H, dtype=dtype)
        w[p + "output.LayerNorm.weight"] = torch.ones(H, dtype=dtype)
        w[p + "output.LayerNorm.bias"] = torch.zeros(H, dtype=dtype)
    return w


def load_bert_safetensors(path: str) -> dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    raw = load_file(path)
    return {(k[5:] if k.startswith("bert.") else k): v.float() for k, v in raw.items()}


class BertReference:
    """fp32 torch encoder; ``embed`` returns mean-pooled last hidden states."""

    def __init__(self, cfg: BertConfig, weights: dict[str, torch.Tensor], device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.w = {k: v.to(self.device, torch.float32) for k, v in weights.items()}

    def _ln(self, x, name):
        return torch.nn.functional.layer_norm(x, (self.cfg.hidden,), self.w[name + ".weight"], self.w[name + ".bias"],
                                              self.cfg.layer_norm_eps)

    def _lin(self, x, name):
        return x @ self.w[name + ".weight"].t() + self.w[name + ".bias"]

    @torch.no_grad()
    def hidden(self, ids: list[int]) -> torch.Tensor:
        cfg = self.cfg
        S = len(ids)
        t = torch.tensor(ids, device=self.device)
        x = (self.w["embeddings.word_embeddings.weight"][t] + self.w["embeddings.position_embeddings.weight"][:S]
             + self.w["embeddings.token_type_embeddings.weight"][0])
        x = self._ln(x, "embeddings.LayerNorm")
        H, nh, hd = cfg.hidden, cfg.n_head, cfg.head_dim
        for i in range(cfg.n_layer):
            p = f"encoder.layer.{i}."
            q = self._lin(x, p + "attention.self.query").view(S, nh, hd).transpose(0, 1)
            k = self._lin(x, p + "attention.self.key").view(S, nh, hd).transpose(0, 1)
            v = self._lin(x, p + "attention.self.value").view(S, nh, hd).transpose(0, 1)
            att = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(hd), dim=-1)
            a = (att @ v).transpose(0, 1).reshape(S, H)
            x = self._ln(x + self._lin(a, p + "attention.output.dense"), p + "attention.output.LayerNorm")
            h = torch.nn.functional.gelu(self._lin(x, p + "intermediate.dense"))
            x = self._ln(x + self._lin(h, p + "output.dense"), p + "output.LayerNorm")
        return x

    def embed(self, batch: list[list[int]]) -> torch.Tensor:
        return torch.stack([self.hidden(ids).mean(0) for ids in batch])
