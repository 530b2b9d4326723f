"""Model configurations for the tutoring LLM (GPT-2 family) and the relevance gate (BERT).

The reference loads ``gpt2`` (124M) in ``tutoring_server.py:10-12`` and
``bert-base-uncased`` in ``lms_server.py:1258-1260``.  There is no network on the
build/GPU boxes, so weights are random-initialised (seeded) with the same
architecture, or loaded from a local safetensors file when one is supplied.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict, field


@dataclass(frozen=True)
class GPT2Config:
    name: str = "gpt2"
    n_layer: int = 12
    n_embd: int = 768
    n_head: int = 12
    n_positions: int = 1024
    vocab_size: int = 50257
    layer_norm_epsilon: float = 1e-5
    eos_token_id: int = 50256
    initializer_range: float = 0.02

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    @property
    def n_inner(self) -> int:
        return 4 * self.n_embd

    @property
    def vocab_padded(self) -> int:
        # Padded to a multiple of 64 so the LM-head GEMM tiles evenly (50257 -> 50304).  (A
        # 256-multiple for 256x256 LM-head tiles measured 1 % slower in situ: profiles/r1_lmhead_256_ab.log)
        return (self.vocab_size + 63) // 64 * 64

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layer * self.n_embd * dtype_bytes

    def num_params(self) -> int:
        d, L, V, P = self.n_embd, self.n_layer, self.vocab_size, self.n_positions
        per_layer = 4 * d + (d * 3 * d + 3 * d) + (d * d + d) + (d * 4 * d + 4 * d) + (4 * d * d + d)
        return V * d + P * d + L * per_layer + 2 * d

    def to_dict(self) -> dict:
        return asdict(self)


GPT2_CONFIGS = {
    "gpt2": GPT2Config("gpt2", 12, 768, 12),
    "gpt2-small": GPT2Config("gpt2", 12, 768, 12),
    "gpt2-medium": GPT2Config("gpt2-medium", 24, 1024, 16),
    "gpt2-large": GPT2Config("gpt2-large", 36, 1280, 20),
    "gpt2-xl": GPT2Config("gpt2-xl", 48, 1600, 25),
    # tiny config for unit tests (fast on CPU, still exercises every code path)
    "gpt2-tiny": GPT2Config("gpt2-tiny", 2, 128, 2, n_positions=256, vocab_size=1000, eos_token_id=999),
}


def gpt2_config(name: str) -> GPT2Config:
    try:
        return GPT2_CONFIGS[name]
    except KeyError as e:
        raise ValueError(f"unknown GPT-2 config {name!r}; choose from {sorted(GPT2_CONFIGS)}") from e


@dataclass(frozen=True)
class BertConfig:
    name: str = "bert-base-uncased"
    n_layer: int = 12
    hidden: int = 768
    n_head: int = 12
    intermediate: int = 3072
    vocab_size: int = 30522
    max_position: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0
    cls_token_id: int = 101
    sep_token_id: int = 102
    initializer_range: float = 0.02

    @property
    def head_dim(self) -> int:
        return self.hidden // self.n_head


BERT_CONFIGS = {
    "bert-base-uncased": BertConfig(),
    "bert-tiny": BertConfig("bert-tiny", 2, 128, 2, 512, vocab_size=1000, max_position=128),
}


def bert_config(name: str) -> BertConfig:
    try:
        return BERT_CONFIGS[name]
    except KeyError as e:
        raise ValueError(f"unknown BERT config {name!r}; choose from {sorted(BERT_CONFIGS)}") from e


@dataclass
class GenerationConfig:
    """Decode semantics of the reference ``model.generate`` call (tutoring_server.py:21-29).

    ``do_sample`` is unset there, so decoding is greedy; ``temperature``/``top_k``/
    ``top_p`` are accepted and ignored for parity.
    """

    max_length: int = 150  # total length, prompt included
    repetition_penalty: float = 1.2
    do_sample: bool = False
    temperature: float = 0.7
    top_k: int = 50
    top_p: float = 0.9
    eos_token_id: int | None = None
    extra: dict = field(default_factory=dict)
