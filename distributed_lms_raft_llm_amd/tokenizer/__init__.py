"""Tokenizers backed by the native C++ library (``native/csrc/tokenizers.cpp``).

``GPT2BPE``      -- GPT-2 byte-level BPE (``tutoring_server.py:11,20,30``).  Pass the real
                    ``vocab.json``/``merges.txt`` to reproduce GPT-2 ids exactly; without them a
                    synthetic vocabulary is used (no network for the real files): byte tokens
                    plus, by default, one hashed id per word, so a prompt's token count is close
                    to real GPT-2's (the tutoring prompt template is ~25 tokens, not ~100 bytes).
``BertWordPiece``-- bert-base-uncased WordPiece (``lms_server.py:97-101``), ``vocab.txt`` or a
                    deterministic hashed synthetic vocabulary; ``[CLS] ... [SEP]``, truncation 512.
"""
from __future__ import annotations

import ctypes
import os

from .. import native

EOS = "<|endoftext|>"


class GPT2BPE:
    def __init__(self, vocab_json: str | None = None, merges_txt: str | None = None, eos_token_id: int = 50256,
                 synthetic_words: bool = True, vocab_size: int | None = None):
        """``vocab_size``: the model's vocabulary (synthetic word ids stay below it); default
        ``eos_token_id + 1`` (GPT-2's EOS is its last id)."""
        vocab_json = vocab_json or os.environ.get("DLMS_GPT2_VOCAB")
        merges_txt = merges_txt or os.environ.get("DLMS_GPT2_MERGES")
        L = native.lib()
        self._h = L.dlms_bpe_create(vocab_json.encode() if vocab_json else None,
                                    merges_txt.encode() if merges_txt else None)
        if not self._h:
            raise ValueError(f"could not load BPE vocabulary {vocab_json!r} / {merges_txt!r}")
        self.synthetic = bool(L.dlms_bpe_is_synthetic(self._h))
        self.eos_token_id = eos_token_id
        self.synthetic_words = False
        if self.synthetic and synthetic_words and (vocab_size or eos_token_id + 1) > 512:
            self.synthetic_words = L.dlms_bpe_set_synthetic_words(self._h, vocab_size or eos_token_id + 1) == 0

    def encode(self, text: str) -> list[int]:
        L = native.lib()
        ids: list[int] = []
        # <|endoftext|> is a special token, never merged through BPE
        pieces = text.split(EOS)
        for k, piece in enumerate(pieces):
            if k:
                ids.append(self.eos_token_id)
            if not piece:
                continue
            b = piece.encode("utf-8")
            cap = len(b) + 16
            buf = (ctypes.c_int * cap)()
            n = L.dlms_bpe_encode(self._h, b, len(b), buf, cap)
            if n > cap:
                buf = (ctypes.c_int * n)()
                n = L.dlms_bpe_encode(self._h, b, len(b), buf, n)
            ids.extend(buf[:n])
        return ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        L = native.lib()
        out: list[str] = []
        run: list[int] = []

        def flush():
            if run:
                arr = (ctypes.c_int * len(run))(*run)
                cap = 8 * len(run) + 64
                buf = ctypes.create_string_buffer(cap)
                n = L.dlms_bpe_decode(self._h, arr, len(run), buf, cap)
                if n > cap:
                    buf = ctypes.create_string_buffer(n)
                    n = L.dlms_bpe_decode(self._h, arr, len(run), buf, n)
                out.append(buf.raw[:n].decode("utf-8", errors="replace"))
                run.clear()

        for t in ids:
            if int(t) == self.eos_token_id:
                flush()
                if not skip_special_tokens:
                    out.append(EOS)
            else:
                run.append(int(t))
        flush()
        return "".join(out)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                native.lib().dlms_bpe_destroy(self._h)
        except Exception:
            pass


class BertWordPiece:
    def __init__(self, vocab_txt: str | None = None, vocab_size: int = 30522, max_length: int = 512):
        vocab_txt = vocab_txt or os.environ.get("DLMS_BERT_VOCAB")
        L = native.lib()
        self._h = L.dlms_wp_create(vocab_txt.encode() if vocab_txt else None, vocab_size)
        if not self._h:
            raise ValueError(f"could not load WordPiece vocabulary {vocab_txt!r}")
        self.synthetic = not vocab_txt
        self.max_length = max_length
        self.pad_token_id, self.cls_token_id, self.sep_token_id, self.unk_token_id = (
            L.dlms_wp_special(self._h, i) for i in range(4))

    def encode(self, text: str, max_length: int | None = None, add_special_tokens: bool = True) -> list[int]:
        L = native.lib()
        ml = self.max_length if max_length is None else max_length
        b = text.encode("utf-8")
        cap = len(b) + 8
        buf = (ctypes.c_int * cap)()
        n = L.dlms_wp_encode(self._h, b, len(b), ml, int(add_special_tokens), buf, cap)
        if n > cap:
            buf = (ctypes.c_int * n)()
            n = L.dlms_wp_encode(self._h, b, len(b), ml, int(add_special_tokens), buf, n)
        return list(buf[:n])

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                native.lib().dlms_wp_destroy(self._h)
        except Exception:
            pass
