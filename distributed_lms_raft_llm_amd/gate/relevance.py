"""BERT relevance gate for ``GetLLMAnswer`` (C11, ``lms_server.py:97-104,1249-1271``).

Semantics kept: bert-base-uncased, mean of ``last_hidden_state`` over all tokens ([CLS] and [SEP]
included), truncation at 512 tokens, cosine similarity, reject when ``< 0.6``.

What changes (SURVEY.md §7.1 design choice 2): the model is built ONCE per process (the reference
re-loads it from disk on every query, ~563 ms), runs on the MI355X through the HIP kernels
(``engine/bert_engine.py``) -- or the torch reference on CPU hosts -- and assignment embeddings are
computed when the PostAssignment entry is applied and cached, so a query costs one short
encoder pass -- and concurrent queries SHARE that pass: ``check`` hands its query to a small
batching thread that packs every query waiting within ``window_ms`` (or up to ``max_batch``) into
one varlen encoder pass (the reference runs a full BERT forward per request, on CPU, after
re-loading the model).
"""
from __future__ import annotations

import hashlib
import logging
import os
import threading
import time
from collections import OrderedDict
from concurrent.futures import Future

import torch

from ..models.bert import BertReference, init_bert_weights, load_bert_safetensors
from ..models.config import bert_config
from ..tokenizer import BertWordPiece
from ..utils.metrics import METRICS

log = logging.getLogger("dlms.gate")


class RelevanceGate:
    def __init__(self, encoder, tokenizer: BertWordPiece, threshold: float = 0.6, cache_size: int = 4096,
                 window_ms: float = 1.0, max_batch: int = 64):
        self.encoder = encoder
        self.tok = tokenizer
        self.threshold = threshold
        self._cache: OrderedDict[str, torch.Tensor] = OrderedDict()
        self._cache_size = cache_size
        self._lock = threading.Lock()  # one encoder pass at a time (GPU stream / CPU threads)
        # the embedding cache has its own lock, never held across encoder work: the aio front end
        # reads it on the event-loop thread while the batcher may be inside a long encoder pass
        self._cache_lock = threading.Lock()
        self.device = getattr(encoder, "device", torch.device("cpu"))
        # query batching: concurrent GetLLMAnswer calls share one packed encoder pass
        self.window_s = window_ms / 1e3
        self.max_batch = max_batch
        self._pending: list[tuple[list[int], torch.Tensor, Future]] = []
        self._pcv = threading.Condition()
        self._batcher: threading.Thread | None = None
        self.passes = 0
        self.batched_queries = 0
        self._last_pass_s = 0.0  # duration of the previous encoder pass (adaptive batching window)
        # cap of that adaptive wait (DLMS_GATE_MAX_WAIT_MS): longer = fewer, larger passes beside
        # the tutoring decode on a shared GPU, at that much more gate latency
        self.max_wait_s = float(os.environ.get("DLMS_GATE_MAX_WAIT_MS", "8")) / 1e3
        self._last_end = 0.0
        # fill_under_load: under load a pass waits for max_batch queries (up to max_wait_s) instead
        # of for as long as the previous pass took -- the gate service (gate/service.py) runs the
        # cross-node batch this way so its passes take as little of the tutor's GPU as possible
        self.fill_under_load = False
        # under load, passes run on this stream (a CU-masked one: gate/service.py --cus) so that
        # they never hold the CUs a co-located tutor's decode kernels are waiting for
        self.load_stream = None

    @classmethod
    def create(cls, model: str = "bert-base-uncased", device: str = "auto", threshold: float = 0.6,
               weights: str | None = None, vocab: str | None = None, seed: int = 0):
        cfg = bert_config(model)
        w = load_bert_safetensors(weights) if weights else init_bert_weights(cfg, seed=seed)
        if device == "auto":
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if str(device).startswith("cuda"):
            from ..engine.bert_engine import HipBertEncoder

            enc = HipBertEncoder(cfg, w, device=device)
            if os.environ.get("DLMS_GATE_WARM", "1") != "0":
                t0 = time.perf_counter()
                n = enc.warm_graphs()
                log.info("relevance gate: %d encoder graphs captured in %.2f s", n, time.perf_counter() - t0)
        else:
            enc = BertReference(cfg, w, device="cpu")
        tok = BertWordPiece(vocab, vocab_size=cfg.vocab_size, max_length=cfg.max_position)
        log.info("relevance gate: %s on %s (%s vocab)", model, device, "synthetic" if tok.synthetic else "real")
        return cls(enc, tok, threshold)

    # ------------------------------------------------------------------ embeddings
    @staticmethod
    def _key(text: str) -> str:
        return hashlib.sha1(text.encode("utf-8")).hexdigest()

    def embed(self, texts: list[str]) -> torch.Tensor:
        ids = [self.tok.encode(t) for t in texts]
        with self._lock, torch.no_grad():
            return self.encoder.embed(ids).float()

    def _cached(self, text: str) -> torch.Tensor:
        k = self._key(text)
        v = self._cache_get(k)
        if v is not None:
            return v
        v = self.embed([text])[0]
        with self._cache_lock:
            self._cache[k] = v
            if len(self._cache) > self._cache_size:
                self._cache.popitem(last=False)
        return v

    def _cache_get(self, k: str) -> torch.Tensor | None:
        with self._cache_lock:
            v = self._cache.get(k)
            if v is not None:
                self._cache.move_to_end(k)
            return v

    def warm(self, text: str):
        self._cached(text)

    # ------------------------------------------------------------------ query batching
    def _submit(self, text: str, a: torch.Tensor) -> Future:
        """Queue the query for the next shared batch; the Future resolves to cosine(query, ``a``)."""
        fut: Future = Future()
        ids = self.tok.encode(text)
        with self._pcv:
            if self._batcher is None:
                self._batcher = threading.Thread(target=self._batch_loop, name="gate-batcher", daemon=True)
                self._batcher.start()
            self._pending.append((ids, a, fut))
            self._pcv.notify()
        return fut

    def _score(self, text: str, a: torch.Tensor) -> float:
        """Cosine(query embedding, ``a``), computed in the next shared batch."""
        return self._submit(text, a).result()

    def _cosines(self, q: torch.Tensor, a: torch.Tensor) -> list[float]:
        if hasattr(self.encoder, "cosine"):  # HIP cosine kernel: [n, n], keep the diagonal
            return torch.diagonal(self.encoder.cosine(q, a)).float().cpu().tolist()
        return torch.nn.functional.cosine_similarity(q, a, dim=1).tolist()

    def _batch_loop(self):
        while True:
            with self._pcv:
                while not self._pending:
                    self._pcv.wait()
                # the first query waits for company: window_s when the gate was idle, but under
                # load as long as the previous pass took (capped at max_wait_s) -- queries keep arriving
                # during a pass anyway, and every pass is a chain of small kernels that competes with
                # the tutoring decode for the same GPU, so one pass per several queries is the point
                # (serving bench: 1 ms windows gave ~1 query per pass at 1.2 k q/s per node and
                # slowed the co-located tutor's decode ~2x)
                now = time.monotonic()
                busy = now - self._last_end < 0.05
                if busy and self.fill_under_load:
                    wait = self.max_wait_s
                else:
                    wait = min(max(self.window_s, self._last_pass_s if busy else 0.0), self.max_wait_s)
                end = now + wait
                while len(self._pending) < self.max_batch and time.monotonic() < end:
                    self._pcv.wait(max(0.0, end - time.monotonic()))
                batch, self._pending = self._pending[: self.max_batch], self._pending[self.max_batch:]
            t_pass = time.monotonic()
            try:
                import contextlib

                ctx = torch.cuda.stream(self.load_stream) if (busy and self.load_stream is not None) else \
                    contextlib.nullcontext()
                with self._lock, torch.no_grad(), ctx:
                    q = self.encoder.embed([ids for ids, _, _ in batch]).float()
                    a = torch.stack([x.to(q.device, torch.float32) for _, x, _ in batch])
                    sims = self._cosines(q, a)  # one device->host copy for the whole batch
                self.passes += 1
                self.batched_queries += len(batch)
                METRICS.observe("gate_batch", len(batch))
                self._last_end = time.monotonic()
                self._last_pass_s = self._last_end - t_pass
                for s, (_, _, fut) in zip(sims, batch):
                    fut.set_result(float(s))
            except BaseException as e:  # never strand a caller
                for _, _, fut in batch:
                    if not fut.done():
                        fut.set_exception(e)

    def similarity(self, query: str, text: str) -> float:
        return self._score(query, self._cached(text))

    def check(self, query: str, assignment_text: str) -> tuple[bool, float]:
        s = self.similarity(query, assignment_text)
        return s >= self.threshold, s

    async def check_async(self, query: str, assignment_text: str) -> tuple[bool, float]:
        """``check`` for an event loop: the query waits for its shared batch WITHOUT holding a
        thread (the LMS aio front end's GetLLMAnswer); only an assignment-embedding cache miss
        (normally computed when the PostAssignment entry was applied) runs on the executor."""
        import asyncio

        loop = asyncio.get_running_loop()
        a = self._cache_get(self._key(assignment_text))  # never waits on an encoder pass
        if a is None:
            a = await loop.run_in_executor(None, self._cached, assignment_text)
        s = float(await asyncio.wrap_future(self._submit(query, a)))
        return s >= self.threshold, s

    def attach_state(self, state):
        """Embed assignment texts as PostAssignment entries are applied (off the query path)."""

        def on_apply(op, args):
            if op == "PostAssignment" and len(args) == 4:
                threading.Thread(target=self._safe_warm, args=(args[3],), daemon=True).start()

        state.listeners.append(on_apply)

    def _safe_warm(self, text):
        try:
            self.warm(text)
        except Exception:
            log.exception("gate warm-up failed")
