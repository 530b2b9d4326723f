"""The relevance gate as ONE batched service of the GPU tier (VERDICT r5 "what's missing" #2).

The reference gates inside every LMS server (``lms_server.py:97-104,1249-1271``: BERT re-loaded per
query, CPU), and its LMS servers run on separate machines (``README.md:104-110``).  Here the gate's
encoder lives where the GPU is: one ``GateServer`` per GPU (its own process, ``python -m
distributed_lms_raft_llm_amd.gate``, or hosted by the tutoring server with ``--gate-port``) holds ONE
HIP BERT encoder and batches the queries of every LMS node into shared encoder passes
(``RelevanceGate``'s adaptive window); LMS nodes -- GPU-less machines included -- call it through
``RemoteGate``, which keeps the local gate only as a fallback for when no gate server answers.

Wire: an internal gRPC service (``lmsinternal.Gate/<Method>``, JSON bodies through generic
handlers, like ``utils/debug_rpc.py``), so ``lms.proto`` stays byte-identical:

  Score  {"query", "key", ["text"]} -> {"similarity"} | {"missing": true}
         ``key`` = sha1 of the assignment text (``RelevanceGate._key``): the text itself travels only
         when the server has not embedded it yet ({"missing": true} asks for it once)
  ScoreBatch {"items": [{"query", "key", ["text"]}]} -> {"sims", "missing"}   the same for many
         queries: ``RemoteGate.check_async`` batches an LMS node's concurrent queries into one RPC
  Embed  {"text"} -> {"key"}      embed + cache an assignment (LMS nodes call it when a
                                   PostAssignment entry is applied, off the query path)

Deployment: its own process per GPU (``python -m distributed_lms_raft_llm_amd.gate``) is the serving
configuration.  Hosted inside the tutoring server (``--gate-port``) the gate's RPC and batching
threads share the tutor's interpreter lock with its decode loop: fine one query at a time (LMS path
p50 31.7 ms), but at 5.5 k q/s it starved the decode (165 k tok/s, profiles/r6_gate_tier.jsonl).

The similarity comes back raw; every LMS node applies its own threshold (``--gate-threshold``),
exactly the reference's ``< 0.6`` rule.
"""
from __future__ import annotations

import asyncio
import json
import logging
import threading
import time

import grpc

from ..utils.metrics import METRICS

log = logging.getLogger("dlms.gate.service")

SERVICE = "lmsinternal.Gate"


def _unary(fn):
    async def h(body: bytes, context) -> bytes:
        return json.dumps(await fn(json.loads(body) if body else {})).encode()

    return grpc.unary_unary_rpc_method_handler(h)


class GateServer:
    """aio gRPC server around one ``RelevanceGate`` (its batcher thread does the encoder passes)."""

    def __init__(self, gate, port: int = 0, host: str = "[::]"):
        self.gate = gate
        self.host, self.port = host, port
        self.scored = 0
        self.missing = 0
        self.batch_rpcs = 0
        self._loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self._loop.run_forever, name="gate-aio", daemon=True)
        self._thread.start()
        self._server = None

    async def _score(self, req: dict) -> dict:
        g = self.gate
        a = g._cache_get(req["key"])
        if a is None:
            text = req.get("text")
            if text is None:
                self.missing += 1
                return {"missing": True}
            a = await asyncio.get_running_loop().run_in_executor(None, g._cached, text)
        s = float(await asyncio.wrap_future(g._submit(req["query"], a)))
        self.scored += 1
        METRICS.inc("gate_service_scored")
        return {"similarity": s}

    async def _score_batch(self, req: dict) -> dict:
        """{"items": [{"query", "key", ["text"]}, ...]} -> {"sims": [float | null], "missing": [i, ...]}:
        one RPC per LMS-node batch (the per-RPC cost of a Python gRPC server, ~0.1 ms of GIL-held
        time, would otherwise cap the service near the 5.5 k q/s operating point)."""
        g = self.gate
        loop = asyncio.get_running_loop()
        items = req["items"]
        futs, missing = [], []
        for i, it in enumerate(items):
            a = g._cache_get(it["key"])
            if a is None:
                if it.get("text") is None:
                    missing.append(i)
                    futs.append(None)
                    continue
                a = await loop.run_in_executor(None, g._cached, it["text"])
            futs.append(asyncio.wrap_future(g._submit(it["query"], a)))
        sims = [None] * len(items)
        live = [(i, f) for i, f in enumerate(futs) if f is not None]
        for (i, _), v in zip(live, await asyncio.gather(*(f for _, f in live))):
            sims[i] = float(v)
        self.scored += len(live)
        self.missing += len(missing)
        self.batch_rpcs += 1
        METRICS.inc("gate_service_scored", len(live))
        return {"sims": sims, "missing": missing}

    async def _embed(self, req: dict) -> dict:
        text = req["text"]
        await asyncio.get_running_loop().run_in_executor(None, self.gate._cached, text)
        return {"key": self.gate._key(text)}

    def _health(self) -> dict:
        return {"gate": True, "scored": self.scored, "missing": self.missing, "batch_rpcs": self.batch_rpcs,
                "passes": self.gate.passes,
                "batched_queries": self.gate.batched_queries, "device": str(self.gate.device)}

    def start(self) -> "GateServer":
        from ..utils.debug_rpc import debug_handler

        async def make():
            srv = grpc.aio.server(options=[("grpc.max_receive_message_length", 64 << 20)])
            srv.add_generic_rpc_handlers((
                grpc.method_handlers_generic_handler(SERVICE, {"Score": _unary(self._score),
                                                               "ScoreBatch": _unary(self._score_batch),
                                                               "Embed": _unary(self._embed)}),
                debug_handler(health=self._health)))
            port = srv.add_insecure_port(f"{self.host}:{self.port}")
            await srv.start()
            return srv, port

        self._server, self.port = asyncio.run_coroutine_threadsafe(make(), self._loop).result(30)
        if not self.port:
            raise RuntimeError(f"gate server: could not bind {self.host}")
        log.info("gate server on port %d (%s)", self.port, self.gate.device)
        return self

    def stop(self, grace: float = 0.5):
        if self._server is not None:
            asyncio.run_coroutine_threadsafe(self._server.stop(grace), self._loop).result(10)
        self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(5)


class RemoteGate:
    """The LMS node's gate when the encoder lives in the GPU tier: ``check`` / ``check_async`` /
    ``attach_state`` like ``RelevanceGate``.  Tries the gate servers in order (a failed one is
    skipped for ``retry_s``); when none answers, the local ``fallback`` gate decides (created by
    ``fallback_factory`` on a background thread at start-up, so it is ready when needed), or -- no
    fallback -- the query is admitted (the tutoring tier still answers; the gate only filters)."""

    def __init__(self, addresses: list[str], threshold: float = 0.6, fallback_factory=None, timeout: float = 10.0,
                 retry_s: float = 2.0):
        if not addresses:
            raise ValueError("RemoteGate: at least one gate server address")
        self.addresses = list(addresses)
        self.threshold = threshold
        self.timeout = timeout
        self.retry_s = retry_s
        self._down_until = {a: 0.0 for a in self.addresses}
        self._sync_ch: dict[str, grpc.Channel] = {}
        self._aio_ch: dict[tuple[int, str], object] = {}
        self._lock = threading.Lock()
        self.remote_calls = 0
        self.fallbacks = 0
        self.max_inflight = 2  # ScoreBatch RPCs in flight per event loop
        self.max_batch = 256
        self._abatch: dict[int, dict] = {}
        self._fallback = None
        self._fallback_ready = threading.Event()
        if fallback_factory is not None:
            def build():
                try:
                    self._fallback = fallback_factory()
                except Exception:
                    log.exception("gate fallback could not be built")
                finally:
                    self._fallback_ready.set()

            threading.Thread(target=build, name="gate-fallback-init", daemon=True).start()
        else:
            self._fallback_ready.set()

    @staticmethod
    def key(text: str) -> str:
        from .relevance import RelevanceGate

        return RelevanceGate._key(text)

    def _live(self) -> list[str]:
        now = time.monotonic()
        live = [a for a in self.addresses if self._down_until[a] <= now]
        return live or list(self.addresses)  # all marked down: try them anyway

    def _mark_down(self, addr: str, err):
        self._down_until[addr] = time.monotonic() + self.retry_s
        METRICS.inc("gate_remote_errors")
        log.warning("gate server %s failed (%s)", addr, getattr(err, "code", lambda: err)())

    # ------------------------------------------------------------------ sync (threads front end)
    def _call(self, addr: str, method: str, req: dict) -> dict:
        with self._lock:
            ch = self._sync_ch.get(addr)
            if ch is None:
                ch = self._sync_ch[addr] = grpc.insecure_channel(addr)
        fn = ch.unary_unary(f"/{SERVICE}/{method}", request_serializer=None, response_deserializer=None)
        return json.loads(fn(json.dumps(req).encode(), timeout=self.timeout))

    def similarity(self, query: str, text: str) -> float:
        req = {"query": query, "key": self.key(text)}
        for addr in self._live():
            try:
                r = self._call(addr, "Score", req)
                if r.get("missing"):
                    r = self._call(addr, "Score", dict(req, text=text))
                self.remote_calls += 1
                METRICS.inc("gate_remote_calls")
                return float(r["similarity"])
            except grpc.RpcError as e:
                self._mark_down(addr, e)
        return self._fallback_similarity(query, text)

    def check(self, query: str, assignment_text: str) -> tuple[bool, float]:
        s = self.similarity(query, assignment_text)
        return s >= self.threshold, s

    # ------------------------------------------------------------------ async (aio front end)
    def _achannel(self, addr: str):
        loop = asyncio.get_running_loop()
        k = (id(loop), addr)
        ch = self._aio_ch.get(k)
        if ch is None:
            ch = self._aio_ch[k] = grpc.aio.insecure_channel(addr)
        return ch

    async def _acall(self, addr: str, method: str, req: dict) -> dict:
        fn = self._achannel(addr).unary_unary(f"/{SERVICE}/{method}", request_serializer=None,
                                              response_deserializer=None)
        return json.loads(await fn(json.dumps(req).encode(), timeout=self.timeout))

    async def check_async(self, query: str, assignment_text: str) -> tuple[bool, float]:
        """Queued for this node's next ScoreBatch RPC: a batch goes out at once when fewer than
        ``max_inflight`` are in flight, else when one returns (everything queued meanwhile rides
        along) -- no added wait at low load, one RPC per many queries under load."""
        loop = asyncio.get_running_loop()
        st = self._abatch.get(id(loop))
        if st is None:
            st = self._abatch[id(loop)] = {"queue": [], "inflight": 0}
        fut = loop.create_future()
        st["queue"].append((query, self.key(assignment_text), assignment_text, fut))
        if st["inflight"] < self.max_inflight:
            st["inflight"] += 1
            loop.create_task(self._flush(st))
        s = await fut
        return s >= self.threshold, s

    async def _flush(self, st: dict):
        try:
            while st["queue"]:
                batch, st["queue"] = st["queue"][: self.max_batch], st["queue"][self.max_batch:]
                sims = await self._score_remote(batch)
                for (_, _, _, fut), sv in zip(batch, sims):
                    if not fut.done():
                        fut.set_result(sv)
        finally:
            st["inflight"] -= 1

    async def _score_remote(self, batch) -> list[float]:
        items = [{"query": q, "key": k} for q, k, _, _ in batch]
        for addr in self._live():
            try:
                r = await self._acall(addr, "ScoreBatch", {"items": items})
                if r["missing"]:
                    again = [dict(items[i], text=batch[i][2]) for i in r["missing"]]
                    r2 = await self._acall(addr, "ScoreBatch", {"items": again})
                    for i, sv in zip(r["missing"], r2["sims"]):
                        r["sims"][i] = sv
                self.remote_calls += len(batch)
                METRICS.inc("gate_remote_calls", len(batch))
                METRICS.observe("gate_remote_batch", len(batch))
                return [float(x) for x in r["sims"]]
            except grpc.RpcError as e:
                self._mark_down(addr, e)
        loop = asyncio.get_running_loop()
        return [await loop.run_in_executor(None, self._fallback_similarity, q, t) for q, _, t, _ in batch]

    # ------------------------------------------------------------------ fallback / warm-up
    def _fallback_similarity(self, query: str, text: str) -> float:
        self.fallbacks += 1
        METRICS.inc("gate_remote_fallbacks")
        self._fallback_ready.wait()
        if self._fallback is None:
            return 1.0  # no gate anywhere: admit (the filter is advisory; the tutor still answers)
        return self._fallback.similarity(query, text)

    def warm(self, text: str):
        for addr in self._live():
            try:
                self._call(addr, "Embed", {"text": text})
                return
            except grpc.RpcError as e:
                self._mark_down(addr, e)

    def attach_state(self, state):
        """Embed assignment texts in the gate tier as PostAssignment entries are applied."""

        def on_apply(op, args):
            if op == "PostAssignment" and len(args) == 4:
                threading.Thread(target=self._safe_warm, args=(args[3],), daemon=True).start()

        state.listeners.append(on_apply)

    def _safe_warm(self, text):
        try:
            self.warm(text)
        except Exception:
            log.exception("remote gate warm-up failed")

    def close(self):
        for ch in self._sync_ch.values():
            ch.close()
        self._sync_ch.clear()


def main(argv=None):
    """``python -m distributed_lms_raft_llm_amd.gate``: one gate server (one encoder) for this GPU."""
    import argparse
    import os
    import signal

    from .relevance import RelevanceGate

    ap = argparse.ArgumentParser(description="relevance gate server (GPU tier)")
    ap.add_argument("--port", type=int, default=int(os.environ.get("DLMS_GATE_PORT", "50060")))
    ap.add_argument("--host", default="[::]")
    ap.add_argument("--model", default="bert-base-uncased")
    ap.add_argument("--device", default=os.environ.get("DLMS_GATE_DEVICE", "auto"))
    ap.add_argument("--weights", default=None)
    ap.add_argument("--vocab", default=None)
    ap.add_argument("--max-batch", type=int, default=127,
                    help="queries per shared encoder pass (<= 127: the encoder's hipGraph buckets hold 128 sequences)")
    ap.add_argument("--max-wait-ms", type=float, default=40.0,
                    help="under load a pass waits up to this long for company: fewer, fuller passes take less of the "
                         "GPU the tutor's decode needs (the tutor at 5.5 k q/s is ~0.76 s p50 anyway)")
    ap.add_argument("--cus", type=int, default=int(os.environ.get("DLMS_GATE_CUS", "0")),
                    help="under load, run encoder passes on a stream limited to this many CUs (0: all) -- the "
                         "rest stay free for a co-located tutor's decode")
    ap.add_argument("--log-level", default=os.environ.get("DLMS_LOG", "INFO"))
    args = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    gate = RelevanceGate.create(model=args.model, device=args.device, weights=args.weights, vocab=args.vocab)
    gate.max_batch = args.max_batch
    gate.max_wait_s = args.max_wait_ms / 1e3
    gate.fill_under_load = True
    if args.cus > 0 and str(gate.device).startswith("cuda"):
        from .. import ops

        gate.load_stream = ops.cu_masked_stream(args.cus)
        log.info("gate passes under load on %d CUs", args.cus)
    srv = GateServer(gate, args.port, args.host).start()
    print(f"Gate Server started on port {srv.port}", flush=True)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: done.set())
    signal.signal(signal.SIGINT, lambda *a: done.set())
    done.wait()
    srv.stop()


class GateWorker:
    """The gate's encoder inside the TUTORING ENGINE process, run by the continuous batcher between
    decode chunks (``ContinuousBatcher.attach_side_work``): each pass is enqueued on the decode
    stream right behind a chunk and read back asynchronously (a pinned copy + event, like the
    batcher's stop flags), so the relevance gate never time-slices the GPU with another process
    and never interleaves kernel by kernel with a decode chunk.  The tutor's front-end processes
    terminate the gate's gRPC calls and tokenize (``tutor/frontend.py``: ``lmsinternal.Gate`` on the
    tutoring port); this object sees token ids only.

    Items: ``(query_ids | None, key, assignment_ids | None)``: score the query against the assignment
    embedding cached under ``key`` -- embedding ``assignment_ids`` in the same pass when given and not
    cached yet; ``query_ids`` None = embed only.  Results per item: a float, "missing" (key unknown,
    no text sent) or None (embed only)."""

    def __init__(self, encoder, max_seqs: int = 127, cache_size: int = 8192, min_gap_s: float = 0.0):
        self.enc = encoder
        self.max_seqs = max_seqs
        self.min_gap_s = min_gap_s  # under load: at most one pass per this interval (fuller passes)
        self.cache: "OrderedDict[str, object]" = __import__("collections").OrderedDict()
        self.cache_size = cache_size
        self._lock = threading.Lock()
        self._pending: list = []  # (items, cb)
        self._inflight = __import__("collections").deque()  # passes enqueued, oldest first
        self.max_inflight = 4  # passes in flight = passes per decode-chunk gap under load
        self._last_start = 0.0
        self.passes = 0
        self.scored = 0
        self.batcher = None

    def attach(self, batcher):
        self.batcher = batcher
        batcher.attach_side_work(self.work, self.pending)

    def submit(self, items: list, cb):
        with self._lock:
            self._pending.append((items, cb))
        if self.batcher is not None:
            self.batcher.kick()

    def _split(self, items, cb, n: int):
        """(head, tail) of one request that does not fit the pass being packed: head = its first n
        items, tail = the rest; cb gets the results of both, in item order, once both have them."""
        got = [None, None]

        def part(idx):
            def f(res):
                got[idx] = res
                if got[0] is not None and got[1] is not None:
                    cb(got[0] + got[1])
            return f

        return (items[:n], part(0)), (items[n:], part(1))

    def _need(self, items, new_keys, limit: int | None = None):
        """Encoder sequences the items need (a query each, plus each assignment neither cached nor
        already in this pass); with ``limit``: how many leading items fit in ``limit`` sequences."""
        n, seen = 0, set()
        for i, (q, k, a) in enumerate(items):
            add = q is not None
            add += a is not None and k not in seen and k not in new_keys and self._cached(k) is None
            if limit is not None and n + add > limit:
                return i
            n += add
            if a is not None:
                seen.add(k)
        return len(items) if limit is not None else n

    def pending(self) -> bool:
        return bool(self._pending) or bool(self._inflight)

    def _cached(self, key):
        v = self.cache.get(key)
        if v is not None:
            self.cache.move_to_end(key)
        return v

    def work(self, idle: bool):
        while self._inflight:
            ev = self._inflight[0][0]
            if idle:
                ev.synchronize()
            if not ev.query():
                break
            self._deliver()
        now = time.monotonic()
        if not idle and now - self._last_start < self.min_gap_s:
            return
        # up to max_inflight passes back to back between two decode chunks (one pass per chunk
        # capped the served gate at ~2.35 k queries/s at 5.5 k q/s offered: profiles/r6_gate_tier_final.jsonl)
        while self._pending and len(self._inflight) < self.max_inflight:
            if not self._one_pass(now):
                break

    def _one_pass(self, now: float) -> bool:
        """Pack and enqueue one encoder pass; False when no request could be taken."""
        import torch

        # one pass: requests packed into max_seqs encoder sequences; the request that does not fit
        # any more is split so its head fills the pass (its callback fires once every item has a
        # result) -- whole-request packing left passes half full when requests were large
        with self._lock:
            take, nseq, new_keys = [], 0, {}
            while self._pending and nseq < self.max_seqs:
                items, cb = self._pending[0]
                need = self._need(items, new_keys)
                if nseq + need <= self.max_seqs:
                    self._pending.pop(0)
                else:
                    room = self.max_seqs - nseq
                    cnt = self._need(items, new_keys, limit=room)
                    if cnt == 0 or (take and room < 16):  # not worth a split for a sliver
                        break
                    head, tail = self._split(items, cb, cnt)
                    self._pending[0] = tail
                    items, cb = head
                    need = self._need(items, new_keys)
                take.append((items, cb))
                nseq += need
                for q, k, a in items:
                    if a is not None and self._cached(k) is None:
                        new_keys.setdefault(k, a)
        if not take:
            return False
        seqs, qrefs = [], []  # qrefs: (request index, item index, assignment key)
        results = [[None] * len(items) for items, _ in take]
        for ri, (items, _) in enumerate(take):
            for ii, (q, k, a) in enumerate(items):
                if q is None:
                    continue
                if self._cached(k) is None and k not in new_keys:
                    results[ri][ii] = "missing"
                    continue
                qrefs.append((ri, ii, k))
                seqs.append(q)
        keys = list(new_keys)
        seqs += [new_keys[k] for k in keys]
        self._last_start = now
        if not seqs:
            self._finish(None, take, results, qrefs)
            return True
        with torch.no_grad():
            pooled = self.enc.embed(seqs).float()
            for j, k in enumerate(keys):
                self.cache[k] = pooled[len(qrefs) + j]
                if len(self.cache) > self.cache_size:
                    self.cache.popitem(last=False)
            host = None
            gpu = pooled.is_cuda
            if qrefs:
                q = pooled[: len(qrefs)]
                a = torch.stack([self.cache[k] for _, _, k in qrefs])
                if hasattr(self.enc, "cosine"):  # the HIP cosine kernel (encoder.hip): [n, n], the diagonal
                    sims = torch.diagonal(self.enc.cosine(q, a)).float().contiguous()
                else:
                    sims = torch.nn.functional.cosine_similarity(q, a, dim=1, eps=1e-8)
                if gpu:  # read back behind the pass, without waiting for it here
                    host = torch.empty(len(qrefs), dtype=torch.float32, pin_memory=True)
                    host.copy_(sims, non_blocking=True)
                else:
                    host = sims
        self.passes += 1
        if gpu:
            ev = torch.cuda.Event()
            ev.record()
            self._inflight.append((ev, host, take, results, qrefs))
        else:
            self._finish(host, take, results, qrefs)
        return True

    def _deliver(self):
        _, host, take, results, qrefs = self._inflight.popleft()
        self._finish(host, take, results, qrefs)

    def _finish(self, host, take, results, qrefs):
        if host is not None:
            for (ri, ii, _), s in zip(qrefs, host.tolist()):
                results[ri][ii] = float(s)
            self.scored += len(qrefs)
            METRICS.inc("gate_service_scored", len(qrefs))
        for (items, cb), res in zip(take, results):
            try:
                cb(res)
            except Exception:  # noqa: BLE001 -- one caller's relay error must not stop the batcher
                log.exception("gate result delivery failed")
