"""Tutoring service (``lms.Tutoring.GetLLMAnswer``) backed by the MI355X GPT-2 engine.

Reference behaviour (``tutoring_server.py:15-49``): wrap the query in a fixed prompt, run GPT-2
``generate(max_length=150, repetition_penalty=1.2)`` (greedy), return the decoded sequence -- prompt
included -- with ``success=True``; listen on ``[::]:50054`` with 10 worker threads.

Here concurrent queries are batched.  On the GPU engine the default is continuous batching
(``engine/scheduler.py``): a query is prefilled into a free KV-cache slot of the running batch as
soon as it arrives and leaves at its own EOS/max_length, every live query advancing in
hipGraph-replayed decode chunks.  The window batcher (``--batching window``, and the only mode of
the CPU torch reference engine, BASELINE config 1) collects requests for up to
``batch_window_ms`` (or until ``max_batch``) and runs them as one batched ``generate``.
Per-request latency, batch sizes and tokens/s land in the metrics registry.
"""
from __future__ import annotations

import argparse
import logging
import os
import queue
import signal
import threading
import time
from concurrent import futures
from dataclasses import dataclass

import grpc
import torch

from .. import wire
from ..engine.scheduler import Overloaded
from ..models.config import GenerationConfig, gpt2_config
from ..models.gpt2 import init_gpt2_weights, load_safetensors_weights
from ..tokenizer import GPT2BPE
from ..utils.config import parse_with_config
from ..utils.debug_rpc import debug_handler
from ..utils.metrics import METRICS
from ..wire import pb

log = logging.getLogger("dlms.tutor")

PROMPT_TEMPLATE = ("You are an intelligent assistant. Answer the following question in detail:\n"
                   "Question: {query}\nAnswer:")


def default_max_queue(engine, max_queue: int | None) -> int:
    """Admission limit of a serving replica: queries that may wait for a KV slot beyond the
    engine's slots (one batch of slots by default -- about one generation of queueing delay)
    before it answers RESOURCE_EXHAUSTED; 0 = unbounded."""
    return engine.max_batch if max_queue is None else int(max_queue)


def build_prompt(query: str) -> str:
    return PROMPT_TEMPLATE.format(query=query)


@dataclass
class _Req:
    ids: list[int]
    fut: futures.Future
    t0: float


class Batcher:
    """Dynamic batching in front of an engine with ``generate(prompts, max_length, penalty)``."""

    def __init__(self, engine, gen: GenerationConfig, max_batch: int = 64, window_ms: float = 2.0):
        self.engine = engine
        self.gen = gen
        self.max_batch = max_batch
        self.window = window_ms / 1e3
        self.q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, name="tutor-batcher", daemon=True)
        self._t.start()

    def submit(self, ids: list[int]) -> futures.Future:
        f: futures.Future = futures.Future()
        self.q.put(_Req(ids, f, time.perf_counter()))
        METRICS.set("tutor_queue_depth", self.q.qsize())
        return f

    def _loop(self):
        while not self._stop.is_set():
            try:
                first = self.q.get(timeout=0.1)
            except queue.Empty:
                continue
            batch = [first]
            deadline = time.perf_counter() + self.window
            while len(batch) < self.max_batch:
                rem = deadline - time.perf_counter()
                if rem <= 0:
                    break
                try:
                    batch.append(self.q.get(timeout=rem))
                except queue.Empty:
                    break
            self._run(batch)

    def _run(self, batch: list[_Req]):
        t0 = time.perf_counter()
        try:
            outs = self.engine.generate([r.ids for r in batch], self.gen.max_length, self.gen.repetition_penalty)
        except Exception as e:  # fail the whole batch, keep serving
            log.exception("generation failed")
            for r in batch:
                r.fut.set_exception(e)
            return
        dt = time.perf_counter() - t0
        new = sum(len(o) - len(r.ids) for o, r in zip(outs, batch))
        METRICS.observe("tutor_batch_size", len(batch))
        METRICS.observe("tutor_batch_ms", dt * 1e3)
        METRICS.inc("tutor_tokens_generated", new)
        METRICS.set("tutor_tokens_per_s", new / dt if dt > 0 else 0.0)
        now = time.perf_counter()
        for o, r in zip(outs, batch):
            METRICS.observe("tutor_query_ms", (now - r.t0) * 1e3)
            r.fut.set_result(o)

    def stop(self):
        self._stop.set()
        self._t.join(timeout=2)


class TutoringServicer:
    def __init__(self, batcher: Batcher, tokenizer: GPT2BPE, max_length: int, timeout: float = 300.0):
        self.batcher = batcher
        self.tok = tokenizer
        self.max_length = max_length
        self.timeout = timeout

    def GetLLMAnswer(self, request, context):
        # like generate(), a prompt already at max_length comes back unchanged (engines handle it)
        ids = self.tok.encode(build_prompt(request.query))
        try:
            out = self.batcher.submit(ids).result(timeout=self.timeout)
        except Overloaded as e:  # shed load now rather than queue past the client's deadline
            context.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, str(e))
        except Exception as e:
            # a failed batcher (e.g. a tensor-parallel peer stalled in an xGMI collective) will not
            # serve again in this process: UNAVAILABLE makes the LMS's TutoringClient fail over to
            # a healthy replica (INTERNAL is not retried), and TutoringServer exits this process
            # for its supervisor to restart
            failed = getattr(self.batcher, "failed", None) is not None
            code = grpc.StatusCode.UNAVAILABLE if failed else grpc.StatusCode.INTERNAL
            context.abort(code, f"generation failed: {e}")
        return pb.QueryResponse(success=True, response=self.tok.decode(out, skip_special_tokens=True))


def make_engine(model: str, device: str, max_batch: int, max_length: int, weights: str | None = None, seed: int = 0,
                tp_group=None, weight_dtype: str = "bf16"):
    """GPU: the HIP engine (TP over ``tp_group`` when given).  CPU: the torch reference engine, or
    the sharded torch slot engine when a (gloo) TP group is given."""
    cfg = gpt2_config(model)
    w = load_safetensors_weights(weights) if weights else init_gpt2_weights(cfg, seed=seed)
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    if device.startswith("cuda"):
        from ..engine.gpt2_engine import HipGPT2Engine

        return HipGPT2Engine(cfg, w, device=device, max_batch=max_batch, max_length=max_length, tp_group=tp_group,
                             weight_dtype=weight_dtype)
    if tp_group is not None:
        from ..parallel.tp import TorchSlotEngine

        return TorchSlotEngine(cfg, w, group=tp_group, max_batch=max_batch or 8, max_length=max_length)
    from ..engine.gpt2_engine import TorchGPT2Engine

    return TorchGPT2Engine(cfg, w, max_length=max_length)


def make_gate_worker(model: str, weights: str | None, device):
    """The relevance gate's encoder for ``--serve-gate`` (gate/service.py GateWorker): the HIP BERT
    on the tutor's GPU (its graphs captured now), or the torch reference on a CPU engine."""
    import torch

    from ..gate.service import GateWorker
    from ..models.bert import BertReference, init_bert_weights, load_bert_safetensors
    from ..models.config import bert_config

    cfg = bert_config(model)
    w = load_bert_safetensors(weights) if weights else init_bert_weights(cfg, seed=0)
    if str(device).startswith("cuda") and torch.cuda.is_available():
        from ..engine.bert_engine import HipBertEncoder

        enc = HipBertEncoder(cfg, w, device=device, graph_max_rows=8192, graph_max_seqs=256)
        enc.warm_graphs()
    else:
        enc = BertReference(cfg, w, device="cpu")
    log.info("relevance gate served on the tutoring port (%s on %s, passes between decode chunks)", model, device)
    # under load at most one pass per DLMS_GATE_MIN_GAP_MS (fuller passes, fewer stops of the decode
    # stream); idle, a query is scored at the next batcher iteration
    return GateWorker(enc, max_seqs=255 if str(device).startswith("cuda") else 127,
                      min_gap_s=float(os.environ.get("DLMS_GATE_MIN_GAP_MS", "10")) / 1e3)


class TutoringServer:
    def __init__(self, engine, port: int = 50054, host: str = "[::]", max_batch: int = 64, window_ms: float = 2.0,
                 max_length: int = 150, repetition_penalty: float = 1.2, tokenizer: GPT2BPE | None = None,
                 workers: int = 64, batching: str = "auto", chunk: int = 8, max_queue: int | None = None):
        self.gen = GenerationConfig(max_length=max_length, repetition_penalty=repetition_penalty)
        self.tok = tokenizer or GPT2BPE(eos_token_id=getattr(getattr(engine, "cfg", None), "eos_token_id", 50256))
        if batching == "auto":
            batching = "continuous" if hasattr(engine, "admit") else "window"
        if batching == "continuous":
            from ..engine.scheduler import ContinuousBatcher

            if engine.max_length != max_length:
                raise ValueError("continuous batching: engine max_length differs from the server's")
            self.batcher = ContinuousBatcher(engine, repetition_penalty, chunk=chunk,
                                             max_queue=default_max_queue(engine, max_queue))
        else:
            self.batcher = Batcher(engine, self.gen, max_batch=max_batch, window_ms=window_ms)
        self.batching = batching
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                                  options=[("grpc.max_send_message_length", wire.DEFAULT_MAX_MESSAGE),
                                           ("grpc.max_receive_message_length", wire.DEFAULT_MAX_MESSAGE)])
        wire.register(self.server, "Tutoring", TutoringServicer(self.batcher, self.tok, max_length))
        self.engine = engine
        self._stopping = threading.Event()
        self.server.add_generic_rpc_handlers((debug_handler(health=self._health),))
        self.port = self.server.add_insecure_port(f"{host}:{port}")
        if self.port == 0:
            raise RuntimeError(f"could not bind {host}:{port}")

    def _health(self) -> dict:
        b = self.batcher
        out = {"batching": self.batching, "engine": type(getattr(self.engine, "engine", self.engine)).__name__,
               "max_length": self.gen.max_length}
        eng = getattr(self.engine, "engine", self.engine)
        if getattr(eng, "device", None) is not None and eng.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(eng.device)
            out.update(hbm_used_gb=round((total - free) / 2**30, 2), hbm_total_gb=round(total / 2**30, 2),
                       kv_cache_gb=round(eng.kv_cache_bytes() / 2**30, 3), slots=eng.max_batch)
            METRICS.set("tutor_hbm_used_gb", out["hbm_used_gb"])
        if self.batching == "continuous":
            out.update(active=b.active, completed=b.completed, ok=b._error is None and b._thread.is_alive())
        else:
            out.update(queued=b.q.qsize(), ok=b._t.is_alive())
        gw = getattr(getattr(self, "pool", None), "gate_worker", None)
        if gw is not None:  # --serve-gate: the relevance gate's passes between decode chunks
            out.update(gate=True, scored=gw.scored, passes=gw.passes, batched_queries=gw.scored,
                       device=str(getattr(gw.enc, "device", "cpu")))
        return out

    def start(self, on_fatal=None, poll_s: float = 0.25):
        """``on_fatal(error)``: called once if the batcher fails for good (a stalled TP peer, a
        device error): the CLI exits the process non-zero so a supervisor starts a fresh one --
        never a re-exec of a process that initialised the GPU."""
        self.server.start()
        log.info("tutoring server on port %d", self.port)
        self._arm_fatal(on_fatal, poll_s)
        return self

    def _arm_fatal(self, on_fatal, poll_s: float):
        if on_fatal is not None:
            def watch():
                while not self._stopping.is_set():
                    err = getattr(self.batcher, "failed", None)
                    if err is not None:
                        log.error("batcher failed (%s): this replica stops serving", err)
                        METRICS.inc("tutor_fatal_total")
                        on_fatal(err)
                        return
                    self._stopping.wait(poll_s)

            threading.Thread(target=watch, name="tutor-fatal-watch", daemon=True).start()

    def stop(self):
        self._stopping.set()
        self.server.stop(0.5).wait()
        self.batcher.stop()


class AioTutoringServicer:
    """``Tutoring.GetLLMAnswer`` as a coroutine: a query holds no thread while it decodes (the
    threaded servicer parks one worker per query, capping a replica at ``workers`` queries in
    flight -- far below the 1024-query operating point)."""

    def __init__(self, batcher, tokenizer: GPT2BPE, timeout: float = 300.0):
        self.batcher = batcher
        self.tok = tokenizer
        self.timeout = timeout

    async def GetLLMAnswer(self, request, context):
        import asyncio

        ids = self.tok.encode(build_prompt(request.query))
        try:
            out = await asyncio.wait_for(asyncio.wrap_future(self.batcher.submit(ids)), self.timeout)
        except Overloaded as e:
            await context.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, str(e))
        except Exception as e:
            failed = getattr(self.batcher, "failed", None) is not None
            code = grpc.StatusCode.UNAVAILABLE if failed else grpc.StatusCode.INTERNAL
            await context.abort(code, f"generation failed: {e}")
        return pb.QueryResponse(success=True, response=self.tok.decode(out, skip_special_tokens=True))


class AioTutoringServer(TutoringServer):
    """The continuous-batching tutoring server with a ``grpc.aio`` front end on its own event-loop
    thread: thousands of queries in flight per replica (the reference's tutoring
    server is a 10-thread synchronous gRPC server).  Same engine, batcher, health/debug RPCs,
    fatal hook and stop() as ``TutoringServer``."""

    def __init__(self, engine, port: int = 50054, host: str = "[::]", max_length: int = 150,
                 repetition_penalty: float = 1.2, tokenizer: GPT2BPE | None = None, chunk: int = 8,
                 max_queue: int | None = None):
        import asyncio

        from ..engine.scheduler import ContinuousBatcher

        if not hasattr(engine, "admit"):
            raise ValueError("the aio front end needs a slot engine (continuous batching)")
        if engine.max_length != max_length:
            raise ValueError("continuous batching: engine max_length differs from the server's")
        self.gen = GenerationConfig(max_length=max_length, repetition_penalty=repetition_penalty)
        self.tok = tokenizer or GPT2BPE(eos_token_id=getattr(getattr(engine, "cfg", None), "eos_token_id", 50256))
        self.batcher = ContinuousBatcher(engine, repetition_penalty, chunk=chunk,
                                             max_queue=default_max_queue(engine, max_queue))
        self.batching = "continuous"
        self.engine = engine
        self._stopping = threading.Event()
        self._loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self._loop.run_forever, name="tutor-aio", daemon=True)
        self._thread.start()

        async def make():
            srv = grpc.aio.server(migration_thread_pool=futures.ThreadPoolExecutor(max_workers=4),
                                  options=[("grpc.max_send_message_length", wire.DEFAULT_MAX_MESSAGE),
                                           ("grpc.max_receive_message_length", wire.DEFAULT_MAX_MESSAGE)])
            wire.register(srv, "Tutoring", AioTutoringServicer(self.batcher, self.tok))
            srv.add_generic_rpc_handlers((debug_handler(health=self._health),))
            return srv, srv.add_insecure_port(f"{host}:{port}")

        self.server, self.port = asyncio.run_coroutine_threadsafe(make(), self._loop).result(30)
        if self.port == 0:
            raise RuntimeError(f"could not bind {host}:{port}")

    def start(self, on_fatal=None, poll_s: float = 0.25):
        import asyncio

        asyncio.run_coroutine_threadsafe(self.server.start(), self._loop).result(30)
        log.info("tutoring server (aio) on port %d", self.port)
        self._arm_fatal(on_fatal, poll_s)
        return self

    def stop(self):
        import asyncio

        self._stopping.set()
        try:
            asyncio.run_coroutine_threadsafe(self.server.stop(0.5), self._loop).result(10)
        finally:
            self.batcher.stop()
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(5)


class PooledTutoringServer(TutoringServer):
    """The continuous-batching engine behind ``n`` front-end processes (``tutor/frontend.py``):
    this process keeps the GPU and the scheduler; gRPC termination and (de)tokenization run in
    the front ends, which share the public port.  Same health/metrics surface, fatal hook and
    stop() as ``TutoringServer``."""

    def __init__(self, engine, pool, max_length: int = 150, repetition_penalty: float = 1.2, chunk: int = 8,
                 max_queue: int | None = None):
        from ..engine.scheduler import ContinuousBatcher

        if not hasattr(engine, "admit"):
            raise ValueError("the front-end pool needs a slot engine (continuous batching)")
        if engine.max_length != max_length:
            raise ValueError("continuous batching: engine max_length differs from the server's")
        self.gen = GenerationConfig(max_length=max_length, repetition_penalty=repetition_penalty)
        self.batcher = ContinuousBatcher(engine, repetition_penalty, chunk=chunk,
                                             max_queue=default_max_queue(engine, max_queue))
        self.batching = "continuous"
        self.engine = engine
        self.pool = pool
        self.port = 0
        self._stopping = threading.Event()

    def start(self, on_fatal=None, poll_s: float = 0.25):
        self.pool.serve(self.batcher, health=self._health)
        self.port = self.pool.port
        log.info("tutoring server on port %d (%d front-end processes)", self.port, self.pool.n)
        self._arm_fatal(on_fatal, poll_s)
        return self

    def stop(self):
        self._stopping.set()
        try:
            self.pool.stop()
        finally:
            self.batcher.stop()


EXIT_FATAL = 75  # EX_TEMPFAIL: the supervisor restarts the replica


def main(argv=None):
    ap = argparse.ArgumentParser(description="GPT-2 tutoring server (MI355X HIP engine)")
    ap.add_argument("--port", type=int, default=int(os.environ.get("DLMS_TUTOR_PORT", "50054")))
    ap.add_argument("--host", default="[::]")
    ap.add_argument("--model", default=os.environ.get("DLMS_MODEL", "gpt2"))
    ap.add_argument("--weights", default=None, help="local safetensors checkpoint (HF GPT-2 layout)")
    ap.add_argument("--vocab", default=None, help="GPT-2 vocab.json")
    ap.add_argument("--merges", default=None, help="GPT-2 merges.txt")
    ap.add_argument("--device", default=os.environ.get("DLMS_DEVICE", "auto"))
    ap.add_argument("--max-batch", type=int, default=0,
                    help="decode slots per engine; 0 (default) = as many as free HBM holds (engine/memory.py), "
                         "so one replica reaches the 1024-query operating point")
    ap.add_argument("--window-ms", type=float, default=2.0)
    ap.add_argument("--max-length", type=int, default=150)
    ap.add_argument("--repetition-penalty", type=float, default=1.2)
    ap.add_argument("--weight-dtype", choices=("bf16", "fp8"), default="bf16",
                    help="fp8: W8A8 e4m3 MFMA GEMMs for QKV / c_fc / LM head (GPU engine)")
    ap.add_argument("--tp", type=int, default=0, help="tensor-parallel degree under torchrun (default: world)")
    ap.add_argument("--batching", choices=("auto", "continuous", "window"), default="auto")
    ap.add_argument("--chunk", type=int, default=8, help="decode steps between scheduler polls")
    ap.add_argument("--max-queue", type=int, default=None,
                    help="queries that may wait for a KV slot before the replica answers RESOURCE_EXHAUSTED "
                         "(default: one batch of slots; 0 = unbounded)")
    ap.add_argument("--frontend", choices=("aio", "threads"), default="aio",
                    help="aio: asyncio gRPC front end (thousands of queries in flight); threads: a worker per query")
    ap.add_argument("--frontends", type=int, default=4,
                    help="gRPC front-end processes sharing the port (tutor/frontend.py); 0 = serve gRPC in "
                         "this process (--frontend)")
    ap.add_argument("--warm-batch", type=int, default=1024,
                    help="capture the decode graphs of every batch bucket up to this size before serving, so "
                         "the first burst of queries does not pay them (0 = capture on first use)")
    ap.add_argument("--serve-gate", action="store_true",
                    help="also serve the relevance gate (lmsinternal.Gate) on the tutoring port: the front ends "
                         "tokenize, this process runs the BERT encoder passes between decode chunks on the decode "
                         "stream (gate/service.py GateWorker) -- LMS nodes use it with --gate remote "
                         "--gate-addr <this address>")
    ap.add_argument("--gate-model", default="bert-base-uncased")
    ap.add_argument("--gate-vocab", default=None, help="BERT vocab.txt for the gate (synthetic if absent)")
    ap.add_argument("--gate-weights", default=None, help="local safetensors for the gate model")
    ap.add_argument("--log-level", default=os.environ.get("DLMS_LOG", "INFO"))
    args, _ = parse_with_config(ap, argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    tp_group = proxy = pool = None
    if args.frontends > 0 and args.batching != "window":
        # spawned before anything here touches the GPU; only the rank that serves a TP group
        # (every --tp-th rank under torchrun) gets front ends, on its group's port
        tp = args.tp or world
        rank = int(os.environ.get("RANK", "0"))
        if rank % tp == 0:
            from ..models.config import bert_config
            from .frontend import FrontendPool

            gate_fe = None
            if args.serve_gate:
                bc = bert_config(args.gate_model)
                gate_fe = dict(vocab=args.gate_vocab, vocab_size=bc.vocab_size, max_length=bc.max_position)
            pool = FrontendPool(args.frontends, args.port + rank // tp, args.host, args.vocab, args.merges,
                                eos=gpt2_config(args.model).eos_token_id, gate=gate_fe)
    if world > 1:  # torchrun: TP groups of --tp consecutive ranks, one front end (port + group) each
        import torch.distributed as dist

        from ..engine.tp_serving import TPEngineProxy, serve_follower
        from ..parallel.tp import init_distributed, tp_groups

        rank, world, local = init_distributed("nccl" if args.device != "cpu" and torch.cuda.is_available()
                                              else "gloo")
        tp = args.tp or world
        tp_group, dp_idx, _ = tp_groups(tp)
        ctrl = None
        for g in range(world // tp):  # every rank creates every group, keeps its own
            grp = dist.new_group(list(range(g * tp, (g + 1) * tp)), backend="gloo")
            if g == dp_idx:
                ctrl = grp
        src = dp_idx * tp
        device = f"cuda:{local}" if args.device != "cpu" and torch.cuda.is_available() else "cpu"
        eng = make_engine(args.model, device, args.max_batch, args.max_length, args.weights, tp_group=tp_group,
                          weight_dtype=args.weight_dtype)
        if rank != src:
            n = serve_follower(eng, ctrl, src)
            log.info("TP follower rank %d done after %d commands", rank, n)
            if hasattr(eng, "close"):
                eng.close()
            return
        proxy = eng = TPEngineProxy(eng, ctrl, src)
        args.port += dp_idx
    else:
        eng = make_engine(args.model, args.device, args.max_batch, args.max_length, args.weights,
                          weight_dtype=args.weight_dtype)
    args.max_batch = getattr(eng, "max_batch", 0) or args.max_batch or 64
    if args.warm_batch > 0 and hasattr(eng, "warm_decode_graphs"):
        # (a TP proxy mirrors the call to every rank of its group: the captures' warm-up steps run
        # the group's collectives, engine/tp_serving.py)
        n, secs = eng.warm_decode_graphs(args.repetition_penalty, args.warm_batch)
        log.info("captured %d decode graphs (batch buckets <= %d) in %.1f s", n, args.warm_batch, secs)
    tok = GPT2BPE(args.vocab, args.merges, eos_token_id=eng.cfg.eos_token_id)
    if pool is not None and hasattr(eng, "admit"):
        srv = PooledTutoringServer(eng, pool, args.max_length, args.repetition_penalty, chunk=args.chunk,
                                   max_queue=args.max_queue)
        if args.serve_gate:
            pool.gate_worker = make_gate_worker(args.gate_model, args.gate_weights, getattr(eng, "device", "cpu"))
            pool.gate_worker.attach(srv.batcher)
    else:
        if pool is not None:  # not a slot engine (CPU window batching): serve in-process
            pool.stop(timeout=2)
            pool = None
    if pool is not None:
        pass
    elif args.frontend == "aio" and args.batching != "window" and hasattr(eng, "admit"):
        srv = AioTutoringServer(eng, args.port, args.host, args.max_length, args.repetition_penalty, tokenizer=tok,
                                chunk=args.chunk, max_queue=args.max_queue)
    else:
        srv = TutoringServer(eng, args.port, args.host, args.max_batch, args.window_ms, args.max_length,
                             args.repetition_penalty, tokenizer=tok, batching=args.batching, chunk=args.chunk,
                             max_queue=args.max_queue)
    done = threading.Event()
    fatal: list = []

    def on_fatal(err):
        fatal.append(err)
        done.set()

    srv.start(on_fatal=on_fatal)
    print(f"Tutoring Server started on port {srv.port}", flush=True)
    signal.signal(signal.SIGTERM, lambda *a: done.set())
    signal.signal(signal.SIGINT, lambda *a: done.set())
    done.wait()
    srv.stop()
    if proxy is not None:
        proxy.close()  # releases the followers, which close their engines (below, same order)
        eng = proxy.engine
    if hasattr(eng, "close"):
        eng.close()  # (TP: every rank of the group, the xGMI teardown is collective)
    if fatal:  # exit, never re-exec: a supervisor starts a fresh process on a clean device state
        log.error("exiting with status %d after a fatal serving error", EXIT_FATAL)
        os._exit(EXIT_FATAL)


if __name__ == "__main__":
    main()
