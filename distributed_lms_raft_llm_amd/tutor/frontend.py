"""Multi-process gRPC front end for one tutoring engine.

One Python process cannot both terminate thousands of gRPC calls per second and keep the GPU
fed: measured on the null engine (``scripts/bench_grpc.py --engine null``), a single ``grpc.aio``
process tops out near 1.7k queries/s (~200k tok/s) and past that gRPC core cancels the calls
the application has not picked up.  So the serving process is split the way the hardware is:

* the ENGINE process owns the GPU (HipGPT2Engine + ContinuousBatcher) and nothing else;
* ``n`` FRONT-END processes (spawned before the engine touches the GPU) share the public port
  (``SO_REUSEPORT``: the kernel spreads client connections over them), run grpc.aio, tokenize the
  prompt and detokenize the answer, and exchange token ids with the engine over one Unix socket
  each -- batched: every message carries all requests (or results) that accumulated since the
  last one, so the engine process pays microseconds per query.

Wire (pickled tuples on ``multiprocessing.connection``, this machine only, authkey'd):
  front end -> engine   ("q", [(rid, ids), ...])   ("metrics", cid)   ("health", cid)
  engine -> front end   ("ready", port)  ("r", [(rid, ids | None, code, msg), ...])
                        ("metrics", cid, snapshot)  ("health", cid, dict)  ("stop",)
The debug ``Metrics`` / ``Health`` RPCs on any front end answer with the ENGINE's registry (the
tokens counter the benchmarks read) plus the front end's own under ``"frontend"``.

Failure semantics match the single-process server: a failed batcher turns every pending and
later query into UNAVAILABLE (the LMS's TutoringClient fails over), the engine process exits
non-zero for its supervisor, and each front end exits when its engine connection closes.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import logging
import multiprocessing as mp
import os
import secrets
import tempfile
import threading
import time
from concurrent import futures
from multiprocessing.connection import Client, Listener

import grpc

from .. import wire
from ..utils.metrics import METRICS
from ..wire import pb

log = logging.getLogger("dlms.tutor.frontend")

DEBUG_SERVICE = "lmsinternal.Debug"


# ----------------------------------------------------------------------------- front-end process
def _frontend_main(path: str, authkey: bytes, idx: int, host: str, vocab, merges, eos: int, timeout: float,
                   log_level: int, gate: dict | None = None):
    logging.basicConfig(level=log_level, format=f"%(asctime)s fe{idx} %(name)s %(levelname)s %(message)s")
    from ..tokenizer import GPT2BPE
    from .server import build_prompt

    tok = GPT2BPE(vocab, merges, eos_token_id=eos)
    btok = None
    if gate is not None:  # the relevance gate served here too: BERT WordPiece on this side of the relay
        from ..tokenizer import BertWordPiece

        btok = BertWordPiece(gate.get("vocab"), vocab_size=gate["vocab_size"], max_length=gate["max_length"])
    conn = Client(path, family="AF_UNIX", authkey=authkey)
    msg = conn.recv()
    if msg[0] != "ready":
        return
    port = msg[1]
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    pending: dict[int, asyncio.Future] = {}
    gpending: dict[int, asyncio.Future] = {}  # relevance-gate requests (rid -> future of per-item results)
    calls: dict[int, threading.Event] = {}
    replies: dict[int, object] = {}
    outbox: list = []
    state = {"dead": None, "flush": False}
    rids = itertools.count(1)
    send_lock = threading.Lock()

    def send(m):
        with send_lock:
            conn.send(m)

    def flush():
        state["flush"] = False
        if outbox and state["dead"] is None:
            batch = outbox[:]
            outbox.clear()
            try:
                send(("q", batch))
            except OSError as e:
                die(f"engine connection lost: {e}")

    def die(why: str, clean: bool = False):
        if state["dead"] is None:
            state["dead"] = why
            (log.info if clean else log.error)("front end %d: %s", idx, why)
        for f in pending.values():
            if not f.done():
                f.set_result((None, "UNAVAILABLE", why))
        pending.clear()
        for f in gpending.values():
            if not f.done():
                f.set_result(None)
        gpending.clear()

    def deliver(items):
        for rid, ids, code, msg_ in items:
            f = pending.pop(rid, None)
            if f is not None and not f.done():
                f.set_result((ids, code, msg_))

    def gdeliver(items):
        for rid, res in items:
            f = gpending.pop(rid, None)
            if f is not None and not f.done():
                f.set_result(res)

    def reader():  # engine -> front end (own thread: recv blocks)
        while True:
            try:
                m = conn.recv()
            except (EOFError, OSError):
                loop.call_soon_threadsafe(die, "engine process gone")
                loop.call_soon_threadsafe(stop_ev.set)
                return
            kind = m[0]
            if kind == "r":
                loop.call_soon_threadsafe(deliver, m[1])
            elif kind == "gr":
                loop.call_soon_threadsafe(gdeliver, m[1])
            elif kind in ("metrics", "health"):
                replies[m[1]] = m[2]
                ev = calls.pop(m[1], None)
                if ev is not None:
                    ev.set()
            elif kind == "stop":
                loop.call_soon_threadsafe(stop_ev.set)
                return

    class Servicer:
        async def GetLLMAnswer(self, request, context):
            t0 = time.perf_counter()
            if state["dead"] is not None:
                await context.abort(grpc.StatusCode.UNAVAILABLE, state["dead"])
            ids = tok.encode(build_prompt(request.query))
            rid = next(rids)
            fut = loop.create_future()
            pending[rid] = fut
            outbox.append((rid, ids))
            if not state["flush"]:  # one message per loop iteration, whatever arrived in it
                state["flush"] = True
                loop.call_soon(flush)
            try:
                out, code, why = await asyncio.wait_for(fut, timeout)
            except asyncio.TimeoutError:
                pending.pop(rid, None)
                await context.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation timed out")
            if out is None:
                await context.abort(getattr(grpc.StatusCode, code, grpc.StatusCode.INTERNAL),
                                    f"generation failed: {why}")
            METRICS.observe("frontend_request_ms", (time.perf_counter() - t0) * 1e3)
            return pb.QueryResponse(success=True, response=tok.decode(out, skip_special_tokens=True))

    async def gate_call(items):
        """items [(query_ids | None, key, assignment_ids | None)] -> per-item results from the
        engine's GateWorker (None: the engine is gone)."""
        if state["dead"] is not None:
            return None
        rid = next(rids)
        fut = loop.create_future()
        gpending[rid] = fut
        try:
            send(("g", [(rid, items)]))
        except OSError as e:
            die(f"engine connection lost: {e}")
        try:
            return await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            gpending.pop(rid, None)
            return None

    def gate_handler(kind):
        async def h(body: bytes, context) -> bytes:
            req = json.loads(body) if body else {}
            if kind == "ScoreBatch":
                items = [(btok.encode(it["query"]), it["key"],
                          btok.encode(it["text"]) if it.get("text") is not None else None) for it in req["items"]]
            elif kind == "Score":
                items = [(btok.encode(req["query"]), req["key"],
                          btok.encode(req["text"]) if req.get("text") is not None else None)]
            else:  # Embed
                from ..gate.relevance import RelevanceGate

                items = [(None, RelevanceGate._key(req["text"]), btok.encode(req["text"]))]
            res = await gate_call(items)
            if res is None:
                await context.abort(grpc.StatusCode.UNAVAILABLE, state["dead"] or "gate timed out")
            if kind == "ScoreBatch":
                out = {"sims": [r if isinstance(r, float) else None for r in res],
                       "missing": [i for i, r in enumerate(res) if r == "missing"]}
            elif kind == "Score":
                out = {"missing": True} if res[0] == "missing" else {"similarity": res[0]}
            else:
                out = {"key": items[0][1]}
            return json.dumps(out).encode()

        return grpc.unary_unary_rpc_method_handler(h)

    def ask_engine(kind: str, wait_s: float = 10.0):
        cid = next(rids)
        ev = threading.Event()
        calls[cid] = ev
        send((kind, cid))
        if not ev.wait(wait_s):
            calls.pop(cid, None)
            raise RuntimeError(f"engine did not answer {kind}")
        return replies.pop(cid)

    def debug(kind):
        def h(body: bytes, context) -> bytes:
            out = dict(ask_engine(kind))
            if kind == "metrics":
                out["frontend"] = METRICS.snapshot()
            else:
                out["frontend"] = {"index": idx, "in_flight": len(pending), "ok": state["dead"] is None}
                out["ok"] = bool(out.get("ok", True)) and state["dead"] is None
            return json.dumps(out, default=str).encode()

        return grpc.unary_unary_rpc_method_handler(h)

    stop_ev = asyncio.Event()

    async def serve():
        opts = list(wire.CHANNEL_OPTIONS) + [("grpc.so_reuseport", 1)]
        srv = grpc.aio.server(migration_thread_pool=futures.ThreadPoolExecutor(max_workers=4), options=opts)
        wire.register(srv, "Tutoring", Servicer())
        srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(
            DEBUG_SERVICE, {"Health": debug("health"), "Metrics": debug("metrics")}),))
        if btok is not None:
            from ..gate.service import SERVICE as GATE_SERVICE

            srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(
                GATE_SERVICE, {k: gate_handler(k) for k in ("Score", "ScoreBatch", "Embed")}),))
        bound = srv.add_insecure_port(f"{host}:{port}")
        await srv.start()
        send(("bound", bound))
        await stop_ev.wait()
        die("front end stopping", clean=True)
        await srv.stop(0.5)

    threading.Thread(target=reader, name=f"fe{idx}-reader", daemon=True).start()
    try:
        loop.run_until_complete(serve())
    finally:
        try:
            conn.close()
        except OSError:
            pass


# ----------------------------------------------------------------------------- engine side
class FrontendPool:
    """``n`` front-end processes for one engine.  Create it (``spawn``) BEFORE the engine touches
    the GPU, then ``serve(batcher, health)`` once the engine is up."""

    def __init__(self, n: int, port: int, host: str = "[::]", vocab=None, merges=None, eos: int = 50256,
                 timeout: float = 300.0, gate: dict | None = None):
        """``gate``: also serve the relevance gate (``lmsinternal.Gate``) on this port -- tokenized in
        the front ends, scored by ``gate_worker`` (set before ``serve``) between decode chunks;
        a dict with the BERT tokenizer's ``vocab`` (path or None), ``vocab_size``, ``max_length``."""
        if n < 1:
            raise ValueError("need at least one front end")
        self.n, self.req_port, self.host = n, port, host
        self._dir = tempfile.mkdtemp(prefix="dlms_fe_")
        self.path = os.path.join(self._dir, "engine.sock")
        self.authkey = secrets.token_bytes(16)
        self.listener = Listener(self.path, family="AF_UNIX", authkey=self.authkey)
        ctx = mp.get_context("spawn")
        self.procs = [ctx.Process(target=_frontend_main, name=f"tutor-fe{i}", daemon=True,
                                  args=(self.path, self.authkey, i, host, vocab, merges, eos, timeout,
                                        logging.getLogger().level, gate))
                      for i in range(n)]
        for p in self.procs:
            p.start()
        self.conns: list = []
        self.port = 0
        self._out: list[list] = []
        self._cv = threading.Condition()
        self._stopping = False
        self.batcher = None
        self.gate_worker = None
        self._gout: list[list] = []

    def serve(self, batcher, health=None, accept_timeout: float = 120.0):
        """Accept the front ends, hand them the port (the first binds it -- an ephemeral one if
        ``port`` is 0 -- the rest join it through SO_REUSEPORT) and start relaying."""
        self.batcher, self._health = batcher, health
        self.listener._listener._socket.settimeout(accept_timeout)
        port = self.req_port
        for i in range(self.n):
            c = self.listener.accept()
            c.send(("ready", port))
            kind, bound = c.recv()
            if kind != "bound" or not bound:
                raise RuntimeError(f"front end {i} could not bind {self.host}:{port}")
            port = bound
            self.conns.append(c)
        self.port = port
        self._out = [[] for _ in self.conns]
        self._gout = [[] for _ in self.conns]
        for i, c in enumerate(self.conns):
            threading.Thread(target=self._reader, args=(i, c), name=f"fe{i}-relay", daemon=True).start()
        threading.Thread(target=self._sender, name="fe-sender", daemon=True).start()
        return self

    def _result(self, i: int, rid: int, fut):
        try:
            item = (rid, fut.result(), "OK", "")
        except BaseException as e:  # batcher failure: UNAVAILABLE so clients fail over
            from ..engine.scheduler import Overloaded

            code = "UNAVAILABLE" if getattr(self.batcher, "failed", None) is not None else "INTERNAL"
            if isinstance(e, Overloaded):
                code = "RESOURCE_EXHAUSTED"
            item = (rid, None, code, str(e))
        with self._cv:
            self._out[i].append(item)
            self._cv.notify()

    def _gresult(self, i: int, rid: int, res):
        with self._cv:
            self._gout[i].append((rid, res))
            self._cv.notify()

    def _reader(self, i: int, c):
        while True:
            try:
                m = c.recv()
            except (EOFError, OSError):
                return
            kind = m[0]
            if kind == "q":
                for rid, ids in m[1]:
                    try:
                        f = self.batcher.submit(ids)
                    except BaseException as e:
                        f = futures.Future()
                        f.set_exception(e)
                    f.add_done_callback(lambda fut, rid=rid: self._result(i, rid, fut))
            elif kind == "g":
                for rid, items in m[1]:
                    if self.gate_worker is None:
                        self._gresult(i, rid, None)
                    else:
                        self.gate_worker.submit(items, lambda res, rid=rid: self._gresult(i, rid, res))
            elif kind == "metrics":
                self._send(i, ("metrics", m[1], METRICS.snapshot()))
            elif kind == "health":
                try:
                    h = {"ok": True, **(self._health() if self._health else {})}
                except Exception as e:  # noqa: BLE001 -- report, don't kill the relay
                    h = {"ok": False, "error": str(e)}
                self._send(i, ("health", m[1], h))

    def _send(self, i: int, m):
        with self._cv:  # serialises with the sender thread's writes to the same connection
            try:
                self.conns[i].send(m)
            except OSError:
                pass

    def _sender(self):
        while True:
            with self._cv:
                while not self._stopping and not any(self._out) and not any(self._gout):
                    self._cv.wait()
                if self._stopping:
                    return
                batches = [(i, o) for i, o in enumerate(self._out) if o]
                gbatches = [(i, o) for i, o in enumerate(self._gout) if o]
                self._out = [[] for _ in self.conns]
                self._gout = [[] for _ in self.conns]
                for kind, bb in (("r", batches), ("gr", gbatches)):
                    for i, items in bb:
                        try:
                            self.conns[i].send((kind, items))
                        except OSError:
                            pass

    def stop(self, timeout: float = 10.0):
        with self._cv:
            self._stopping = True
            self._cv.notify_all()
            for c in self.conns:
                try:
                    c.send(("stop",))
                except OSError:
                    pass
        deadline = time.time() + timeout
        for p in self.procs:
            p.join(max(0.1, deadline - time.time()))
            if p.is_alive():
                p.terminate()
                p.join(2)
        for c in self.conns:
            c.close()
        self.listener.close()
        try:
            os.unlink(self.path)
            os.rmdir(self._dir)
        except OSError:
            pass
