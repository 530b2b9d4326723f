#!/usr/bin/env python3
"""Sustained open-loop serving benchmark through gRPC.

Drives ``Tutoring.GetLLMAnswer`` (the tutoring server CLI, one GPU) or ``LMS.GetLLMAnswer`` (a
3-node Raft LMS whose nodes run the BERT relevance gate and call that tutoring server) with
Poisson arrivals from ``--client-procs`` separate client processes, all started BEFORE any
process touches the GPU (spawned interpreters, grpc.aio).  Each offered rate runs ``--warmup``
seconds (discarded: hipGraph capture of new batch buckets, channel setup) followed by a
``--duration`` second measurement window.  Reported per rate, as one JSON line:

* ``tok_s``           -- generated tokens in the window, exact: the tutoring server's own
                         ``tutor_tokens`` counter (debug Metrics RPC) read at both window edges;
* ``completed_qps``   -- answers received in the window; ``offered_qps`` what was sent;
* ``p50_ms``/``p99_ms`` -- client-side latency of the queries SENT in the window (all of which
                         are waited for), ``inflight_mean``/``inflight_max`` summed over clients;
* ``server``          -- the server's queue / ttft / request-latency histograms.

``--closed N`` (one client process): N closed-loop clients instead of the Poisson stream, each
sending its next query the moment the previous answer arrives -- ``--closed 1`` is the reference's
own operating point, one student query at a time (``lms_server.py:1237-1274``); the line then also
reports the dataflow-kernel aborts the tutor counted in the window.

``--engine null`` replaces the GPT-2 engine by a host-only slot engine (fixed ``--null-step-ms``
per decode step): it measures the gRPC front end's own ceiling on any machine.

    python scripts/bench_grpc.py --target tutoring --rates 2000,4000 --duration 30
    python scripts/bench_grpc.py --target lms --rates 1000 --duration 30
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import random
import shutil
import signal
import statistics
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WORDS = ("raft leader election term vote log replication commit index follower candidate heartbeat "
         "snapshot quorum majority state machine consensus partition timeout append entries").split()


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


# ---------------------------------------------------------------------------- client processes
def _client_main(conn):
    """One client process: for each job ``(cfg)`` run an open-loop Poisson stream and reply with
    ``(records, inflight_samples)``; ``None`` ends the process."""
    import asyncio

    import grpc

    from distributed_lms_raft_llm_amd import wire
    from distributed_lms_raft_llm_amd.lms.service import MSG_TUTOR_BUSY as busy_msg
    from distributed_lms_raft_llm_amd.wire import pb

    async def run(cfg):
        rng = random.Random(cfg["seed"])
        # several connections per address (own subchannel pools): the server's front-end
        # processes share the port through SO_REUSEPORT, which balances connections
        opts = list(wire.CHANNEL_OPTIONS) + [("grpc.use_local_subchannel_pool", 1)]
        chans = [grpc.aio.insecure_channel(a, options=opts) for a in cfg["addrs"] for _ in range(cfg["channels"])]
        stubs = [wire.Stub(cfg["service"], c) for c in chans]
        recs, samples = [], []
        out = {"n": 0}
        t_begin, t_stop = cfg["t_begin"], cfg["t_stop"]

        async def one(k, t_send):
            tok, q = cfg["calls"][k % len(cfg["calls"])]
            out["n"] += 1
            try:
                r = await stubs[k % len(stubs)].GetLLMAnswer(pb.QueryRequest(token=tok, query=q),
                                                             timeout=cfg["timeout"])
                ok, n = bool(r.success), len(r.response)
                if r.response == busy_msg:  # the LMS's answer when every tutoring replica refused (load)
                    ok, n = False, "BUSY"
            except grpc.RpcError as e:
                ok, n = False, e.code().name
            out["n"] -= 1
            recs.append((t_send, (time.time() - t_send) * 1e3, ok, n))

        async def sampler():
            while time.time() < t_stop:
                samples.append((time.time(), out["n"]))
                await asyncio.sleep(0.25)

        while time.time() < t_begin:
            await asyncio.sleep(min(0.05, t_begin - time.time()))
        samp = asyncio.ensure_future(sampler())
        if cfg.get("closed"):
            async def loop(j):
                k = j
                while time.time() < t_stop:
                    await one(k, time.time())
                    k += cfg["closed"]

            await asyncio.gather(*(loop(j) for j in range(cfg["closed"])))
            await samp
            for c in chans:
                await c.close()
            return recs, samples
        tasks = set()
        t_next, k = t_begin, 0
        while True:
            t_next += rng.expovariate(cfg["rate"])
            if t_next >= t_stop:
                break
            dt = t_next - time.time()
            if dt > 0:
                await asyncio.sleep(dt)
            task = asyncio.ensure_future(one(k, time.time()))
            tasks.add(task)
            task.add_done_callback(tasks.discard)
            k += 1
        await samp
        if tasks:
            await asyncio.wait(list(tasks), timeout=cfg["timeout"] + 5)
        for c in chans:
            await c.close()
        return recs, samples

    while True:
        cfg = conn.recv()
        if cfg is None:
            return
        conn.send(asyncio.run(run(cfg)))


# ---------------------------------------------------------------------------- null engine
class NullSlotEngine:
    """Host-only slot engine (admit / decode / collect) with a fixed per-step time: the GPU's
    role played by ``time.sleep``, so a run measures the gRPC front end + scheduler alone."""

    def __init__(self, max_batch: int, max_length: int, step_ms: float):
        import numpy as np

        from types import SimpleNamespace

        self.np = np
        self.max_batch, self.max_length, self.step_s = max_batch, max_length, step_ms / 1e3
        self.cfg = SimpleNamespace(eos_token_id=50256)
        self.tok = np.zeros((max_batch, max_length), np.int32)
        self.len = np.zeros(max_batch, np.int32)
        self.fin = np.ones(max_batch, np.int32)

    def admit(self, prompts, slots, penalty):
        for p, s in zip(prompts, slots):
            self.tok[s, :len(p)] = p
            self.tok[s, len(p):] = 262
            self.len[s], self.fin[s] = len(p) + 1, 0

    def decode(self, B, steps, penalty):
        time.sleep(self.step_s * steps)
        live = self.fin[:B] == 0
        self.len[:B][live] = self.np.minimum(self.len[:B][live] + steps, self.max_length)
        self.fin[:B][self.len[:B] >= self.max_length] = 1

    def finished_flags(self, B):
        return self.fin[:B].tolist()

    def collect(self, slots):
        return [self.tok[s, :self.len[s]].tolist() for s in slots]


def serve_null(frontends: int, max_batch: int, max_length: int, step_ms: float, chunk: int):
    from distributed_lms_raft_llm_amd.tutor.server import AioTutoringServer, PooledTutoringServer

    eng = NullSlotEngine(max_batch, max_length, step_ms)
    if frontends > 0:
        from distributed_lms_raft_llm_amd.tutor.frontend import FrontendPool

        srv = PooledTutoringServer(eng, FrontendPool(frontends, 0, "127.0.0.1"), max_length=max_length,
                                   chunk=chunk).start()
    else:
        srv = AioTutoringServer(eng, port=0, host="127.0.0.1", max_length=max_length, chunk=chunk).start()
    print(f"Tutoring Server started on port {srv.port}", flush=True)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: done.set())
    done.wait()
    srv.stop()


# ---------------------------------------------------------------------------- orchestration
def _wait_line(proc, marker: str, timeout: float, log) -> str:
    end = time.time() + timeout
    while time.time() < end:
        line = proc.stdout.readline()
        if not line:
            if proc.poll() is not None:
                raise SystemExit(f"server exited with {proc.returncode} before '{marker}'")
            continue
        log.write(line)
        log.flush()
        if marker in line:
            return line
    raise SystemExit(f"timed out waiting for '{marker}'")


def _drain(proc, log):
    def pump():
        for line in proc.stdout:
            log.write(line)
        log.flush()

    threading.Thread(target=pump, daemon=True).start()


def start_tutor(args, log):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    if args.target == "lms" and args.gate in ("bert", "remote", "remote-proc"):
        # the LMS nodes' BERT gates share the tutor's GPU: its decode chunks on a high-priority stream
        # (LMS path at 3.5 k q/s p50 863 -> 606 ms; alone on the GPU the same setting cost the
        # Tutoring path 16 % at 5.5 k q/s, so it is a co-location setting, not a default)
        env.setdefault("DLMS_BATCHER_STREAM_PRIORITY", "-1")
    if args.engine == "null":
        cmd = [sys.executable, os.path.abspath(__file__), "--serve-null", "--max-length", str(args.max_length),
               "--null-slots", str(args.null_slots), "--null-step-ms", str(args.null_step_ms),
               "--chunk", str(args.chunk), "--frontends", str(args.frontends)]
    else:
        cmd = [sys.executable, "-m", "distributed_lms_raft_llm_amd.tutor.server", "--port", "0", "--host",
               "127.0.0.1", "--max-length", str(args.max_length), "--chunk", str(args.chunk),
               "--model", args.model, "--max-batch", str(args.max_batch), "--frontend", "aio",
               "--frontends", str(args.frontends)]
        if args.target == "lms" and args.gate == "remote":  # the gate served by the tutor (--serve-gate)
            cmd += ["--serve-gate"]
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    line = _wait_line(p, "Tutoring Server started on port", args.startup_timeout, log)
    _drain(p, log)
    addr = f"127.0.0.1:{int(line.rsplit(' ', 1)[1])}"
    if args.target == "lms" and args.gate == "remote":
        args.gate_addr = addr
    return p, addr


def start_gate_proc(args, log):
    """--gate remote-proc: one gate server process on the GPU (python -m distributed_lms_raft_llm_amd.gate)."""
    cmd = [sys.executable, "-m", "distributed_lms_raft_llm_amd.gate", "--port", "0", "--host", "127.0.0.1"]
    p = subprocess.Popen(cmd, cwd=ROOT, env=dict(os.environ, PYTHONUNBUFFERED="1"), stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True)
    line = _wait_line(p, "Gate Server started on port", args.startup_timeout, log)
    _drain(p, log)
    args.gate_addr = f"127.0.0.1:{int(line.rsplit(' ', 1)[1])}"
    return p


def _free_ports(n):
    import socket

    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def start_lms(args, tutor_addr, log, tmp):
    ports = _free_ports(3)
    addrs = [f"127.0.0.1:{p}" for p in ports]
    procs = []
    for i in range(1, 4):
        peers = [a for j, a in enumerate(addrs, 1) if j != i]
        remote = args.gate in ("remote", "remote-proc")
        cmd = [sys.executable, "-m", "distributed_lms_raft_llm_amd.lms.server", str(i), str(ports[i - 1]), *peers,
               "--host", "127.0.0.1", "--advertise", addrs[i - 1], "--data-dir", os.path.join(tmp, f"node{i}"),
               "--tutor", tutor_addr, "--gate", "remote" if remote else args.gate,
               "--gate-threshold", str(args.gate_threshold),
               "--workers", str(args.lms_workers), "--frontend", "aio", "--log-level", "WARNING"]
        env = dict(os.environ, PYTHONUNBUFFERED="1")
        if remote:  # GPU-less LMS nodes: the relevance gate is the GPU tier's service
            cmd += ["--gate-addr", args.gate_addr, "--gate-fallback", "off"]
            env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        _drain(p, log)
        procs.append(p)
    return procs, addrs


def lms_setup(addrs, n_students, timeout):
    """Wait for a leader, register + log in ``n_students`` students, post each an assignment."""
    from distributed_lms_raft_llm_amd import wire
    from distributed_lms_raft_llm_amd.lms.pdf import make_pdf
    from distributed_lms_raft_llm_amd.utils.debug_rpc import debug_call
    from distributed_lms_raft_llm_amd.wire import pb

    end = time.time() + timeout
    leader = None
    while time.time() < end and leader is None:
        for a in addrs:
            try:
                h = debug_call(a, "Health", timeout=2)
                if h.get("role") == "leader":
                    leader = a
            except Exception:
                pass
        time.sleep(0.2)
    if leader is None:
        raise SystemExit("no LMS leader elected")
    st = wire.Stub("LMS", wire.channel(leader))
    rng = random.Random(0)
    tokens = []
    for k in range(n_students):
        u = f"student{k}"
        st.Register(pb.RegisterRequest(username=u, password="pw", role="student"), timeout=30)
        tok = st.Login(pb.LoginRequest(username=u, password="pw"), timeout=30).token
        text = " ".join(rng.choice(WORDS) for _ in range(300))
        assert st.Post(pb.PostRequest(token=tok, type="assignment", file=make_pdf(text), filename=f"hw{k}.pdf"),
                       timeout=60).success
        tokens.append(tok)
    time.sleep(1.0)  # sessions / assignments applied on the followers too
    return tokens


def metrics(addr):
    import grpc

    from distributed_lms_raft_llm_amd.utils.debug_rpc import debug_call

    for attempt in range(5):
        try:
            return debug_call(addr, "Metrics", timeout=10)
        except grpc.RpcError:
            if attempt == 4:
                raise
            time.sleep(0.05)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", choices=("tutoring", "lms"), default="tutoring")
    ap.add_argument("--rates", default="3000", help="offered queries/s (comma-separated: one window each)")
    ap.add_argument("--duration", type=float, default=30.0)
    ap.add_argument("--warmup", type=float, default=8.0)
    ap.add_argument("--client-procs", type=int, default=4)
    ap.add_argument("--channels", type=int, default=4, help="connections per client process and address")
    ap.add_argument("--frontends", type=int, default=4, help="tutoring front-end processes (0: in-process aio)")
    ap.add_argument("--engine", choices=("hip", "null"), default="hip")
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--max-batch", type=int, default=0, help="tutor slots (0: HBM planner)")
    ap.add_argument("--max-length", type=int, default=150)
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--null-slots", type=int, default=4096)
    ap.add_argument("--null-step-ms", type=float, default=1.6)
    ap.add_argument("--gate", choices=("bert", "remote", "remote-proc", "off"), default="bert",
                    help="bert: a gate per LMS node on the GPU; remote: ONE gate served by the tutor (passes "
                         "between decode chunks), LMS nodes GPU-less; remote-proc: a gate server process")
    ap.add_argument("--gate-threshold", type=float, default=0.0, help="0: random-init BERT admits every query")
    ap.add_argument("--lms-workers", type=int, default=32)
    ap.add_argument("--students", type=int, default=64)
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--startup-timeout", type=float, default=600.0)
    ap.add_argument("--closed", type=int, default=0,
                    help="N closed-loop clients (one query at a time each) instead of open-loop --rates")
    ap.add_argument("--out", default=None, help="append JSON lines here")
    ap.add_argument("--log", default=None, help="server stdout/stderr")
    ap.add_argument("--tag", default="")
    ap.add_argument("--serve-null", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.closed:
        args.client_procs, args.rates = 1, "0"
    if args.serve_null:
        return serve_null(args.frontends, args.null_slots, args.max_length, args.null_step_ms, args.chunk)

    # 1. clients first: fresh interpreters, before any process here touches the GPU
    ctx = mp.get_context("spawn")
    clients = []
    for _ in range(args.client_procs):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_client_main, args=(b,), daemon=True)
        p.start()
        clients.append((p, a))

    log = open(args.log, "a") if args.log else open(os.devnull, "w")
    tmp = tempfile.mkdtemp(prefix="bench_grpc_")
    procs = []
    try:
        t_boot = time.time()
        tutor, tutor_addr = start_tutor(args, log)
        procs.append(tutor)
        if args.target == "lms" and args.gate == "remote-proc":
            procs.append(start_gate_proc(args, log))
        if args.target == "lms":
            lms_procs, addrs = start_lms(args, tutor_addr, log, tmp)
            procs += lms_procs
            tokens = lms_setup(addrs, args.students, args.startup_timeout)
            service = "LMS"
        else:
            addrs, tokens, service = [tutor_addr], [f"t{k}" for k in range(args.students)], "Tutoring"
        boot_s = time.time() - t_boot
        rng = random.Random(1)
        calls = [(tokens[k % len(tokens)], "explain " + " ".join(rng.choice(WORDS) for _ in range(rng.randint(6, 14))))
                 for k in range(512)]
        for rate in [float(r) for r in args.rates.split(",") if r.strip()]:
            t_begin = time.time() + 2.0
            t_meas = t_begin + args.warmup
            t_stop = t_meas + args.duration
            for i, (_, conn) in enumerate(clients):
                conn.send({"addrs": addrs, "service": service, "rate": rate / len(clients), "t_begin": t_begin,
                           "t_stop": t_stop, "calls": calls[i::len(clients)], "seed": 7919 * i + int(rate),
                           "timeout": args.timeout, "channels": args.channels, "closed": args.closed})
            time.sleep(max(0.0, t_meas - time.time()))
            m0, w0 = metrics(tutor_addr), time.time()
            time.sleep(max(0.0, t_stop - time.time()))
            m1, w1 = metrics(tutor_addr), time.time()
            # the LMS nodes' own view (gate batching, the whole GetLLMAnswer, tutor failovers): where
            # the LMS path's latency goes beyond the tutoring tier's
            lms_m = {a: metrics(a) for a in addrs} if args.target == "lms" else {}
            results = [conn.recv() for _, conn in clients]
            recs = [r for rr, _ in results for r in rr]
            win = [r for r in recs if t_meas <= r[0] < t_stop]
            if os.environ.get("BENCH_GRPC_DUMP"):
                with open(os.environ["BENCH_GRPC_DUMP"], "w") as f:
                    json.dump({"t_begin": t_begin, "t_meas": t_meas, "t_stop": t_stop, "recs": recs}, f)
            ok = [r for r in win if r[2]]
            done_in_win = [r for r in recs if r[2] and t_meas <= r[0] + r[1] / 1e3 < t_stop]
            lat = [r[1] for r in ok]
            # in-flight: sum over clients per 0.25 s sample, inside the window
            buckets: dict[int, int] = {}
            for _, samples in results:
                for t, n in samples:
                    if t_meas <= t < t_stop:
                        buckets[int((t - t_meas) * 4)] = buckets.get(int((t - t_meas) * 4), 0) + n
            infl = list(buckets.values())
            c0, c1 = m0["counters"], m1["counters"]
            tokens_win = c1.get("tutor_tokens", 0.0) - c0.get("tutor_tokens", 0.0)
            hist = m1.get("histograms", {})
            line = {
                "bench": "serving_grpc", "target": f"{service}.GetLLMAnswer", "engine": args.engine,
                "model": args.model, "tag": args.tag,
                "offered_qps": rate if not args.closed else None, "closed_clients": args.closed or None,
                "duration_s": args.duration, "warmup_s": args.warmup,
                "client_procs": args.client_procs, "nodes": 3 if args.target == "lms" else 0,
                "gate": args.gate if args.target == "lms" else None,
                "tok_s": round(tokens_win / (w1 - w0), 1),
                "completed_qps": round(len(done_in_win) / args.duration, 1),
                "sent_in_window": len(win), "ok": len(ok), "failed": len(win) - len(ok),
                "fail_codes": {c: sum(1 for r in win if not r[2] and r[3] == c)
                               for c in sorted({r[3] for r in win if not r[2]})},
                # how fast each failure kind came back (admission control: RESOURCE_EXHAUSTED / BUSY
                # should return in milliseconds, a deadline in --timeout seconds)
                "fail_p50_ms": {c: round(pct([r[1] for r in win if not r[2] and r[3] == c], 0.5), 1)
                                for c in sorted({r[3] for r in win if not r[2]})},
                "p50_ms": round(pct(lat, 0.5), 1) if lat else None, "p99_ms": round(pct(lat, 0.99), 1) if lat else None,
                "mean_ms": round(statistics.mean(lat), 1) if lat else None,
                "inflight_mean": round(statistics.mean(infl), 1) if infl else 0,
                "inflight_max": max(infl) if infl else 0,
                "tokens_per_query": round(tokens_win / max(1, len(done_in_win)), 1),
                "server": {k: {q: round(v, 2) for q, v in hist[k].items() if q in ("count", "p50", "p99")}
                           for k in ("tutor_queue_ms", "tutor_ttft_ms", "tutor_request_ms", "tutor_tpot_ms")
                           if k in hist},
                "boot_s": round(boot_s, 1),
                "dataflow_aborts": c1.get("engine_dataflow_aborts", 0.0) - c0.get("engine_dataflow_aborts", 0.0),
                "dataflow_aborts_total": c1.get("engine_dataflow_aborts", 0.0),
            }
            if args.target == "lms" and args.gate in ("remote", "remote-proc"):
                from distributed_lms_raft_llm_amd.utils.debug_rpc import debug_call

                g = debug_call(args.gate_addr, "Health", timeout=10)
                line["gate_service"] = {k: g.get(k) for k in ("scored", "missing", "passes", "batched_queries",
                                                               "device")}
            if lms_m:
                line["lms_nodes"] = {
                    a: {k: {q: round(v, 2) for q, v in m.get("histograms", {})[k].items() if q in ("count", "p50", "p99")}
                        for k in ("gate_ms", "gate_batch", "llm_answer_ms") if k in m.get("histograms", {})}
                    for a, m in lms_m.items()}
            print(json.dumps(line), flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(line) + "\n")
    finally:
        for _, conn in clients:
            try:
                conn.send(None)
            except Exception:
                pass
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for p, _ in clients:
            p.join(5)
        shutil.rmtree(tmp, ignore_errors=True)
        log.close()


if __name__ == "__main__":
    main()
