#!/usr/bin/env python3
"""End-to-end deployment runs of BASELINE.json's five configs, as real processes.

    python scripts/run_config.py --config 2 [--students 64 --queries 4 ...]

Each run launches the tutoring tier (``tutoring_server.py``; under torchrun for TP > 1), an LMS
Raft cluster of N ``lms_server.py --config`` processes (BERT relevance gate in-process on the
leader's GPU when one exists), then drives the reference GUI's student workflow through the
client library for every synthetic student -- register, login, post an assignment (a generated
PDF for config 5), ask the LLM tutor -- with all students in flight at once.  Config 4 kills the
Raft leader in the middle of the query load and checks that every query still succeeds.

Prints one JSON line: end-to-end GetLLMAnswer latency percentiles, delivered generated-token
rate, gate rejections, Raft failover time.  Synthetic data and random-init weights throughout
(no network).  The configs ("tp" / "model" / "nodes" can be overridden for smaller boxes):

  1  gpt2         CPU tutor (torch reference engine), 1 LMS node, gate off     (plumbing)
  2  gpt2         1 GPU, 3-node Raft + BERT gate
  3  gpt2-medium  1 GPU, continuous batching of concurrent queries, 5-node Raft
  4  gpt2-large   TP=4 over xGMI, hipGraph decode, 5-node Raft, leader killed under load
  5  gpt2-xl      TP=8, fp8 (W8A8) GEMMs, 5-node Raft, full PDF -> gate -> LLM workflow
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    1: dict(model="gpt2", device="cpu", nodes=1, gate="off", tp=1, pdf=False, kill_leader=False),
    2: dict(model="gpt2", device="cuda", nodes=3, gate="bert", tp=1, pdf=False, kill_leader=False),
    3: dict(model="gpt2-medium", device="cuda", nodes=5, gate="bert", tp=1, pdf=False, kill_leader=False),
    4: dict(model="gpt2-large", device="cuda", nodes=5, gate="bert", tp=4, pdf=False, kill_leader=True),
    5: dict(model="gpt2-xl", device="cuda", nodes=5, gate="bert", tp=8, pdf=True, kill_leader=False,
            weight_dtype="fp8"),
}

TOPICS = ["raft consensus and leader election", "gradient descent for linear regression",
          "binary search trees and rotations", "virtual memory and page tables", "tcp congestion control"]


def free_ports(n: int) -> list[int]:
    socks = []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


class Proc:
    def __init__(self, cmd, log_path, env=None):
        self.log = open(log_path, "w")
        self.p = subprocess.Popen(cmd, stdout=self.log, stderr=subprocess.STDOUT, env=env, cwd=ROOT,
                                  start_new_session=True)

    def alive(self) -> bool:
        return self.p.poll() is None

    def kill(self, sig=signal.SIGKILL, wait: float = 30.0):
        if self.alive():
            try:
                os.killpg(self.p.pid, sig)
            except ProcessLookupError:
                pass
        try:
            self.p.wait(timeout=wait)
        except subprocess.TimeoutExpired:
            os.killpg(self.p.pid, signal.SIGKILL)
            self.p.wait()


def progress(msg: str):
    print(f"[run_config {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def wait_for(pred, timeout: float, what: str, procs=()):
    end = time.time() + timeout
    t0 = last = time.time()
    while time.time() < end:
        if pred():
            progress(f"{what}: ready after {time.time() - t0:.1f} s")
            return
        if time.time() - last > 30:
            progress(f"waiting for {what} ({time.time() - t0:.0f} s)")
            last = time.time()
        for p in procs:
            if not p.alive():
                raise RuntimeError(f"a process died while waiting for {what}: see {p.log.name}")
        time.sleep(0.2)
    raise TimeoutError(what)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=2)
    ap.add_argument("--model")
    ap.add_argument("--tp", type=int)
    ap.add_argument("--nodes", type=int)
    ap.add_argument("--device")
    ap.add_argument("--gate", choices=["bert", "off"])
    ap.add_argument("--weight-dtype", choices=["bf16", "fp8"], help="tutor GEMM weights (config 5: fp8)")
    ap.add_argument("--gate-model", default="bert-base-uncased")
    ap.add_argument("--gate-threshold", type=float, default=0.6)
    ap.add_argument("--students", type=int, default=32)
    ap.add_argument("--queries", type=int, default=2, help="LLM queries per student")
    ap.add_argument("--max-length", type=int, default=150)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--startup-timeout", type=float, default=600)
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    cfg.setdefault("weight_dtype", "bf16")
    for k in ("model", "tp", "nodes", "device", "gate", "weight_dtype"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)

    import yaml

    from distributed_lms_raft_llm_amd.client import LMSClient
    from distributed_lms_raft_llm_amd.lms.pdf import make_pdf
    from distributed_lms_raft_llm_amd.utils.debug_rpc import debug_call

    work = args.workdir or tempfile.mkdtemp(prefix=f"dlms_cfg{args.config}_")
    os.makedirs(work, exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT)
    ports = free_ports(cfg["nodes"] + 2)
    tutor_port, master_port, lms_ports = ports[0], ports[1], ports[2:]
    procs: list[Proc] = []
    result = {"config": args.config, **cfg, "students": args.students, "queries_per_student": args.queries}
    try:
        # ---------------------------------------------------------------- tutoring tier
        tut = [os.path.join(ROOT, "tutoring_server.py"), "--model", cfg["model"], "--device", cfg["device"],
               "--port", str(tutor_port), "--host", "127.0.0.1", "--max-length", str(args.max_length),
               "--max-batch", str(args.max_batch), "--log-level", "WARNING"]
        if cfg["device"] != "cpu":
            tut += ["--weight-dtype", cfg["weight_dtype"]]
        if cfg["tp"] > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={cfg['tp']}",
                   "--master-addr=127.0.0.1", f"--master-port={master_port}"] + tut + ["--tp", str(cfg["tp"])]
        else:
            cmd = [sys.executable] + tut
        tenv = dict(env)
        if cfg["gate"] == "bert" and cfg["device"] != "cpu":
            # the LMS nodes' gates share the GPU: decode chunks on a high-priority stream (scripts/bench_grpc.py)
            tenv.setdefault("DLMS_BATCHER_STREAM_PRIORITY", "-1")
        tutor = Proc(cmd, os.path.join(work, "tutor.log"), tenv)
        procs.append(tutor)
        progress(f"config {args.config}: {cfg} -> {work}")

        # ---------------------------------------------------------------- LMS Raft cluster
        servers = {i + 1: f"127.0.0.1:{p}" for i, p in enumerate(lms_ports)}
        nodes: dict[int, Proc] = {}
        for i in servers:
            conf = {"servers": servers, "host": "127.0.0.1", "tutor": f"127.0.0.1:{tutor_port}",
                    "gate": cfg["gate"], "gate_model": args.gate_model, "gate_threshold": args.gate_threshold,
                    "gate_device": "auto" if cfg["device"] != "cpu" else "cpu",
                    "data_dir": os.path.join(work, f"node{i}"), "no_fsync": True, "log_level": "WARNING"}
            path = os.path.join(work, f"node{i}.yaml")
            with open(path, "w") as f:
                yaml.safe_dump(conf, f)
            nodes[i] = Proc([sys.executable, os.path.join(ROOT, "lms_server.py"), "--config", path, str(i)],
                            os.path.join(work, f"node{i}.log"), env)
            procs.append(nodes[i])

        t0 = time.time()
        wait_for(lambda: "Tutoring Server started" in open(os.path.join(work, "tutor.log")).read(),
                 args.startup_timeout, "tutoring server", [tutor])

        def leader():
            for i, a in servers.items():
                if not nodes[i].alive():
                    continue
                try:
                    h = debug_call(a, "Health", timeout=1)
                    if h.get("role") == "leader":
                        return i
                except Exception:
                    pass
            return None

        wait_for(lambda: leader() is not None, args.startup_timeout, "Raft leader", list(nodes.values()))
        result["startup_s"] = round(time.time() - t0, 2)

        # ---------------------------------------------------------------- workload
        addrs = [servers[i] for i in sorted(servers)]
        inst = LMSClient(addrs, timeout=10)
        inst.register("prof", "pw", "instructor")
        lat: list[float] = []
        answers: list[int] = []
        errors: list[str] = []
        rejected = [0]
        lock = threading.Lock()
        start_q = threading.Event()

        def student(k: int):
            cl = LMSClient(addrs, timeout=10, llm_timeout=600, discover_timeout=30)
            try:
                topic = TOPICS[k % len(TOPICS)]
                u = f"student{k}"
                cl.register(u, "pw", "student")
                deadline = time.time() + 30
                while not cl.login(u, "pw"):
                    if time.time() > deadline:
                        raise RuntimeError("login never succeeded")
                    time.sleep(0.1)
                text = f"Assignment {k}: an essay on {topic}. " * 8
                if cfg["pdf"]:
                    ok = cl.post_assignment(data=make_pdf(text), filename=f"hw{k}.pdf")
                else:
                    ok = cl.post_assignment(data=text.encode(), filename=f"hw{k}.txt")
                if not ok:
                    raise RuntimeError("assignment post failed")
                start_q.wait()
                for q in range(args.queries):
                    t = time.perf_counter()
                    resp = cl.ask_llm(f"Can you explain {topic} for my assignment, part {q}?")
                    dt = (time.perf_counter() - t) * 1e3
                    with lock:
                        if "does not relate to your assignment" in resp:
                            rejected[0] += 1
                        elif resp.startswith("The tutoring service is unavailable") or "Invalid session" in resp:
                            errors.append(resp[:80])
                        elif not resp.startswith("You are an intelligent assistant"):
                            errors.append(resp[:80])  # any other LMS message is a failed query
                        else:
                            lat.append(dt)
                            answers.append(len(resp))
            except Exception as e:  # noqa: BLE001 -- recorded in the result
                with lock:
                    errors.append(repr(e)[:200])
            finally:
                cl.close()

        progress(f"{args.students} students x {args.queries} queries")
        ths = [threading.Thread(target=student, args=(k,)) for k in range(args.students)]
        for t in ths:
            t.start()
        time.sleep(1.0)  # let registrations/logins/posts land before the query burst
        failover = {}
        tq = time.perf_counter()
        start_q.set()
        if cfg["kill_leader"]:
            time.sleep(0.5)
            old = leader()
            tk = time.time()
            nodes[old].kill()
            wait_for(lambda: leader() not in (None, old), 30, "re-election")
            failover = {"killed_leader": old, "failover_s": round(time.time() - tk, 3), "new_leader": leader()}
        for t in ths:
            while t.is_alive():
                t.join(timeout=30)
                if t.is_alive():
                    progress(f"{len(lat)} answered, {len(errors)} errors so far")
        wall = time.perf_counter() - tq
        inst.close()

        result.update({
            "answered": len(lat), "gate_rejected": rejected[0], "errors": len(errors), "error_samples": errors[:3],
            "p50_ms": round(statistics.median(lat), 1) if lat else None,
            "p90_ms": round(sorted(lat)[int(0.9 * (len(lat) - 1))], 1) if lat else None,
            "max_ms": round(max(lat), 1) if lat else None,
            "queries_per_s": round(len(lat) / wall, 2), "wall_s": round(wall, 2),
            "data": "synthetic students/assignments/queries, random-init weights", **failover,
        })
        try:
            m = debug_call(f"127.0.0.1:{tutor_port}", "Metrics")
            result["tutor_tokens"] = m["counters"].get("tutor_tokens") or m["counters"].get("tutor_tokens_generated")
            if result["tutor_tokens"]:
                result["tutor_tokens_per_s"] = round(result["tutor_tokens"] / wall, 1)
        except Exception:
            pass
    finally:
        for p in procs:
            p.kill(signal.SIGTERM, wait=20)
    print(json.dumps(result), flush=True)
    return 0 if result.get("errors", 1) == 0 and result.get("answered", 0) > 0 else 1


if __name__ == "__main__":
    sys.exit(main())
