"""TP serving on CPU (gloo, world 2): rank 0 runs the continuous batcher over a TPEngineProxy that
mirrors every admit/decode to the follower rank; the sharded slot engines must reproduce the
unsharded fp32 greedy decode token for token, for staggered arrivals that reuse slots."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_lms_raft_llm_amd.models.config import GPT2Config
from distributed_lms_raft_llm_amd.models.gpt2 import (GPT2Reference, init_gpt2_weights, perturb_norms_and_biases,
                                                      reference_generate)

pytestmark = pytest.mark.timeout(300)

CFG = GPT2Config("gpt2-tp-serve", n_layer=2, n_embd=192, n_head=3, n_positions=64, vocab_size=500,
                 eos_token_id=499)
T = 24


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _weights():
    w = init_gpt2_weights(CFG, seed=5)
    perturb_norms_and_biases(w, scale=0.1)
    return w


def _prompts():
    g = torch.Generator().manual_seed(9)
    return [torch.randint(0, CFG.vocab_size - 1, (n,), generator=g).tolist() for n in (3, 7, 1, 12, 5, 9)]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_lms_raft_llm_amd.engine.scheduler import ContinuousBatcher
        from distributed_lms_raft_llm_amd.engine.tp_serving import TPEngineProxy, serve_follower
        from distributed_lms_raft_llm_amd.parallel.tp import TorchSlotEngine

        ctrl = dist.new_group(backend="gloo")
        eng = TorchSlotEngine(CFG, _weights(), group=dist.group.WORLD, max_batch=3, max_length=T)
        if rank == 0:
            proxy = TPEngineProxy(eng, ctrl, src=0)
            cb = ContinuousBatcher(proxy, repetition_penalty=1.2, chunk=2)
            futs = []
            for i, p in enumerate(_prompts()):
                futs.append(cb.submit(p))
                if i % 2:
                    time.sleep(0.01)
            outs = [f.result(200) for f in futs]
            cb.stop()
            proxy.close()
            q.put((rank, outs))
        else:
            q.put((rank, serve_follower(eng, ctrl, src=0)))
    finally:
        dist.destroy_process_group()


def test_tp_serving_matches_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in procs]
    res = dict(q.get(timeout=240) for _ in range(2))
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    ref = reference_generate(GPT2Reference(CFG, _weights()), _prompts(), max_length=T, repetition_penalty=1.2)
    assert res[0] == ref
    assert res[1] > 2  # the follower executed the mirrored admits/decodes


def test_torch_slot_engine_unsharded_matches_reference():
    from distributed_lms_raft_llm_amd.engine.scheduler import ContinuousBatcher
    from distributed_lms_raft_llm_amd.parallel.tp import TorchSlotEngine

    eng = TorchSlotEngine(CFG, _weights(), max_batch=2, max_length=T)
    cb = ContinuousBatcher(eng, chunk=3)
    try:
        outs = cb.generate(_prompts(), timeout=120)
    finally:
        cb.stop()
    ref = reference_generate(GPT2Reference(CFG, _weights()), _prompts(), max_length=T, repetition_penalty=1.2)
    assert outs == ref


def test_tutoring_server_cli_under_torchrun_tp2(tmp_path):
    """``torchrun --nproc-per-node 2 tutoring_server.py --device cpu``: rank 0 serves gRPC, rank 1
    follows; the answer equals the unsharded reference decode of the templated prompt."""
    import signal
    import subprocess
    import sys

    from distributed_lms_raft_llm_amd import wire
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.tokenizer import GPT2BPE
    from distributed_lms_raft_llm_amd.tutor.server import build_prompt
    from distributed_lms_raft_llm_amd.wire import pb

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _port()
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(root, "tutoring_server.py"),
           "--device", "cpu", "--model", "gpt2-tiny", "--max-length", "160", "--max-batch", "4",
           "--port", str(port), "--host", "127.0.0.1"]
    log = open(tmp_path / "tutor.log", "w")
    p = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, env=env, start_new_session=True)
    try:
        deadline = time.time() + 120
        while "Tutoring Server started" not in (tmp_path / "tutor.log").read_text():
            assert p.poll() is None and time.time() < deadline, (tmp_path / "tutor.log").read_text()
            time.sleep(0.2)
        stub = wire.Stub("Tutoring", wire.channel(f"127.0.0.1:{port}"))
        r = stub.GetLLMAnswer(pb.QueryRequest(token="t", query="what is a term?"), timeout=120)
        cfg = gpt2_config("gpt2-tiny")
        tok = GPT2BPE(eos_token_id=cfg.eos_token_id)
        ids = tok.encode(build_prompt("what is a term?"))
        ref = reference_generate(GPT2Reference(cfg, init_gpt2_weights(cfg, seed=0)), [ids], max_length=160)[0]
        assert r.success and r.response == tok.decode(ref)
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
    # (torchrun's own agent prints a SignalException traceback for the SIGTERM; the ranks must not)
    out = (tmp_path / "tutor.log").read_text()
    assert "[rank0]: Traceback" not in out and "[rank1]: Traceback" not in out, out
