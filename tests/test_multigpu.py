"""Tensor parallelism across SEPARATE GPUs of one node (one process per GPU, RCCL over xGMI):
the paths the one-GPU functional tests (test_tp_gpu.py, test_xgmi_gpu.py) cannot reach --
xGMI peer-memory visibility between devices, RCCL all-reduce captured inside the decode
hipGraph, the ``dist.all_gather_into_tensor`` branch of the vocab-parallel argmax, and the
one-shot xGMI kernels across devices.  Each test needs N visible GPUs and is skipped otherwise
(``multigpu(n)`` marker, tests/conftest.py); the 8-GPU scaling run is the driver's."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    # (importing the package before the first GPU call sets HSA_ENABLE_IPC_MODE_LEGACY=0 exactly as
    # the tutor and bench.py get it: distributed_lms_raft_llm_amd/__init__.py)
    import distributed_lms_raft_llm_amd  # noqa: F401

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    assert os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device(f"cuda:{rank}"))


def _xgmi_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from distributed_lms_raft_llm_amd.parallel.xgmi import XgmiComm

        comm = XgmiComm(dist.group.WORLD, f"cuda:{rank}", 4 << 20)
        out = {}
        for call, n in enumerate([4, 3072, 64 * 1600, 1 << 20]):
            g = torch.Generator().manual_seed(100 * rank + call)
            t = torch.randn(n, generator=g).cuda()
            comm.all_reduce_(t)
            out[call] = t.cpu().numpy()
        keys = torch.arange(33, dtype=torch.int64, device="cuda") * 10 + rank
        ag = torch.zeros(world, 33, dtype=torch.int64, device="cuda")
        comm.all_gather_u64(keys, ag)
        out["ag"] = ag.cpu().numpy()
        comm.check()
        comm.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [pytest.param(n, marks=pytest.mark.multigpu(n)) for n in (2, 4, 8)])
def test_xgmi_one_shot_across_devices(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_xgmi_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = dict(q.get(timeout=600) for _ in range(world))
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    for call, n in enumerate([4, 3072, 64 * 1600, 1 << 20]):
        want = np.zeros(n, dtype=np.float32)
        for r in range(world):  # the kernel sums in rank order: bit-exact
            want += torch.randn(n, generator=torch.Generator().manual_seed(100 * r + call)).numpy()
        for r in range(world):
            np.testing.assert_array_equal(res[r][call], want)
    for r in range(world):
        np.testing.assert_array_equal(res[r]["ag"], np.stack([np.arange(33) * 10 + p for p in range(world)]))


def _setup():
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights, perturb_norms_and_biases

    cfg = gpt2_config("gpt2")  # 12 heads: TP=8 exercises the uneven head split (2,2,2,2,1,1,1,1)
    w = init_gpt2_weights(cfg, seed=3)
    perturb_norms_and_biases(w)
    for k, v in w.items():
        if v.dim() == 2:
            w[k] = v.to(torch.bfloat16).float()
    g = torch.Generator().manual_seed(4)
    prompts = [torch.randint(0, cfg.vocab_size - 1, (L,), generator=g).tolist() for L in (5, 19, 32, 2)]
    return cfg, w, prompts


def _tp_worker(rank, world, port, q, p2p, batch):
    _init(rank, world, port)
    try:
        from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

        cfg, w, prompts = _setup()
        # p2p=False: RCCL all-reduce + all_gather_into_tensor, captured in the decode hipGraph
        eng = HipGPT2Engine(cfg, w, max_batch=batch, max_length=48, tp_group=dist.group.WORLD, use_graph=True,
                            p2p=p2p)
        assert (eng.xgmi is not None) == p2p
        outs = eng.generate(prompts)
        if eng.xgmi is not None:
            eng.xgmi.check()
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("p2p", [False, True], ids=["rccl-graph", "xgmi-graph"])
@pytest.mark.parametrize("batch", [4, 32], ids=["latency-path", "tiled-path"])
@pytest.mark.parametrize("world", [pytest.param(n, marks=pytest.mark.multigpu(n)) for n in (2, 4, 8)])
def test_tp_across_devices_matches_oracle(world, p2p, batch):
    """TP=N tokens: identical on every rank, and equal to the fp32 oracle's greedy choice wherever
    it is decisive (teacher-forced margin rule, models/gpt2.py)."""
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, teacher_forced_check

    cfg, w, prompts = _setup()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, p2p, batch)) for r in range(world)]
    [p.start() for p in procs]
    res = dict(q.get(timeout=800) for _ in range(world))
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert all(res[r] == res[0] for r in range(world))
    oracle = GPT2Reference(cfg, w, device="cuda:0")
    decisive = total = 0
    for o, p in zip(res[0], prompts):
        r = teacher_forced_check(oracle, o, len(p), 1.2, eps=0.05)
        assert not r["mismatches"], r["mismatches"]
        decisive += r["decisive"]
        total += r["positions"]
    assert decisive >= 0.7 * total
