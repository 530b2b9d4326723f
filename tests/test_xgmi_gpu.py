"""One-shot xGMI collectives (ops/csrc/xgmi.hip, parallel/xgmi.py) on ONE GPU: two processes share
cuda:0 and map each other's buffers through hipIpc handles exactly as TP ranks on different GPUs
do (the cross-GPU xGMI run is the driver's 8-GPU node).  Checked against a plain fp32 sum in rank
order (bit-exact), the int64 integer all-reduce against an exact integer sum, across message sizes
that change the grid between calls (the slab-parity protocol), replayed from a hipGraph, and end
to end in the TP engine."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

SIZES = [4, 1024, 64 * 1280, 4 * 1280, 1 << 20, 8, 256 * 1600]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank: int, n: int, call: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 * rank + 7 * call + n)
    return torch.randn(n, generator=g)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from distributed_lms_raft_llm_amd.parallel.xgmi import XgmiComm

        comm = XgmiComm(dist.group.WORLD, "cuda:0", 4 << 20)
        results = {}
        # eager: sizes alternate so consecutive calls use different grids
        for call, n in enumerate(SIZES * 2):
            t = _data(rank, n, call).cuda()
            comm.all_reduce_(t)
            results[("ar", call)] = t.cpu().numpy()
        # integer all-reduce (the TP fused layer's int64 fixed-point residual), eager
        for call, n in enumerate((2, 2 * 1280, 2 * 3 * 1600, 64 * 1024)):
            g = torch.Generator().manual_seed(500 * rank + call)
            t = torch.randint(-(1 << 46), 1 << 46, (n,), generator=g, dtype=torch.int64).cuda()
            comm.all_reduce_i64_(t)
            results[("i64", call)] = t.cpu().numpy()
        keys = torch.arange(37, dtype=torch.int64) * 1000 + rank
        out = torch.zeros(world, 37, dtype=torch.int64, device="cuda")
        comm.all_gather_u64(keys.cuda(), out)
        results["ag"] = out.cpu().numpy()
        # hipGraph: the call counter lives on the device, so replays keep the protocol going
        x = torch.zeros(64 * 1280, device="cuda")
        k_in = torch.zeros(64, dtype=torch.int64, device="cuda")
        k_out = torch.zeros(world, 64, dtype=torch.int64, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            comm.all_reduce_(x)  # warm-up call outside capture (both ranks)
            comm.all_gather_u64(k_in, k_out)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            comm.all_reduce_(x)
            comm.all_gather_u64(k_in, k_out)
        for rep in range(5):
            x.copy_(_data(rank, x.numel(), 100 + rep).cuda())
            k_in.fill_(rep * 10 + rank)
            g.replay()
            results[("graph", rep)] = (x.cpu().numpy(), k_out.cpu().numpy())
        # latency of a decode-sized all-reduce (64 rows x d=1280 fp32), eager launches
        torch.cuda.synchronize()
        dist.barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(200):
            comm.all_reduce_(x)
        ev1.record()
        ev1.synchronize()
        results["us_per_call"] = ev0.elapsed_time(ev1) * 1e3 / 200
        results["err"] = comm.error()
        comm.close()
        q.put((rank, results))  # numpy, pickled by value (no fd sharing past the worker's exit)
    finally:
        dist.destroy_process_group()


def test_xgmi_allreduce_allgather_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in procs]
    res = dict(q.get(timeout=500) for _ in range(2))
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert res[0]["err"] == 0 and res[1]["err"] == 0
    for call, n in enumerate(SIZES * 2):
        want = _data(0, n, call) + _data(1, n, call)  # rank order, fp32: bit-exact
        for r in (0, 1):
            assert torch.equal(torch.from_numpy(res[r][("ar", call)]), want), (call, n, r)
    for call, n in enumerate((2, 2 * 1280, 2 * 3 * 1600, 64 * 1024)):
        parts = [torch.randint(-(1 << 46), 1 << 46, (n,), generator=torch.Generator().manual_seed(500 * p + call),
                               dtype=torch.int64) for p in (0, 1)]
        for r in (0, 1):
            assert torch.equal(torch.from_numpy(res[r][("i64", call)]), parts[0] + parts[1]), (call, n, r)
    want_ag = torch.stack([torch.arange(37) * 1000 + p for p in (0, 1)])
    assert all(torch.equal(torch.from_numpy(res[r]["ag"]), want_ag) for r in (0, 1))
    for rep in range(5):
        want = _data(0, 64 * 1280, 100 + rep) + _data(1, 64 * 1280, 100 + rep)
        for r in (0, 1):
            x, k = res[r][("graph", rep)]
            assert torch.equal(torch.from_numpy(x), want), (rep, r)
            assert k.tolist() == [[rep * 10] * 64, [rep * 10 + 1] * 64]
    print("xgmi one-shot all-reduce, 320 KB, 2 ranks sharing one GPU: %.1f us/call" % res[0]["us_per_call"])
