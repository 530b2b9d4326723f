"""Tensor-parallel decode on CPU with the gloo backend (multi-process, world size 2 and 3):
sharded weights + all-reduce/all-gather placement reproduce the unsharded model exactly
(fp32), including an uneven head split and vocab shards."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_lms_raft_llm_amd.models.config import GPT2Config
from distributed_lms_raft_llm_amd.models.gpt2 import (GPT2Reference, init_gpt2_weights, perturb_norms_and_biases,
                                                      reference_generate)

pytestmark = pytest.mark.timeout(300)

# 5 heads: world 2 -> (3, 2) heads, world 3 -> (2, 2, 1); vocab 2000 -> 32 tiles of 64
CFG = GPT2Config("gpt2-tp-test", n_layer=2, n_embd=320, n_head=5, n_positions=128, vocab_size=2000,
                 eos_token_id=1999)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_lms_raft_llm_amd.parallel.tp import TorchTPGPT2

        w = init_gpt2_weights(CFG, seed=11)
        perturb_norms_and_biases(w, scale=0.1)
        m = TorchTPGPT2(CFG, w, group=dist.group.WORLD)
        g = torch.Generator().manual_seed(4)
        prompt = torch.randint(0, CFG.vocab_size - 1, (9,), generator=g).tolist()
        hid = m.forward(torch.tensor(prompt), torch.arange(len(prompt)), m.new_cache(40))
        out = m.generate(prompt, max_length=40)
        # numpy pickles by value: a torch tensor would go through the sender's resource-sharer socket,
        # which is gone if this worker exits before the parent reads the queue
        q.put((rank, m.w.head_range, m.w.vocab_range, hid[-1].detach().numpy().copy(), out, prompt))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tp_matches_unsharded(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    heads = [r[1] for r in res]
    assert heads[0][0] == 0 and heads[-1][1] == 5 and all(a[1] == b[0] for a, b in zip(heads, heads[1:]))
    assert max(h[1] - h[0] for h in heads) - min(h[1] - h[0] for h in heads) <= 1  # uneven but balanced
    w = init_gpt2_weights(CFG, seed=11)
    perturb_norms_and_biases(w, scale=0.1)
    ref = GPT2Reference(CFG, w)
    prompt = res[0][5]
    from distributed_lms_raft_llm_amd.models.gpt2 import KVCache

    hid = ref.forward(torch.tensor([prompt]), torch.arange(len(prompt))[None], KVCache.allocate(CFG, 1, 40),
                      torch.zeros(1, dtype=torch.long))[0, -1]
    for r in res:
        torch.testing.assert_close(torch.from_numpy(r[3]), hid, atol=1e-4, rtol=1e-4)
        assert r[4] == res[0][4]  # every rank produced the same tokens
    assert res[0][4] == reference_generate(ref, [prompt], max_length=40)[0]


def test_key_packing_orders_like_argmax():
    from distributed_lms_raft_llm_amd.parallel.tp import pack_keys, unpack_index

    vals = torch.tensor([-3.0, 2.5, 2.5, -0.0, 0.0, 7.0, -7.0])
    idx = torch.tensor([10, 4, 3, 8, 9, 100, 1])
    k = pack_keys(vals, idx)
    order = torch.argsort(k, descending=True)
    # value desc, ties -> lowest index first (torch.argmax semantics)
    assert idx[order].tolist()[:3] == [100, 3, 4]
    assert unpack_index(k).tolist() == idx.tolist()
