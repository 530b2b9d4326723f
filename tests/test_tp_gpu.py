"""HIP engine with tensor parallelism, functional check on ONE GPU: 2, 4 or 8 ranks share cuda:0
over the gloo backend or the one-shot xGMI kernels inside captured graphs (RCCL refuses two ranks
on one device; the 8-GPU RCCL/xGMI run is the driver's scaling bench).  Sharded kernels +
all-reduce/all-gather must reproduce TP=1 -- including BASELINE configs 4 and 5's geometries:
GPT-2-large (d 1280, 20 heads) at TP=4 and GPT-2-XL (d 1600, 25 heads) at TP=8, whose uneven head
split (4,3,3,3,3,3,3,3) and 832/768-column FFN shards run through every HIP kernel."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


GEOMETRIES = {
    "tp5": dict(n_layer=3, n_embd=320, n_head=5, n_positions=256, vocab_size=5000, eos_token_id=4999),
    "large": dict(n_layer=2, n_embd=1280, n_head=20, n_positions=256, vocab_size=5000, eos_token_id=4999),
    "xl": dict(n_layer=2, n_embd=1600, n_head=25, n_positions=256, vocab_size=5000, eos_token_id=4999),
    # GPT-2-124M itself: 12 layers, 12 heads (TP=8: 2,2,2,2,1,1,1,1 -- one-head ranks), the real 50257
    # vocabulary padded to 50304 (6288-column shards through the LM head and the argmax all-gather)
    "124m": dict(n_layer=12, n_embd=768, n_head=12, n_positions=1024, vocab_size=50257, eos_token_id=50256),
    # the same geometry, 2 layers: the xGMI-graph runs (8 ranks' spinning one-shot barriers time-share
    # ONE GPU here; 12 layers of them timed out a barrier -- on 8 GPUs every rank has its own)
    "124m-2l": dict(n_layer=2, n_embd=768, n_head=12, n_positions=1024, vocab_size=50257, eos_token_id=50256),
}


def _setup(geo="tp5", n_prompts=3):
    from distributed_lms_raft_llm_amd.models.config import GPT2Config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights, perturb_norms_and_biases

    cfg = GPT2Config(f"gpt2-{geo}", **GEOMETRIES[geo])
    w = init_gpt2_weights(cfg, seed=21)
    perturb_norms_and_biases(w, scale=0.1)
    for k, v in w.items():  # bf16-exact weights: the oracle sees what the kernels see
        if v.dim() == 2:
            w[k] = v.to(torch.bfloat16).float()
    g = torch.Generator().manual_seed(2)
    lens = [6, 17, 30] if n_prompts == 3 else [int(x) for x in torch.randint(1, 33, (n_prompts,), generator=g)]
    prompts = [torch.randint(0, cfg.vocab_size - 1, (L,), generator=g).tolist() for L in lens]
    return cfg, w, prompts


def _worker(rank, world, port, q, p2p=False, geo="tp5", wdt="bf16", n_prompts=3, max_batch=4):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if p2p and n_prompts > 4:
        # every collective on the one-shot xGMI kernels, as on 8 GPUs with RCCL behind them: the
        # packed 32-prompt prefill's messages (~1.6 MB) would otherwise fall back to this group's gloo
        # calls, which cannot be captured into the prefill graph
        os.environ["DLMS_XGMI_SLAB_MB"] = "8"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

        cfg, w, prompts = _setup(geo, n_prompts)
        # p2p: one-shot xGMI kernels instead of gloo calls -- all on the GPU, so hipGraph capture works
        eng = HipGPT2Engine(cfg, w, max_batch=max_batch, max_length=64, tp_group=dist.group.WORLD, use_graph=p2p,
                            p2p=p2p, weight_dtype=wdt)
        assert (eng.xgmi is not None) == p2p and eng.w.fp8 == (wdt == "fp8")
        hid = eng.prefill_last_hidden(prompts).cpu()
        out = eng.generate(prompts)
        fused = eng.tp_fused_steps
        if geo in ("large", "xl") or (geo.startswith("124m") and len(prompts) <= 4):  # the fused TP layer ran
            assert eng.tp_fused and fused > 0, (eng.tp_fused, fused)
        # a second generation of the same shapes: replays the captured prefill (xGMI) -- same tokens
        assert eng.generate(prompts) == out
        if p2p:
            assert any(st["graph"] is not None for st in eng._pgraphs.values()), "no TP prefill graph"
        q.put((rank, eng.w.head_range, hid.numpy(), out, eng.w.ffn_range, tuple(eng.w.vocab_range),
               int(eng.w.lm_head.shape[0])))
    finally:
        dist.destroy_process_group()


def _run_tp(geo, world, p2p, wdt="bf16", n_prompts=3, max_batch=4):
    """TP=world ranks on cuda:0 vs TP=1 bf16, both margin-checked against the fp32 oracle.  fp8 (W8A8
    prefill, bf16 latency-path decode): last-token hidden states within cosine 0.99 of the bf16
    TP=1 engine, and the oracle's token at every position whose top-1 / top-2 margin exceeds 0.5
    (profiles/r5_config5_tp8_fp8_tests.txt)."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.engine.weights import shard_range
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, teacher_forced_check

    cfg, w, prompts = _setup(geo, n_prompts)
    ref_eng = HipGPT2Engine(cfg, w, max_batch=max_batch, max_length=64, use_graph=False)
    ref_hid = ref_eng.prefill_last_hidden(prompts).cpu()
    ref_out = ref_eng.generate(prompts)
    del ref_eng
    torch.cuda.empty_cache()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, p2p, geo, wdt, n_prompts, max_batch))
             for r in range(world)]
    [p.start() for p in procs]
    import queue as _queue
    import time as _time

    t0, res = _time.time(), []
    try:
        while len(res) < world:  # (a progress line every 30 s: a long shared-GPU run is not a hang)
            try:
                res.append(q.get(timeout=30))
            except _queue.Empty:
                print(f"[tp {geo} x{world}] {len(res)}/{world} ranks done after {_time.time() - t0:.0f} s", flush=True)
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                if dead or _time.time() - t0 > 800:  # a failed rank leaves its peers in a collective
                    raise AssertionError(f"TP ranks failed (exit codes {dead}) or timed out")
        res = sorted(res, key=lambda r: r[0])
    finally:
        [p.join(timeout=60) for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert [r[1] for r in res] == [shard_range(cfg.n_head, world, r) for r in range(world)]
    ftiles = [shard_range(cfg.n_inner // 64, world, r) for r in range(world)]
    assert [r[4] for r in res] == [(a * 64, b * 64) for a, b in ftiles]
    for r in res:
        cos = torch.nn.functional.cosine_similarity(torch.from_numpy(r[2]), ref_hid, dim=-1)
        assert bool((cos > (0.99 if wdt == "fp8" else 0.999)).all()), cos
        assert r[3] == res[0][3]  # every rank emits the same tokens
    # margin-aware exactness against the fp32 oracle (teacher-forced on each engine's own output):
    # TP=world and TP=1 must both pick the oracle's greedy token wherever it is decisive
    oracle = GPT2Reference(cfg, w, device="cuda")
    # (fp8: the margin rule at 0.5 -- e4m3 rounding moves logits by more than the bf16 rule's 0.05 --,
    # every such position the oracle's token; on this random-init geometry 25 of 139 positions
    # clear 0.5, so at least 10 % are required to be decisive)
    for outs, eps, frac in ((res[0][3], 0.5 if wdt == "fp8" else 0.05, 0.1 if wdt == "fp8" else 0.7),
                            (ref_out, 0.05, 0.7)):
        decisive = total = 0
        for o, p in zip(outs, prompts):
            assert o[: len(p)] == p
            r = teacher_forced_check(oracle, o, len(p), 1.2, eps=eps)
            assert not r["mismatches"], r["mismatches"]
            decisive += r["decisive"]
            total += r["positions"]
        assert decisive >= frac * total, (decisive, total)
    return res


@pytest.mark.parametrize("geo,world,p2p", [("large", 4, False), ("large", 4, True), ("xl", 8, False),
                                           ("xl", 8, True)],
                         ids=["large-tp4-gloo", "large-tp4-xgmi-graph", "xl-tp8-gloo", "xl-tp8-xgmi-graph"])
def test_tp_configs_4_and_5_geometry_on_one_gpu(geo, world, p2p):
    """BASELINE configs 4 / 5: GPT-2-large's 20 heads over 4 ranks (5 each), GPT-2-XL's 25 heads
    over 8 ranks (4,3,3,3,3,3,3,3) with 832/768-column FFN shards."""
    res = _run_tp(geo, world, p2p)
    if geo == "xl":
        assert [b - a for a, b in (r[1] for r in res)] == [4, 3, 3, 3, 3, 3, 3, 3]
        assert sorted({b - a for a, b in (r[4] for r in res)}) == [768, 832]


@pytest.mark.parametrize("p2p", [False, True], ids=["gloo", "xgmi-graph"])
def test_tp2_on_one_gpu_matches_tp1(p2p):
    res = _run_tp("tp5", 2, p2p)
    assert [r[1] for r in res] == [(0, 3), (3, 5)]


@pytest.mark.parametrize("p2p", [False, True], ids=["gloo", "xgmi-graph"])
def test_config5_xl_tp8_fp8_on_one_gpu(p2p):
    """BASELINE config 5 as specified: GPT-2-XL geometry, TP=8, fp8 (W8A8 e4m3 QKV / c_fc / LM head in
    the prefill and batches > 8; the bf16 six-kernel fused TP layer at these 3 rows), 8 ranks on one
    GPU."""
    res = _run_tp("xl", 8, p2p, wdt="fp8")
    assert [b - a for a, b in (r[1] for r in res)] == [4, 3, 3, 3, 3, 3, 3, 3]


# (the 32-row xGMI-graph case failed its run0 == run1 check until round 6 fixed the graph warm-up's
# snapshot order in HipGPT2Engine._graph_for -- scripts/tp_debug_repro.py, profiles/r6_tp124m_tests.txt)
@pytest.mark.parametrize("geo,rows,p2p", [("124m", 4, False), ("124m", 32, False), ("124m-2l", 4, True),
                                           ("124m-2l", 32, True)],
                         ids=["124m-tp8-4rows-gloo", "124m-tp8-32rows-gloo", "124m-2l-tp8-4rows-xgmi-graph",
                              "124m-2l-tp8-32rows-xgmi-graph"])
def test_gpt2_124m_tp8_real_geometry_on_one_gpu(geo, rows, p2p):
    """GPT-2-124M at TP=8: heads 2,2,2,2,1,1,1,1 (four one-head ranks), the real
    50257-token vocabulary padded to 50304 and sharded 6288 columns per rank (the last shard partly
    masked), at 4 rows (the fused six-kernel TP layer) and 32 rows (the tiled TP step) -- every rank
    emits the same tokens, which hold the fp32 oracle's greedy choice at every decisive position."""
    res = _run_tp(geo, 8, p2p, n_prompts=rows, max_batch=rows)
    assert [b - a for a, b in (r[1] for r in res)] == [2, 2, 2, 2, 1, 1, 1, 1]
    # the padded vocabulary in 64-column tiles over the ranks (99 or 98 tiles each), contiguous, the
    # last shard holding the 47 padding columns the LM head masks
    vr = [r[5] for r in res]
    assert vr[0][0] == 0 and vr[-1][1] == 50304 and all(vr[i][1] == vr[i + 1][0] for i in range(7)), vr
    assert all(r[6] == b - a and (b - a) % 64 == 0 for r, (a, b) in zip(res, vr)), [r[6] for r in res]
    assert vr[-1][0] < 50257 < vr[-1][1]
