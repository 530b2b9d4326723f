"""GPT-2 engine on the GPU vs the plain-torch fp32 reference with the same bf16-rounded weights."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(name="gpt2", seed=0):
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights, perturb_norms_and_biases

    cfg = gpt2_config(name)
    w = init_gpt2_weights(cfg, seed=seed)
    perturb_norms_and_biases(w)
    # round GEMM/embedding weights to bf16 so the oracle sees exactly what the kernels see
    for k, v in w.items():
        if v.dim() == 2:
            w[k] = v.to(torch.bfloat16).float()
    return cfg, w


def _prompts(cfg, lens, seed=1):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, cfg.vocab_size - 1, (L,), generator=g).tolist() for L in lens]


@pytest.mark.parametrize("name", ["gpt2-tiny", "gpt2", "gpt2-medium", "gpt2-xl"])
def test_prefill_hidden_matches_reference(name):
    """gpt2-xl: 25 heads, d = 1600 (not a multiple of 256/128: ragged LayerNorm lanes, fp8 K pad)."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, KVCache

    cfg, w = _setup(name)
    eng = HipGPT2Engine(cfg, w, max_batch=4, max_length=64)
    prompts = _prompts(cfg, [7, 32, 1])
    got = eng.prefill_last_hidden(prompts)
    ref_m = GPT2Reference(cfg, w, device="cuda")
    for b, p in enumerate(prompts):
        cache = KVCache.allocate(cfg, 1, 64, device="cuda")
        t = torch.tensor([p], device="cuda")
        hid = ref_m.forward(t, torch.arange(len(p), device="cuda")[None], cache, torch.zeros(1, dtype=torch.long,
                                                                                             device="cuda"))
        ref = hid[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[b], ref, dim=0).item()
        assert cos > 0.999, cos
        torch.testing.assert_close(got[b], ref, atol=0.1, rtol=0.05)


def _assert_teacher_forced(model, outs, prompts, eps=0.05, min_decisive=0.7):
    """Every generated token equals the fp32 oracle's greedy choice (teacher-forced on the
    engine's own prefix) wherever the oracle's top-1/top-2 margin exceeds ``eps``."""
    from distributed_lms_raft_llm_amd.models.gpt2 import teacher_forced_check

    total = decisive = 0
    for o, p in zip(outs, prompts):
        assert o[: len(p)] == p
        r = teacher_forced_check(model, o, len(p), 1.2, eps)
        assert not r["mismatches"], r["mismatches"]
        total += r["positions"]
        decisive += r["decisive"]
    assert total > 0 and decisive >= min_decisive * total, (decisive, total)


@pytest.mark.parametrize("name,batch", [("gpt2-tiny", 3), ("gpt2", 1), ("gpt2", 3), ("gpt2", 8), ("gpt2", 24),
                                        ("gpt2-medium", 1), ("gpt2-medium", 2), ("gpt2-xl", 2)])
def test_generate_matches_reference_tokens(name, batch):
    """bf16 engine vs fp32 oracle, margin-aware and exact: batch 1 runs the dataflow decode, 2 the
    latency path, 3/8/24 the mid path (tests/test_mid_gpu.py covers it in depth)."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference

    cfg, w = _setup(name)
    T = 48
    eng = HipGPT2Engine(cfg, w, max_batch=max(8, batch), max_length=T)
    prompts = _prompts(cfg, [5, 20, 11, 1, 30, 8, 16, 2][:batch] + [9] * max(0, batch - 8))
    got = eng.generate(prompts, repetition_penalty=1.2)
    for g_ in got:
        assert len(g_) <= T
    _assert_teacher_forced(GPT2Reference(cfg, w, device="cuda"), got, prompts)


def test_latency_path_matches_tiled_path(monkeypatch):
    """The latency-shaped decode step (B <= 8; by default it serves B <= 2 and the mid path 3+,
    DLMS_SMALL_MAX_ROWS widens it back) and the tiled step produce the same greedy tokens under the
    margin rule (both checked against the fp32 oracle), and the path is actually taken."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference

    monkeypatch.setenv("DLMS_SMALL_MAX_ROWS", "8")
    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [7, 19, 3, 32], seed=9)
    fast = HipGPT2Engine(cfg, w, max_batch=4, max_length=64)
    slow = HipGPT2Engine(cfg, w, max_batch=4, max_length=64, latency_path=False)
    assert fast._small_ok(4) and not slow._small_ok(4)
    ref = GPT2Reference(cfg, w, device="cuda")
    _assert_teacher_forced(ref, fast.generate(prompts), prompts)
    _assert_teacher_forced(ref, slow.generate(prompts), prompts)


@pytest.mark.parametrize("name", ["gpt2", "gpt2-medium", "gpt2-large", "gpt2-xl"])
def test_fused_mlp_batch1(name, monkeypatch):
    """Batch 1 runs LN2 -> c_fc -> GELU -> c_proj as one kernel into the int64 fixed-point residual:
    exact under the margin rule against the fp32 oracle, identical across graph replay / eager and
    across repeated runs (integer atomics), and tracking the unfused path."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference

    monkeypatch.setenv("DLMS_DATAFLOW", "0")  # the launch-per-op batch-1 path under test
    cfg, w = _setup(name)
    prompts = _prompts(cfg, [13], seed=21)
    fused = HipGPT2Engine(cfg, w, max_batch=1, max_length=64)
    assert fused.fused_mlp and fused.xr is not None
    # batch 1 of 12 / 16 heads: attention fused with the out-projection in 4 head-group slabs
    assert bool(fused.ao_groups) == (name in ("gpt2", "gpt2-medium"))
    a = fused.generate(prompts)
    assert fused.generate(prompts) == a
    assert HipGPT2Engine(cfg, w, max_batch=1, max_length=64, use_graph=False).generate(prompts) == a
    _assert_teacher_forced(GPT2Reference(cfg, w, device="cuda"), a, prompts)
    monkeypatch.setenv("DLMS_FUSED_MLP", "0")
    plain = HipGPT2Engine(cfg, w, max_batch=1, max_length=64)
    assert not plain.fused_mlp
    _assert_teacher_forced(GPT2Reference(cfg, w, device="cuda"), plain.generate(prompts), prompts)


@pytest.mark.parametrize("batch,rows", [(2, "2"), (3, "4")])
def test_fused_mlp_small_batch(batch, rows, monkeypatch):
    """2+ rows on the fused-MLP path (split attention, out-projection added in place into the
    fixed-point residual): exact under the margin rule, identical across graph / eager and runs."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference

    monkeypatch.setenv("DLMS_FUSED_MLP_ROWS", rows)
    monkeypatch.setenv("DLMS_SMALL_MAX_ROWS", "8")  # (3+ rows default to the mid path)
    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [13, 4, 27][:batch], seed=23)
    eng = HipGPT2Engine(cfg, w, max_batch=8, max_length=64)
    assert eng.fused_mlp_rows >= batch
    a = eng.generate(prompts)
    assert eng.generate(prompts) == a
    assert HipGPT2Engine(cfg, w, max_batch=8, max_length=64, use_graph=False).generate(prompts) == a
    _assert_teacher_forced(GPT2Reference(cfg, w, device="cuda"), a, prompts)


def test_graph_replay_equals_eager():
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [32] * 5 + [9, 17])
    a = HipGPT2Engine(cfg, w, max_batch=8, max_length=80, use_graph=True).generate(prompts)
    b = HipGPT2Engine(cfg, w, max_batch=8, max_length=80, use_graph=False).generate(prompts)
    assert a == b


def test_prefill_graph_equals_eager():
    """A (rows, prompts) prefill shape seen twice is replayed from a hipGraph (padded tile table):
    tokens bit-identical to eager prefills, also for a different length mix of the same shape and
    through the continuous-batching admit path."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    cfg, w = _setup("gpt2")
    g_eng = HipGPT2Engine(cfg, w, max_batch=8, max_length=72)
    e_eng = HipGPT2Engine(cfg, w, max_batch=8, max_length=72)
    e_eng.prefill_graphs = False
    mixes = [[32], [32], [32], [20, 12, 30], [30, 20, 12], [31, 1, 30], [40, 17]]
    for i, lens in enumerate(mixes):
        prompts = _prompts(cfg, lens, seed=10 + i)
        assert g_eng.generate(prompts) == e_eng.generate(prompts), lens
    assert (32, 1) in g_eng._pgraphs and g_eng._pgraphs[(32, 1)]["graph"] is not None
    assert (62, 3) in g_eng._pgraphs and g_eng._pgraphs[(62, 3)]["graph"] is not None
    assert not e_eng._pgraphs
    # admit into arbitrary slots (the serving path), twice with one shape
    for eng in (g_eng, e_eng):
        eng._reset_slots(0, 8)
    for rep in range(2):
        prompts = _prompts(cfg, [9, 23], seed=30 + rep)
        outs = []
        for eng in (g_eng, e_eng):
            eng.admit(prompts, [5, 2])
            eng.decode(8, 6)
            outs.append(eng.collect([5, 2]))
        assert outs[0] == outs[1]


@pytest.mark.parametrize("use_graph,parts", [(True, 2), (False, 2), (True, 4)])
def test_overlapped_multi_stream_step_equals_serial(use_graph, parts, monkeypatch):
    """The multi-stream decode step (row ranges on 2-4 free-running streams) computes exactly what
    the single-stream step computes."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    # same split-K as the single-stream step, so the sums (and tokens) must be bit-identical; the
    # production cap for concurrent parts (2) changes the summation order: see the test below
    monkeypatch.setenv("DLMS_OVERLAP_SPLIT_CAP", "8")
    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [32] * 6 + [9, 17, 3, 25], seed=5)
    ov = HipGPT2Engine(cfg, w, max_batch=16, max_length=72, use_graph=use_graph, overlap=True, overlap_min_batch=2,
                       overlap_parts=parts)
    assert ov._overlap_ok(16)
    a = ov.generate(prompts)
    b = HipGPT2Engine(cfg, w, max_batch=16, max_length=72, use_graph=use_graph, overlap=False).generate(prompts)
    assert a == b


def test_multi_step_graph_equals_single_step(monkeypatch):
    """Several decode steps per graph replay (each row part runs them back to back on its own
    stream, joining once per replay) compute exactly what one step per replay computes."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [32] * 6 + [9, 17, 3, 25], seed=5)
    kw = dict(max_batch=16, max_length=72, overlap=True, overlap_min_batch=2, overlap_parts=2)
    a = HipGPT2Engine(cfg, w, **kw).generate(prompts)
    monkeypatch.setenv("DLMS_STEPS_PER_GRAPH", "4")
    eng = HipGPT2Engine(cfg, w, **kw)
    assert eng.steps_per_graph == 4
    assert eng.generate(prompts) == a


def test_warm_decode_graphs_covers_first_use():
    """The server's start-up capture (``warm_decode_graphs``) leaves nothing for the first queries
    to capture, and the tokens are those of an engine that captured on first use."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [5 + (3 * i) % 20 for i in range(10)], seed=41)
    ref = HipGPT2Engine(cfg, w, max_batch=64, max_length=61).generate(prompts)
    eng = HipGPT2Engine(cfg, w, max_batch=64, max_length=61)
    n, secs = eng.warm_decode_graphs(1.2, 64)
    assert n >= 2 and len(eng._graphs) == n and secs >= 0
    keys = set(eng._graphs)
    assert eng.generate(prompts) == ref
    assert set(eng._graphs) == keys  # every decode graph of the 16-row bucket was already there


@pytest.mark.parametrize("batch", [1, 2, 5, 24])
def test_multi_step_graph_small_paths(batch, monkeypatch):
    """Latency path (fused MLP at 1-2 rows) and the mid path (5, 24 rows) with
    4 steps per graph replay: the same tokens as one step per replay."""
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    monkeypatch.setenv("DLMS_DATAFLOW", "0")  # graph replays of the launch-per-op steps
    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [5 + (7 * i) % 27 for i in range(batch)], seed=29)
    monkeypatch.setenv("DLMS_STEPS_PER_GRAPH_SMALL", "1")
    a = HipGPT2Engine(cfg, w, max_batch=max(8, batch), max_length=61).generate(prompts)
    monkeypatch.setenv("DLMS_STEPS_PER_GRAPH_SMALL", "4")
    eng = HipGPT2Engine(cfg, w, max_batch=max(8, batch), max_length=61)
    assert eng.steps_per_graph_small == 4
    assert eng.generate(prompts) == a


def test_production_throughput_path_matches_fp32_oracle():
    """The exact path every BENCH step runs -- default knobs, the BENCH shape: 1024 rows of
    32-token prompts to max_length 150, i.e. two 512-row parts on HIP streams (overlap_min_batch
    512), split-K cap 2, 768-block persistent attention, 8 decode steps per graph replay, the
    panel-resident LM head, LN1 fused into ``decode_update`` and the split-K slabs summed by
    ``add_layernorm``, and the 64x96 GEMM tiles of 256 < M <= 512 (QKV + K/V scatter, c_fc + GELU,
    c_proj) -- with the
    64x96 dispatch asserted from the launch census and every row checked against the fp32 oracle
    with the margin rule."""
    from distributed_lms_raft_llm_amd import ops
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.gpt2 import GPT2Reference, teacher_forced_check_batch

    cfg, w = _setup("gpt2")
    B, T = 1024, 150
    eng = HipGPT2Engine(cfg, w, max_batch=B, max_length=T)  # nothing overridden
    assert eng._overlap_ok(B) and not eng._small_ok(B)
    assert (eng.overlap_split_cap, eng.persist_attn_blocks, eng.steps_per_graph, eng.overlap_parts) == (2, 768, 8, 2)
    assert eng.ps_lm and eng.gemm96
    prompts = _prompts(cfg, [32] * B, seed=5)
    ops.gemm_tile_reset()
    got = eng.generate(prompts, repetition_penalty=1.2)
    # per captured step and part: QKV, c_fc, c_proj on 64x96 in each of 12 layers
    assert ops.gemm_tile_count(64, 96) >= 3 * cfg.n_layer * 2
    assert all(len(g_) <= T for g_ in got)
    res = teacher_forced_check_batch(GPT2Reference(cfg, w, device="cuda"), got, [len(p) for p in prompts])
    bad = [(i, r["mismatches"][:2]) for i, r in enumerate(res) if r["mismatches"]]
    assert not bad, bad[:4]
    total, decisive = sum(r["positions"] for r in res), sum(r["decisive"] for r in res)
    assert total > 50 * B and decisive >= 0.7 * total, (decisive, total)


def test_continuous_batching_matches_static(monkeypatch):
    """Requests admitted into free slots of a running batch (8 slots, 14 staggered requests)
    produce BIT-IDENTICALLY what a static batch of each request alone produces: rows are
    independent sequences and, with the prefill split-K pinned (M-independent), every row's
    arithmetic is the same whatever else shares the batch.  (Launch-per-op throughout: a lone
    live slot would otherwise decode on the dataflow kernel, which sums in another order --
    tests/test_dataflow_gpu.py checks that path through the batcher against the oracle.)"""
    import time

    monkeypatch.setenv("DLMS_DATAFLOW", "0")
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.engine.scheduler import ContinuousBatcher

    cfg, w = _setup("gpt2")
    T = 64
    prompts = _prompts(cfg, [3, 30, 12, 1, 25, 7, 40, 16, 2, 33, 9, 21, 5, 63], seed=3)
    eng = HipGPT2Engine(cfg, w, max_batch=8, max_length=T, prefill_split=2)
    cb = ContinuousBatcher(eng, repetition_penalty=1.2, chunk=4)
    try:
        futs = []
        for i, p in enumerate(prompts):
            futs.append(cb.submit(p))
            if i % 4 == 3:
                time.sleep(0.02)
        got = [f.result(120) for f in futs]
    finally:
        cb.stop()
    solo = HipGPT2Engine(cfg, w, max_batch=1, max_length=T, prefill_split=2)
    for g_, p in zip(got, prompts):
        assert g_ == solo.generate([p], repetition_penalty=1.2)[0]
    assert cb.completed == len(prompts)


def test_fp8_engine_tracks_bf16():
    """W8A8 e4m3 engine (QKV, c_fc, LM head on the fp8 MFMA path): last-token hidden states stay
    close to the bf16 engine's and greedy decode agrees on the first tokens."""
    cfg, w = _setup("gpt2")
    prompts = _prompts(cfg, [12, 30, 5], seed=7)
    _fp8_vs_bf16(cfg, w, prompts)


def test_fp8_engine_tracks_bf16_xl():
    cfg, w = _setup("gpt2-xl")
    _fp8_vs_bf16(cfg, w, _prompts(cfg, [12, 3], seed=8), first_token=False, min_cos=0.97)


def _fp8_vs_bf16(cfg, w, prompts, first_token=True, min_cos=0.99):
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    e16 = HipGPT2Engine(cfg, w, max_batch=4, max_length=48)
    e8 = HipGPT2Engine(cfg, w, max_batch=4, max_length=48, weight_dtype="fp8")
    assert e8.w.fp8 and e8.w.layers[0].w_qkv8 is not None
    h16, h8 = e16.prefill_last_hidden(prompts), e8.prefill_last_hidden(prompts)
    for a, b in zip(h16, h8):
        assert torch.nn.functional.cosine_similarity(a, b, dim=0).item() > min_cos
    g16, g8 = e16.generate(prompts), e8.generate(prompts)
    for a, b, p in zip(g16, g8, prompts):
        assert b[: len(p)] == p and len(b) <= 48
        if first_token:
            assert a[len(p)] == b[len(p)]
