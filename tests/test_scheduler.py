"""Continuous-batching scheduler (engine/scheduler.py) on a CPU fake engine that follows the slot
protocol: admission into free slots while others run, slot reuse, per-request outputs identical
to running each request alone, pass-through of degenerate prompts, loud failure propagation."""
import threading
import time
from types import SimpleNamespace

import pytest

from distributed_lms_raft_llm_amd.engine.scheduler import ContinuousBatcher

V, EOS = 97, 96


def next_token(seq):
    return (sum(seq) * 31 + len(seq) * 7) % V


def solo(prompt, T, stop_at_eos=True):
    seq = list(prompt)
    while len(seq) < T:
        t = next_token(seq)
        seq.append(t)
        if t == EOS and stop_at_eos:
            break
    return seq


class FakeSlotEngine:
    def __init__(self, max_batch=4, max_length=40):
        self.max_batch, self.max_length = max_batch, max_length
        self.cfg = SimpleNamespace(eos_token_id=EOS)
        self.seqs = [[EOS] for _ in range(max_batch)]
        self.fin = [1] * max_batch
        self.lock = threading.Lock()
        self.admitted_while_busy = 0
        self.buckets = []
        self.fail_after = None
        self.stop_at_eos = True

    def _step(self, s):
        if self.fin[s]:
            return
        t = next_token(self.seqs[s])
        self.seqs[s].append(t)
        if (t == EOS and self.stop_at_eos) or len(self.seqs[s]) >= self.max_length:
            self.fin[s] = 1

    def admit(self, prompts, slots, penalty):
        assert len(set(slots)) == len(slots)
        if any(not f for f in self.fin):
            self.admitted_while_busy += 1
        for p, s in zip(prompts, slots):
            assert self.fin[s], "admitted into a live slot"
            self.seqs[s] = list(p)
            self.fin[s] = 0
            self._step(s)  # prefill emits the first token

    def decode(self, B, steps, penalty):
        self.buckets.append(B)
        if self.fail_after is not None:
            self.fail_after -= 1
            if self.fail_after < 0:
                raise RuntimeError("device lost")
        assert not any(not self.fin[s] for s in range(B, self.max_batch)), "live slot outside bucket"
        for _ in range(steps):
            for s in range(B):
                self._step(s)
        time.sleep(0.001)

    def finished_flags(self, B):
        return self.fin[:B]

    def collect(self, slots):
        return [list(self.seqs[s]) for s in slots]


def _prompts(n, seed=0):
    import random

    r = random.Random(seed)
    return [[r.randrange(0, V - 1) for _ in range(r.randrange(1, 12))] for _ in range(n)]


def test_outputs_match_solo_runs_with_staggered_arrivals():
    eng = FakeSlotEngine(max_batch=4, max_length=40)
    cb = ContinuousBatcher(eng, chunk=3)
    try:
        prompts = _prompts(23)
        futs = []
        for i, p in enumerate(prompts):
            futs.append(cb.submit(p))
            if i % 5 == 0:
                time.sleep(0.005)
        outs = [f.result(10) for f in futs]
    finally:
        cb.stop()
    assert outs == [solo(p, 40) for p in prompts]
    assert cb.completed == 23
    from distributed_lms_raft_llm_amd.utils.metrics import METRICS

    h = METRICS.snapshot()["histograms"]
    assert h["tutor_ttft_ms"]["count"] >= 23 and h["tutor_tpot_ms"]["count"] > 0
    assert 0.0 <= METRICS.snapshot()["gauges"]["tutor_kv_slot_occupancy"] <= 1.0
    assert eng.admitted_while_busy > 0  # requests joined a running batch
    assert max(eng.buckets) <= 4


def test_decode_chunks_capped_by_remaining_budget():
    """A lone request decodes at most one step past its max_length budget (no whole no-op chunk
    at the end of every query): prompt 7, max_length 40 -> 32 decode steps needed."""
    eng = FakeSlotEngine(max_batch=4, max_length=40)
    eng.stop_at_eos = False  # every sequence runs to max_length
    steps = []
    orig = eng.decode

    def decode(B, n, penalty):
        steps.append(n)
        orig(B, n, penalty)

    eng.decode = decode
    cb = ContinuousBatcher(eng, chunk=8)
    try:
        out = cb.submit([1, 2, 3, 4, 5, 6, 7]).result(10)
    finally:
        cb.stop()
    assert len(out) == 40
    need = 40 - 7 - 1
    assert need <= sum(steps) <= need + 1, steps
    assert steps[:4] == [8, 8, 8, 8]


def test_passthrough_and_empty_prompt():
    eng = FakeSlotEngine(max_batch=2, max_length=10)
    cb = ContinuousBatcher(eng)
    try:
        long = list(range(12))
        assert cb.submit(long).result(5) == long
        assert cb.submit([]).result(5) == solo([EOS], 10)
    finally:
        cb.stop()


def test_engine_failure_fails_waiters_and_rejects_new():
    eng = FakeSlotEngine(max_batch=2, max_length=400)
    eng.fail_after = 1
    cb = ContinuousBatcher(eng, chunk=1)
    f = cb.submit([1, 2, 3])
    with pytest.raises(RuntimeError, match="device lost"):
        f.result(5)
    time.sleep(0.05)
    with pytest.raises(RuntimeError):
        cb.submit([1])
    cb.stop()


def test_stop_cancels_pending():
    eng = FakeSlotEngine(max_batch=1, max_length=10 ** 6)
    eng.stop_at_eos = False  # neither request can finish before stop()
    cb = ContinuousBatcher(eng, chunk=1)
    f1 = cb.submit([1])
    f2 = cb.submit([2])
    time.sleep(0.02)
    cb.stop()
    for f in (f1, f2):
        with pytest.raises(RuntimeError):
            f.result(5)


def test_kv_capacity_planner():
    from distributed_lms_raft_llm_amd.engine.memory import GIB, plan_max_batch, slot_bytes
    from distributed_lms_raft_llm_amd.models.config import gpt2_config

    small = gpt2_config("gpt2")
    # KV dominates: 12 layers * 2 * 12 heads * 150 * 64 * 2 B = 5.27 MiB per slot
    assert 5.2 * 2**20 < slot_bytes(small, 150) < 5.5 * 2**20
    assert plan_max_batch(small, 150, free_bytes=287 * GIB, cap=4096) == 4096
    assert plan_max_batch(small, 150, free_bytes=287 * GIB, cap=10**9) == 49152
    assert plan_max_batch(small, 150, free_bytes=8 * GIB) == 256  # 4 GiB reserve + prefill workspace
    xl = gpt2_config("gpt2-xl")
    # 25 heads over 8 ranks: rank 0 holds 4 heads -> the planner sizes for the biggest shard
    assert slot_bytes(xl, 150, 8, 0) > slot_bytes(xl, 150, 8, 7)
    with pytest.raises(MemoryError):
        plan_max_batch(small, 150, free_bytes=1 * GIB)


class AsyncFakeEngine(FakeSlotEngine):
    """Fake whose flags/collect are snapshots taken when requested (like the device copies the
    pipelined loop enqueues) and read later."""

    def flags_async(self, B):
        snap = list(self.fin[:B])
        return SimpleNamespace(result=lambda: snap)

    def collect_async(self, slots):
        snap = [list(self.seqs[s]) for s in slots]
        return SimpleNamespace(result=lambda: snap)


@pytest.mark.parametrize("engine_cls", [FakeSlotEngine, AsyncFakeEngine])
def test_pipelined_loop_readmits_retired_slots_immediately(engine_cls):
    """Two slots, chunk 1, many short requests: a slot retired from chunk k's flags is re-admitted
    while chunk k+1's (stale) flags still call it finished -- the new request must not be retired
    with the old one's flags."""
    eng = engine_cls(max_batch=2, max_length=12)
    cb = ContinuousBatcher(eng, chunk=1)
    try:
        prompts = _prompts(30, seed=7)
        outs = [f.result(10) for f in [cb.submit(p) for p in prompts]]
    finally:
        cb.stop()
    assert outs == [solo(p, 12) for p in prompts]
    assert cb.completed == 30 and eng.admitted_while_busy > 0


def test_stalled_tp_peer_fails_requests_instead_of_returning_garbage():
    """The xGMI barrier's error word is polled once per chunk (``health_async``): when a TP peer
    timed out, every live request fails loudly and the batcher refuses new work."""
    from distributed_lms_raft_llm_amd.engine.scheduler import PeerStalled

    class StallingEngine(FakeSlotEngine):
        def __init__(self):
            super().__init__(max_batch=2, max_length=10 ** 6)
            self.stop_at_eos = False
            self.chunks = 0

        def decode(self, B, steps, penalty):
            super().decode(B, steps, penalty)
            self.chunks += 1

        def health_async(self):
            word = 1 if self.chunks >= 3 else 0  # a peer stalls during the third chunk
            return SimpleNamespace(result=lambda: word)

    eng = StallingEngine()
    cb = ContinuousBatcher(eng, chunk=2)
    f = cb.submit([1, 2, 3])
    with pytest.raises(PeerStalled):
        f.result(10)
    time.sleep(0.05)
    with pytest.raises(RuntimeError):
        cb.submit([4])
    cb.stop()


def test_cancelled_caller_does_not_kill_the_batcher():
    """the aio servicer awaits ``asyncio.wrap_future(batcher.submit(...))`` under
    ``wait_for``; a timeout or client cancel cancels that chain.  A request cancelled while it runs
    must not make ``_retire``'s ``set_result`` raise (which used to fail the batcher and exit the
    replica): its slot is freed and every other request is served."""
    import asyncio

    eng = FakeSlotEngine(max_batch=2, max_length=60)
    eng.stop_at_eos = False
    cb = ContinuousBatcher(eng, chunk=1)

    async def ask(prompt, timeout):
        return await asyncio.wait_for(asyncio.wrap_future(cb.submit(prompt)), timeout)

    async def main():
        res = await asyncio.gather(ask([1, 2], 0.005), ask([3], 0.005), ask([4, 5], 30.0), ask([6], 30.0),
                                   return_exceptions=True)
        return res

    try:
        res = asyncio.run(main())
        assert isinstance(res[0], asyncio.TimeoutError) and isinstance(res[1], asyncio.TimeoutError)
        assert res[2] == solo([4, 5], 60, False) and res[3] == solo([6], 60, False)
        time.sleep(0.1)  # the abandoned requests run to the end and retire
        assert cb.failed is None
        assert cb.submit([7]).result(10) == solo([7], 60, False)
    finally:
        cb.stop()
    assert cb.failed is None


def test_cancelled_while_queued_is_never_admitted():
    eng = FakeSlotEngine(max_batch=1, max_length=30)
    eng.stop_at_eos = False
    cb = ContinuousBatcher(eng, chunk=1)
    try:
        f1 = cb.submit([1])
        f2 = cb.submit([2])  # queued behind f1 (one slot)
        assert f2.cancel()
        assert f1.result(10) == solo([1], 30, False)
        assert cb.submit([3]).result(10) == solo([3], 30, False)
    finally:
        cb.stop()
    assert cb.completed == 2 and cb.failed is None


def test_dataflow_abort_makes_no_progress_and_is_retried():
    """A chunk whose persistent dataflow launch aborted commits no row state (ops/csrc/dataflow.hip):
    the batcher counts it, gives the live requests their step budget back, and the outputs are
    exactly those of an engine that never aborted."""
    from distributed_lms_raft_llm_amd.utils.metrics import METRICS

    class AbortingEngine(AsyncFakeEngine):
        def __init__(self):
            super().__init__(max_batch=2, max_length=40)
            self.stop_at_eos = False
            self.chunks = 0
            self._aborted = False

        def decode(self, B, steps, penalty):
            self.chunks += 1
            self._aborted = self.chunks in (2, 3, 7)
            if self._aborted:  # the launch drained without committing: nothing advanced
                self.buckets.append(B)
                return
            super().decode(B, steps, penalty)

        def dataflow_status_async(self):
            a = self._aborted
            return SimpleNamespace(result=lambda: a)

    before = METRICS.snapshot()["counters"].get("tutor_dataflow_aborts", 0)
    eng = AbortingEngine()
    cb = ContinuousBatcher(eng, chunk=4)
    try:
        prompts = [[1, 2, 3], [9], [4, 4]]
        outs = [f.result(10) for f in [cb.submit(p) for p in prompts]]
    finally:
        cb.stop()
    assert outs == [solo(p, 40, False) for p in prompts]
    assert METRICS.snapshot()["counters"]["tutor_dataflow_aborts"] - before == 3
