"""Host side of the persistent dataflow decode (``ops/csrc/dataflow.hip``): per-CU work
assignment, the per-CU packed weight streams, the device tables and the launch.

One launch decodes up to ``nsteps`` greedy steps for 1-2 rows (the reference serves each
student query with its own ``model.generate``: ``tutoring_server.py:21-29``).  Every CU owns
fixed weight rows and streams exactly those, in the order it consumes them, from a private
contiguous region of ``packed`` into an LDS ring; phases hand off through fresh-per-step
counters and tagged granules in ``scratch``.  See the kernel file for the protocol.

Work split over G CUs (``assign``; pure Python so CPU tests check it):
  * W_qkv rows (3d) and LM-head rows (padded vocab) split evenly;
  * the MLP in G / J intermediate slices, each on J CUs that publish 1/J of the c_proj outputs;
  * each head's attention on ``GS`` CUs, each publishing 1/GS of the W_o outputs.
Why the output partitions (round 4): the r3 in-kernel trace (profiles/r3_df_trace_g200_gs2.json)
put the granule edge at 0.27 us of a 19.1 us layer but each residual PUBLISH at 0.92 us and the
two residual edges at 2.9-3.4 us -- the 64-bit counted atomics are issue- and memory-side-bound,
so the fewer residual words a CU adds, the shorter both the publish and the edge behind it.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _check, _stream, lib

P = ctypes.c_void_p


class DfCu(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("q0", "nq", "f0", "nf", "v0", "nv", "ah", "ao0", "aon", "ak0", "akn",
                                            "pd0", "pdn", "acp", "mcp", "lm_off")] + \
               [("off", ctypes.c_longlong), ("step_bytes", ctypes.c_longlong)]


class DfLayer(ctypes.Structure):
    _fields_ = [(n, P) for n in ("ln1_g", "ln1_b", "b_qkv", "b_o", "ln2_g", "ln2_b", "b_fc", "b_p",
                                 "k_cache", "v_cache")]


_INT_FIELDS = ("R", "D", "H", "L", "V", "T", "seen_words", "eos", "nsteps", "A", "C", "max_nq", "swl", "ring_bytes",
               "ldx", "n_slots", "P", "nt_weights", "ko", "kf", "fault_step", "pad_args1", "gather_pause", "spec_rem", "argmax_slots", "pad_args2")


class DfArgs(ctypes.Structure):
    _fields_ = [(n, P) for n in ("packed", "cus", "layers", "wte", "wpe", "lnf_g", "lnf_b", "lens", "finished",
                                 "out_tokens", "seen", "cur_tok", "cur_pos", "cur_kvlen", "slots", "x_out",
                                 "scratch", "err", "trace")] + \
               [("step_words", ctypes.c_longlong)] + [(n, ctypes.c_int) for n in _INT_FIELDS] + \
               [("exp_att", ctypes.c_int * 8), ("exp_mlp", ctypes.c_int * 8)] + \
               [("eps", ctypes.c_float), ("penalty", ctypes.c_float)]


LDS_MAX = 160 * 1024
SUPPORTED_D = (128, 256, 768, 1024)  # GPT-2 small / medium (+ tiny test widths); large / XL measured slower
MAX_ROWS = 2
ERRORS = {1: "arrival-counter wait timed out", 2: "q/k/v granule wait timed out", 3: "LDS hand-off wait timed out",
          4: "weight loader timed out", 5: "injected fault (test hook)"}
NOT_RESIDENT = -2  # dataflow.hip DF_NOT_RESIDENT: the device cannot hold the whole grid at once


class DataflowUnavailable(RuntimeError):
    """The launch was refused before anything ran (the grid cannot be co-resident): serve the
    launch-per-op path instead."""


def _bind_once():
    L = lib()
    if getattr(L, "_df_bound", False):
        return L
    L.dlms_dataflow_decode.argtypes = [ctypes.POINTER(DfArgs), ctypes.c_int, P]
    L.dlms_dataflow_decode.restype = ctypes.c_int
    for n in ("dlms_df_args_size", "dlms_df_cu_size", "dlms_df_layer_size", "dlms_df_threads", "dlms_df_copies"):
        getattr(L, n).restype = ctypes.c_int
    L.dlms_df_lds_fixed.argtypes = [ctypes.c_int] * 4
    L.dlms_df_lds_fixed.restype = ctypes.c_int
    L.dlms_df_step_words.argtypes = [ctypes.c_int] * 4
    L.dlms_df_step_words.restype = ctypes.c_longlong
    for name, st in (("dlms_df_args_size", DfArgs), ("dlms_df_cu_size", DfCu), ("dlms_df_layer_size", DfLayer)):
        if getattr(L, name)() != ctypes.sizeof(st):
            raise RuntimeError(f"{name}: ctypes mirror and compiled library disagree")
    L._df_bound = True
    return L


def split_even(n: int, parts: int, i: int) -> tuple[int, int]:
    base, rem = divmod(n, parts)
    return i * base + min(i, rem), base + (1 if i < rem else 0)


def pad16(n: int) -> int:
    return max(16, -(-n // 16) * 16)


ROW_PAD = 16  # bf16 elements of padding per streamed row (dataflow.hip ROW_BYTES)


@dataclass
class CuPlan:
    q0: int
    nq: int
    f0: int
    nf: int
    v0: int
    nv: int
    pd0: int = 0      # c_proj output columns [pd0, pd0 + pdn) of this CU's intermediate slice
    pdn: int = 0
    mcp: int = 0      # residual copy its MLP contributions go to
    ah: int = -1      # attention head (-1: none) ...
    ao0: int = 0      # ... its W_o output columns [ao0, ao0 + aon) ...
    aon: int = 0
    ak0: int = 0      # ... over the head dims [ak0, ak0 + akn)
    akn: int = 0
    acp: int = 0      # residual copy its attention contributions go to

    def layer_elems(self, d: int, ko: int, kf: int) -> int:
        """bf16 elements of one layer in the stream: W_qkv rows (padded), the K-major W_o block
        [aon][ko] (attention CUs: its output columns x its head dims), the c_fc rows (padded),
        the K-major c_proj block [pdn][kf]."""
        return (self.nq + self.nf) * (d + ROW_PAD) + (self.aon * ko if self.ah >= 0 else 0) + self.pdn * kf

    def step_elems(self, L: int, d: int, ko: int, kf: int) -> int:
        return L * self.layer_elems(d, ko, kf) + self.nv * (d + ROW_PAD)


def block_k(cus: list[CuPlan]) -> tuple[int, int]:
    """(ko, kf): K of the W_o / c_proj blocks, padded to the 16-deep MFMA step (same for all CUs)."""
    return pad16(max((cu.akn for cu in cus), default=16)), pad16(max(cu.nf for cu in cus))


def assign(d: int, n_head: int, n_inner: int, vocab_padded: int, G: int, GS: int, J: int = 1,
           copies: int = 2, attn_split: str = "dims") -> list[CuPlan]:
    """Work of each of G CUs (see module docstring).

    * W_qkv rows and LM-head rows: split evenly over the G CUs.
    * MLP: the intermediate columns are split into I = G / J slices; the J CUs of a slice each
      compute its c_fc rows (the same h) and publish c_proj for 1/J of the output columns -- so a
      CU adds d / J residual words per row instead of d (the per-CU atomic issue and the memory-side
      atomic count of the post-MLP edge shrink J-fold; the extra c_fc rows are prefetched weight
      bytes, off the critical path).  Slice i's contributions go to residual copy i % copies.
    * Attention: each head on GS CUs, each computing the whole head.  ``attn_split="dims"``: CU g
      owns head dims [g 64/GS, (g + 1) 64/GS) of W_o and publishes all d outputs (contribution
      copy a % copies, the round-3 split); ``"outputs"``: it owns all 64 dims and publishes the
      output columns [g d/GS, (g + 1) d/GS) (copy h % copies) -- d / GS atomics per CU instead of
      d.  (The decoder defaults to "outputs": profiles/r4_df_sweep_v4.jsonl.)  Attention CU
      a = h * GS + g sits at CU (a * G) // A, spreading them over all XCDs.
    Every residual word then receives the same number of contributions per copy."""
    if n_head * GS > G or 64 % GS or (attn_split == "outputs" and d % (16 * GS)):
        raise ValueError(f"dataflow: GS={GS} does not split heads over {G} CUs")
    if G % J or d % (16 * J):
        raise ValueError(f"dataflow: J={J} must divide G={G} and d / J must be a multiple of 16")
    I = G // J
    if I > n_inner:
        raise ValueError("dataflow: more MLP slices than intermediate columns")
    cus = []
    for c in range(G):
        q0, nq = split_even(3 * d, G, c)
        i, j = divmod(c, J)
        f0, nf = split_even(n_inner, I, i)
        v0, nv = split_even(vocab_padded, G, c)
        cus.append(CuPlan(q0, nq, f0, nf, v0, nv, pd0=j * (d // J), pdn=d // J, mcp=i % copies))
    A = n_head * GS
    for a in range(A):
        cu = cus[(a * G) // A]
        h, g = divmod(a, GS)
        cu.ah = h
        if attn_split == "outputs":
            cu.ao0, cu.aon, cu.ak0, cu.akn, cu.acp = g * (d // GS), d // GS, 0, 64, h % copies
        else:
            cu.ao0, cu.aon, cu.ak0, cu.akn, cu.acp = 0, d, g * (64 // GS), 64 // GS, a % copies
    return cus


def expected_contributions(cus: list[CuPlan], copies: int) -> tuple[list[int], list[int]]:
    """(attention, MLP) contributions each residual copy's words receive (the same for every word)."""
    att = [0] * copies
    for cu in cus:
        if cu.ah >= 0 and cu.ao0 == 0:  # one CU per head covers any given column; count column 0's
            att[cu.acp] += 1
    mlp = [0] * copies
    for cu in cus:
        if cu.pd0 == 0:
            mlp[cu.mcp] += 1
    return att, mlp


def pack_weights(w, cus: list[CuPlan], device) -> tuple[torch.Tensor, list[int]]:
    """Every CU's stream in one flat bf16 buffer, in the order the kernel consumes it: per layer
    [W_qkv rows | W_o block | c_fc rows | c_proj block], then its LM-head rows (rows padded by
    ROW_PAD).  Returns the buffer and each CU's first element."""
    cfg = w.cfg
    d, L = cfg.n_embd, cfg.n_layer
    ko, kf = block_k(cus)
    sizes = [cu.step_elems(L, d, ko, kf) for cu in cus]
    starts = np.cumsum([0] + sizes)[:-1].tolist()
    packed = torch.zeros(sum(sizes), dtype=torch.bfloat16, device=device)
    pad = lambda t: torch.nn.functional.pad(t, (0, ROW_PAD))  # noqa: E731
    for l, lw in enumerate(w.layers):
        qkv, fc = pad(lw.w_qkv), pad(lw.w_fc)
        for c, cu in enumerate(cus):
            o = starts[c] + l * cu.layer_elems(d, ko, kf)
            pieces = [qkv[cu.q0: cu.q0 + cu.nq].reshape(-1)]
            if cu.ah >= 0:  # W_o[out, in]: outputs [ao0, +aon) x the head dims [ak0, +akn), K padded to ko
                blk = torch.zeros(cu.aon, ko, dtype=torch.bfloat16, device=device)
                k0 = cu.ah * 64 + cu.ak0
                blk[:, : cu.akn] = lw.w_o[cu.ao0: cu.ao0 + cu.aon, k0: k0 + cu.akn]
                pieces.append(blk.reshape(-1))
            pieces.append(fc[cu.f0: cu.f0 + cu.nf].reshape(-1))
            blk = torch.zeros(cu.pdn, kf, dtype=torch.bfloat16, device=device)
            blk[:, : cu.nf] = lw.w_p[cu.pd0: cu.pd0 + cu.pdn, cu.f0: cu.f0 + cu.nf]
            pieces.append(blk.reshape(-1))
            for piece in pieces:
                packed[o: o + piece.numel()].copy_(piece)
                o += piece.numel()
    lm = pad(w.wte)
    for c, cu in enumerate(cus):
        o = starts[c] + L * cu.layer_elems(d, ko, kf)
        packed[o: o + cu.nv * (d + ROW_PAD)].copy_(lm[cu.v0: cu.v0 + cu.nv].reshape(-1))
    return packed, starts


def ring_window(cus: list[CuPlan], d: int, ko: int, kf: int, nc: int = 4) -> int:
    """``DataflowDecoder.ring_window`` for a plan (bytes): the largest piece of the stream some
    compute wave needs resident at once beyond what every wave has released -- the QKV rows, the
    W_o block, the c_fc rows, the c_proj block (the c_fc rows are released before the wait for it)
    or one 16-row LM-head group (each wave releases everything before its next group first)."""
    rowb = 2 * d + 32
    need = 0
    for cu in cus:
        need = max(need, cu.nq * rowb, cu.aon * ko * 2 if cu.ah >= 0 else 0, cu.nf * rowb, cu.pdn * kf * 2,
                   min(cu.nv, 16) * rowb)
    return need


class DataflowDecoder:
    """Persistent dataflow decode bound to one ``HipGPT2Engine`` (TP=1, bf16, 1-2 rows)."""


    @staticmethod
    def supported(eng) -> bool:
        cfg = eng.cfg
        return (eng.tp_size == 1 and not eng.w.fp8 and cfg.n_embd in SUPPORTED_D and cfg.n_embd == 64 * cfg.n_head
                and eng.w.ffn_local == 4 * cfg.n_embd)

    def __init__(self, eng, grid: int | None = None, gs: int | None = None, j: int | None = None,
                 attn_split: str = "outputs"):
        if not self.supported(eng):
            raise ValueError("dataflow decode: TP=1 bf16 GPT-2 with d in %s only" % (SUPPORTED_D,))
        self.L = _bind_once()
        self.COPIES = int(self.L.dlms_df_copies())  # fixed-point residual copies (assign(): acp / mcp)
        self.eng = eng
        cfg, dev = eng.cfg, eng.device
        props = torch.cuda.get_device_properties(dev)
        # 200 of 256 CUs, 2 CUs per head's attention: batch 1 on one box 29.9-30.3 ms against 33.7 at
        # the full grid with 4 per head and 31.6 launch-per-op (profiles/r3_df_sweep_grid200.jsonl,
        # r3_df_sweep_grid_gs.jsonl): fewer contributors per counted residual word shorten the
        # all-to-all edges more than the extra rows per CU lengthen the phases
        cus = int(props.multi_processor_count)
        G = grid or int(os.environ.get("DLMS_DF_GRID", "0")) or min(cus * 25 // 32, 256)
        gs = gs or int(os.environ.get("DLMS_DF_GS", "2"))
        # each head's 2 attention CUs split W_o by OUTPUT columns (d / 2 residual words each): 29.3
        # vs 30.5 ms at batch 1, 40.1 vs 41.4 at batch 2 against the head-dims split on one box
        # (profiles/r4_df_sweep_v4.jsonl); assign(attn_split="dims") keeps the round-3 split for tests
        split = attn_split
        while (cfg.n_head * gs > G or 64 % gs or (split == "outputs" and cfg.n_embd % (16 * gs))) and gs > 1:
            gs //= 2
        # MLP output groups J (see assign; each CU publishes d / J residual words of c_proj): 2 at
        # d 768 -- batch 1 28.7 vs 29.3 ms at J = 1 (profiles/r4_df_sweep_j2_outputs.jsonl; with the
        # head-dims W_o split 32.4 vs 34.2, r4_df_partition_sweep.jsonl) -- 1 at d 1024 (GPT-2-medium
        # 77.7 at J = 1 vs 82.7, r4_df_sweep_medium_j.jsonl: its CUs' c_fc rows double); J = 4
        # duplicates too many c_fc rows (the MLP phase 2.4 -> 4.1 us, r4_df_trace_j4_vs_r3.txt)
        j = j or int(os.environ.get("DLMS_DF_J", "2" if cfg.n_embd <= 768 else "1"))
        while j > 1 and (G % j or -(-eng.w.ffn_local * j // G) > 64 or cfg.n_embd % (16 * j)):
            j -= 1
        self.G, self.GS, self.J = G, gs, j
        self.cus = assign(cfg.n_embd, cfg.n_head, eng.w.ffn_local, cfg.vocab_padded, G, gs, j, self.COPIES, split)
        self.A = cfg.n_head * gs
        self.ko, self.kf = block_k(self.cus)
        if self.ko > 64 or self.kf > 64:
            raise ValueError("dataflow: more than 64 c_proj / W_o columns per CU")
        self.packed, starts = pack_weights(eng.w, self.cus, dev)
        D = cfg.n_embd
        self.max_nq = max(cu.nq for cu in self.cus)
        if self.max_nq > 64:
            raise ValueError("dataflow: more than 64 W_qkv rows per CU")
        max_nv = max(cu.nv for cu in self.cus)
        self.swl = -(-max_nv // 64) * 2 + 2
        tab = (DfCu * G)()
        for c, cu in enumerate(self.cus):
            tab[c] = DfCu(cu.q0, cu.nq, cu.f0, cu.nf, cu.v0, cu.nv, cu.ah, cu.ao0, cu.aon, cu.ak0, cu.akn, cu.pd0,
                          cu.pdn, cu.acp, cu.mcp, cfg.n_layer * cu.layer_elems(D, self.ko, self.kf) * 2, starts[c] * 2,
                          cu.step_elems(cfg.n_layer, D, self.ko, self.kf) * 2)
        self.max_step_bytes = max(cu.step_elems(cfg.n_layer, D, self.ko, self.kf) for cu in self.cus) * 2
        self.cu_tab = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8).to(dev)
        lt = (DfLayer * cfg.n_layer)()
        for l, lw in enumerate(eng.w.layers):
            lt[l] = DfLayer(lw.ln1_g.data_ptr(), lw.ln1_b.data_ptr(), lw.b_qkv.data_ptr(), lw.b_o.data_ptr(),
                            lw.ln2_g.data_ptr(), lw.ln2_b.data_ptr(), lw.b_fc.data_ptr(), lw.b_p.data_ptr(),
                            eng.kv[l, 0].data_ptr(), eng.kv[l, 1].data_ptr())
        self.layer_tab = torch.frombuffer(bytearray(bytes(lt)), dtype=torch.uint8).to(dev)
        # err[0..3]: code, block, step, site of the first abort; err[4]: 1 + steps run once CU 0
        # committed the row state (0: the launch changed no row state -- nothing to undo)
        self.err = torch.zeros(16, dtype=torch.int32, device=dev)
        self._scratch: dict[int, torch.Tensor] = {}
        self.slots = torch.arange(MAX_ROWS, dtype=torch.int32, device=dev)
        # per-launch constants (the continuous batcher launches once per decode chunk)
        self._ring_bytes = {R: self._ring_bytes_for(R) for R in range(1, MAX_ROWS + 1)}
        self._window = ring_window(self.cus, cfg.n_embd, self.ko, self.kf, self.NC)
        self._exp_att, self._exp_mlp = expected_contributions(self.cus, self.COPIES)
        self._fault_step = -1
        self.launches = 0
        self._args = {R: self._args_template(R) for R in range(1, MAX_ROWS + 1)}

    def _args_template(self, R: int) -> DfArgs:
        """The launch arguments that do not change between launches at R rows (the continuous
        batcher launches once per decode chunk: per launch only the step count, penalty, scratch,
        outputs and the test hook are set).  Fixed choices, each measured against its alternative:
          * weight stream non-temporal: batch 1 28.1 -> 27.6-27.7 ms per query, GPT-2-medium 66.5 ->
            65.7-66.0 (profiles/r4_df_nt_ab.jsonl);
          * loaders pause while the comm wave polls a hand-off (MI355X_MICROARCH.md "gather-pass");
          * residual poll: whole-row reads start 4 adds before the watched word completes: batch 1
            28.8 -> 28.2 ms (1 / 2 / 8: 28.6 / 28.4 / 29.0), medium 66.7 -> 65.6
            (profiles/r4_df_spec_poll_sweep.jsonl);
          * per-step argmax through one key slot per CU instead of an atomic max + arrival counter:
            28.2 -> 27.9 ms per query (profiles/r4_df_xf_slots_ab.jsonl)."""
        eng, cfg, w = self.eng, self.eng.cfg, self.eng.w
        a = DfArgs()
        for name, t in (("packed", self.packed), ("cus", self.cu_tab), ("layers", self.layer_tab), ("wte", w.wte),
                        ("wpe", w.wpe), ("lnf_g", w.lnf_g), ("lnf_b", w.lnf_b), ("lens", eng.lens),
                        ("finished", eng.finished), ("out_tokens", eng.out_tokens), ("seen", eng.seen),
                        ("cur_tok", eng.cur_tok), ("cur_pos", eng.cur_pos), ("cur_kvlen", eng.cur_kvlen),
                        ("slots", self.slots), ("err", self.err)):
            setattr(a, name, t.data_ptr())
        a.step_words = self.step_words(R)
        a.R, a.D, a.H, a.L = R, cfg.n_embd, cfg.n_head, cfg.n_layer
        a.V, a.T, a.seen_words, a.eos = cfg.vocab_size, eng.max_length, eng.seen_words, cfg.eos_token_id
        a.A, a.C, a.max_nq, a.swl = self.A, self.COPIES, self.max_nq, self.swl
        a.ring_bytes, a.ldx, a.n_slots, a.P = self.ring_bytes(R), eng.x.stride(0), eng.max_batch, cfg.n_positions
        a.eps = cfg.layer_norm_epsilon
        a.nt_weights = 1
        a.ko, a.kf = self.ko, self.kf
        a.gather_pause = 1
        a.spec_rem = 4
        a.argmax_slots = int(cfg.vocab_size <= 65535 and self.G <= 256)
        for c in range(self.COPIES):  # contributions each fixed-point residual copy receives
            a.exp_mlp[c] = self._exp_mlp[c]
            a.exp_att[c] = self._exp_att[c]
        return a

    def _ring_bytes_for(self, R: int) -> int:
        fixed = self.L.dlms_df_lds_fixed(self.eng.cfg.n_embd, R, self.max_nq, self.swl)
        return (LDS_MAX - fixed) // 8192 * 8192  # a multiple of the loader's 8 KiB batches

    def ring_bytes(self, R: int) -> int:
        return self._ring_bytes[R]

    def inject_fault(self, step: int = 0):
        """Test hook: the NEXT launch aborts at decode step ``step`` of the launch exactly as a
        timed-out hand-off would (the last CU raises the error word, everyone drains)."""
        self._fault_step = int(step)

    NC = 4          # compute waves per CU (dataflow.hip NC)
    BATCH = 8192    # loader batch bytes (dataflow.hip BATCH)

    def ring_window(self) -> int:
        """The most stream bytes a compute wave needs resident beyond the slowest wave's released
        prefix (every wait in dataflow.hip's compute_wave; see ``ring_window`` above).  The loader
        only fetches whole 8 KiB batches that fit behind that prefix, so a launch needs
        ``ring_window() + BATCH <= ring_bytes`` or a wave would wait forever for bytes the loader
        may not fetch (caught as a hand-off timeout)."""
        return self._window

    def fits(self, R: int) -> bool:
        return self._window + self.BATCH <= self._ring_bytes[R]

    def step_words(self, R: int) -> int:
        return int(self.L.dlms_df_step_words(R, self.eng.cfg.n_embd, self.eng.cfg.n_layer, self.COPIES))

    def _scratch_for(self, R: int, nsteps: int) -> torch.Tensor:
        words = self.step_words(R) * nsteps
        buf = self._scratch.get(R)
        if buf is None or buf.numel() < words:
            cap = self.step_words(R) * max(nsteps, self.eng.max_length)
            buf = torch.empty(cap, dtype=torch.int64, device=self.eng.device)
            self._scratch[R] = buf
        return buf

    TRACE_STEPS, TRACE_EV = 4, 32  # dataflow.hip TR_STEPS / TR_EV

    def trace_buffer(self) -> torch.Tensor:
        """A zeroed stamp buffer for ``run(trace=...)``: [G, TRACE_STEPS, L + 1, TRACE_EV] int64
        wall-clock ticks (100 MHz) of each CU's comm wave at fixed points of every phase."""
        L = self.eng.cfg.n_layer
        return torch.zeros(self.G, self.TRACE_STEPS, L + 1, self.TRACE_EV, dtype=torch.int64, device=self.eng.device)

    def run(self, B: int, nsteps: int, penalty: float, x_out: bool = True, trace: torch.Tensor | None = None):
        """``nsteps`` greedy decode steps (at most) of rows [0, B), B <= 2, on the current stream:
        exactly the state transitions of ``nsteps`` launch-per-op steps (decode_update semantics),
        stopping early once every row has finished."""
        eng = self.eng
        if not 1 <= B <= MAX_ROWS or nsteps <= 0:
            raise ValueError(f"dataflow run: B in [1, {MAX_ROWS}], nsteps > 0")
        if not self.fits(B):
            raise ValueError(f"dataflow run: a {self.ring_window()} B stream window does not fit the "
                             f"{self.ring_bytes(B)} B ring at {B} rows (grid {self.G})")
        if nsteps * self.max_step_bytes >= 2 ** 32 - 2 ** 24:
            raise ValueError("dataflow run: too many steps for one launch (32-bit stream offsets)")
        scratch = self._scratch_for(B, nsteps)
        scratch[: self._args[B].step_words * nsteps].zero_()
        self.err.zero_()
        a = DfArgs.from_buffer_copy(self._args[B])
        a.scratch = scratch.data_ptr()
        a.x_out = eng.x.data_ptr() if x_out else None
        a.trace = trace.data_ptr() if trace is not None else None
        a.nsteps, a.penalty = nsteps, float(penalty)
        a.fault_step, self._fault_step = self._fault_step, -1
        rc = self.L.dlms_dataflow_decode(ctypes.byref(a), self.G, _stream())
        if rc == NOT_RESIDENT:
            raise DataflowUnavailable(f"dataflow decode: a grid of {self.G} workgroups cannot be co-resident")
        _check(rc, "dlms_dataflow_decode")
        self.launches += 1

    def status_async(self):
        """The last launch's error words as a copy in flight (``HostResult``; ``.result()`` ->
        (code, block, step, site, committed steps))."""
        from ..engine.gpt2_engine import HostResult

        h = torch.empty(5, dtype=torch.int32, pin_memory=True)
        h.copy_(self.err[:5], non_blocking=True)
        return HostResult(lambda: tuple(h.tolist()), keep=(h,))

    @staticmethod
    def describe(st) -> str:
        return f"dataflow decode: {ERRORS.get(st[0], st[0])} (block {st[1]}, step {st[2]}, site {st[3]})"

    def check(self):
        """Raise if the last launch gave up on a hand-off (synchronises)."""
        st = tuple(self.err[:5].cpu().tolist())
        if st[0]:
            raise RuntimeError(self.describe(st))
