"""One-shot collectives over xGMI peer memory for tensor-parallel decode (``ops/csrc/xgmi.hip``).

A TP group of W ranks (one process per GPU) each allocate one uncached HBM buffer, export it as
a hipIpc handle and map every peer's buffer.  ``all_reduce_`` and ``all_gather_u64`` are then
single kernels: copy the local message into the own slab, a per-block flag barrier written
straight into the peers' memory, and a read of all W slabs over the point-to-point xGMI links
(every MI355X has a direct link to each of its 7 peers, so W-1 reads run in parallel; a ring
all-reduce would chain 2(W-1) dependent hops for messages that are only rows x d x 4 bytes).

The call counter and the slab parity live on the device, so the kernels are hipGraph-capturable
and need no host bookkeeping; the sums are taken in rank order, so every rank gets bit-identical
results (the vocab-parallel greedy argmax must agree across ranks).  A barrier that waits for a
peer longer than ~1 s gives up and raises the error word that ``check()`` reports -- the GPU is
never left spinning.

The handle exchange uses ``torch.distributed.all_gather_object`` on the TP group, so it works on
an RCCL group (production) as well as on gloo (the one-GPU functional tests, where two processes
share ``cuda:0`` and map each other's buffers the same way).  The reference has no GPU
collectives at all (gRPC only); this is the §7.2 step 9 "one-shot P2P all-reduce".
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from .. import ops


class XgmiComm:
    def __init__(self, group, device: torch.device | str, slab_bytes: int, cached: bool = False):
        L = ops.lib()
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        if not 1 <= self.world <= ops.XGMI_MAX_RANKS:
            raise ValueError(f"xGMI one-shot collectives support 1..{ops.XGMI_MAX_RANKS} ranks, got {self.world}")
        self.device = torch.device(device)
        self.slab_bytes = int(slab_bytes + 255) // 256 * 256
        self._base = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            ops._check(L.dlms_xgmi_alloc(self.slab_bytes, int(cached), ctypes.byref(self._base)), "dlms_xgmi_alloc")
            h = ctypes.create_string_buffer(L.dlms_ipc_handle_size())
            ops._check(L.dlms_ipc_get_handle(self._base, h), "dlms_ipc_get_handle")
            handles: list = [None] * self.world
            dist.all_gather_object(handles, bytes(h.raw), group=group)
            self._opened: list[ctypes.c_void_p] = []
            bases = []
            for p, hb in enumerate(handles):
                if p == self.rank:
                    bases.append(self._base.value)
                    continue
                ptr = ctypes.c_void_p()
                ops._check(L.dlms_ipc_open(ctypes.create_string_buffer(hb, len(hb)), ctypes.byref(ptr)),
                           f"dlms_ipc_open(rank {p})")
                self._opened.append(ptr)
                bases.append(ptr.value)
        self._bases = (ctypes.c_void_p * ops.XGMI_MAX_RANKS)(*bases)
        # every peer has mapped every buffer before anyone may signal into it
        dist.barrier(group=group)

    def _args(self, inp: torch.Tensor, out: torch.Tensor, n: int) -> ops.XgmiArgs:
        return ops.XgmiArgs(self._bases, inp.data_ptr(), out.data_ptr(), n, self.slab_bytes, self.rank, self.world)

    def fits(self, t: torch.Tensor) -> bool:
        return t.is_contiguous() and t.numel() * t.element_size() <= self.slab_bytes

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group of a contiguous fp32 tensor (numel a multiple of 4)."""
        ops._req(t, torch.float32, "t")
        if not t.is_contiguous() or t.numel() % 4:
            raise ValueError("xgmi all_reduce_: contiguous fp32 with numel % 4 == 0")
        if t.numel() * 4 > self.slab_bytes:
            raise ValueError(f"xgmi all_reduce_: {t.numel() * 4} B exceeds the {self.slab_bytes} B slab")
        if t.device != self.device:
            raise ValueError("xgmi all_reduce_: tensor on another device")
        a = self._args(t, t, t.numel())
        ops._check(ops.lib().dlms_xgmi_allreduce_f32(ctypes.byref(a), ops._stream()), "dlms_xgmi_allreduce_f32")
        return t

    def all_reduce_i64_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place integer sum over the group of a contiguous int64 tensor (even numel): the TP
        fused decode's fixed-point residual partials (exact, identical on every rank)."""
        ops._req(t, torch.int64, "t")
        if not t.is_contiguous() or t.numel() % 2:
            raise ValueError("xgmi all_reduce_i64_: contiguous int64 with an even numel")
        if t.numel() * 8 > self.slab_bytes:
            raise ValueError(f"xgmi all_reduce_i64_: {t.numel() * 8} B exceeds the {self.slab_bytes} B slab")
        if t.device != self.device:
            raise ValueError("xgmi all_reduce_i64_: tensor on another device")
        a = self._args(t, t, t.numel())
        ops._check(ops.lib().dlms_xgmi_allreduce_i64(ctypes.byref(a), ops._stream()), "dlms_xgmi_allreduce_i64")
        return t

    def all_gather_u64(self, src: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """``out[p] = src`` of rank p, for 8-byte elements (int64 packed argmax keys)."""
        ops._req(src, torch.int64, "src", 1)
        ops._req(out, torch.int64, "out", 2)
        n = src.numel()
        if not src.is_contiguous() or not out.is_contiguous() or tuple(out.shape) != (self.world, n):
            raise ValueError(f"xgmi all_gather_u64: out must be contiguous [{self.world}, {n}]")
        if n * 8 > self.slab_bytes:
            raise ValueError("xgmi all_gather_u64: message exceeds the slab")
        a = self._args(src, out, n)
        ops._check(ops.lib().dlms_xgmi_allgather_u64(ctypes.byref(a), ops._stream()), "dlms_xgmi_allgather_u64")
        return out

    def error(self, clear: bool = False) -> int:
        """Non-zero when a barrier timed out waiting for a peer (synchronises the device)."""
        v = ctypes.c_uint()
        with torch.cuda.device(self.device):
            torch.cuda.synchronize()
            ops._check(ops.lib().dlms_xgmi_error(self._base, int(clear), ctypes.byref(v)), "dlms_xgmi_error")
        return v.value

    def error_async(self):
        """The error word as a copy in flight (pinned host memory, enqueued on the current stream
        behind the work issued so far); ``.result()`` waits for that copy only."""
        from ..engine.gpt2_engine import HostResult

        t = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        ops._check(ops.lib().dlms_xgmi_error_async(self._base, ctypes.c_void_p(t.data_ptr()), ops._stream()),
                   "dlms_xgmi_error_async")
        return HostResult(lambda: int(t[0]), keep=(t,))

    def check(self):
        if self.error():
            raise RuntimeError("xGMI collective: a peer never reached the barrier (timed out)")

    def close(self):
        if self._base is None:
            return
        L = ops.lib()
        with torch.cuda.device(self.device):
            torch.cuda.synchronize()
            dist.barrier(group=self.group)  # nobody reads a buffer that is about to go away
            for p in self._opened:
                L.dlms_ipc_close(p)
            self._opened = []
            dist.barrier(group=self.group)
            L.dlms_xgmi_free(self._base)
        self._base = None
