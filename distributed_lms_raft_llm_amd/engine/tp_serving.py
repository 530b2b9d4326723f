"""Serving one tensor-parallel engine from one front end ("the tutoring gRPC front
end runs in rank 0 and broadcasts batch metadata per step").

Rank 0 of a TP group owns the gRPC server and the continuous batcher; its engine is wrapped in
``TPEngineProxy``, which broadcasts every state-changing slot call (admit: prompt ids + target
slots; decode: bucket + step count) to the other ranks over a CPU (gloo) control group before
running it locally.  Followers sit in ``serve_follower`` replaying the same calls on their shard,
so every rank enters the same RCCL collectives (inside the same captured decode graphs) in the
same order.  Reads (finished flags, token collection) stay local to rank 0: the vocab-parallel
argmax is all-gathered, so every rank holds identical token state.

Control traffic is one small pickled tuple per scheduler chunk (not per token), off the GPU
stream; the decode data path never leaves RCCL/xGMI.
"""
from __future__ import annotations

import logging

import torch.distributed as dist

log = logging.getLogger("dlms.tp_serving")

_STOP = ("stop",)


class TPEngineProxy:
    """Slot-protocol engine facade for TP rank 0 (see ``engine/scheduler.py``)."""

    def __init__(self, engine, ctrl_group, src: int):
        self.engine = engine
        self.ctrl_group = ctrl_group
        self.src = src  # global rank of the group's front end (this process)
        self._closed = False

    def __getattr__(self, name):  # cfg, max_batch, max_length, device, ...
        return getattr(self.engine, name)

    def _cast(self, cmd: tuple):
        dist.broadcast_object_list([cmd], src=self.src, group=self.ctrl_group)

    def admit(self, prompts, slots, repetition_penalty: float = 1.2):
        self._cast(("admit", [list(p) for p in prompts], list(slots), float(repetition_penalty)))
        self.engine.admit(prompts, slots, repetition_penalty)

    def decode(self, B: int, steps: int, repetition_penalty: float = 1.2):
        self._cast(("decode", int(B), int(steps), float(repetition_penalty)))
        self.engine.decode(B, steps, repetition_penalty)

    def generate(self, prompts, max_length=None, repetition_penalty: float = 1.2, stats=None):
        self._cast(("generate", [list(p) for p in prompts], max_length, float(repetition_penalty)))
        return self.engine.generate(prompts, max_length, repetition_penalty, stats)

    def warm_decode_graphs(self, repetition_penalty: float = 1.2, max_batch: int | None = None):
        """Every rank captures the same decode graphs: each capture's warm-up step runs the TP
        collectives, so rank 0 must never capture alone (its peers would sit in
        ``serve_follower`` waiting for a command while rank 0 waits in the collective)."""
        self._cast(("warm", float(repetition_penalty), max_batch))
        return self.engine.warm_decode_graphs(repetition_penalty, max_batch)

    def finished_flags(self, B: int):
        return self.engine.finished_flags(B)

    def collect(self, slots):
        return self.engine.collect(slots)

    def flags_async(self, B: int):  # rank-0 reads only: nothing to mirror
        from .scheduler import flags_async

        return flags_async(self.engine, B)

    def collect_async(self, slots):
        from .scheduler import collect_async

        return collect_async(self.engine, slots)

    def health_async(self):  # rank 0's own error word: a peer that stalled breaks its barrier too
        from .scheduler import health_async

        return health_async(self.engine)

    def close(self):
        """Release the followers.  Tolerates followers that are already gone (a launcher that
        signals the whole process group stops them before rank 0 gets here)."""
        if not self._closed:
            self._closed = True
            try:
                self._cast(_STOP)
            except RuntimeError as e:
                log.warning("TP followers unreachable at shutdown: %s", e)


def serve_follower(engine, ctrl_group, src: int) -> int:
    """Mirror rank 0's engine calls until it closes; returns the number of commands executed."""
    n = 0
    while True:
        box = [None]
        dist.broadcast_object_list(box, src=src, group=ctrl_group)
        cmd = box[0]
        op = cmd[0]
        if op == "stop":
            return n
        if op == "admit":
            engine.admit(cmd[1], cmd[2], cmd[3])
        elif op == "decode":
            engine.decode(cmd[1], cmd[2], cmd[3])
        elif op == "generate":
            engine.generate(cmd[1], cmd[2], cmd[3])
        elif op == "warm":
            engine.warm_decode_graphs(cmd[1], cmd[2])
        else:
            raise RuntimeError(f"unknown TP control command {op!r}")
        n += 1
