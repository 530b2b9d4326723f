"""Checked (debug) kernel build: ``DLMS_KERNEL_CHECKS=1`` loads libdlms_hip_checked.so, whose kernels
range-check every data-dependent index (token ids, positions, KV slots, lengths) on the device,
record the first violation and clamp the index so the access stays in bounds (SURVEY.md §5.2:
device bounds-check asserts in debug builds).  Runs in a subprocess: the library variant is fixed
when a process first loads it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, torch
from distributed_lms_raft_llm_amd import ops
assert ops.checked_mode()
dev = "cuda"
res = {}
V, P, D = 100, 40, 64
wte = torch.randn(V, D, device=dev).bfloat16()
wpe = torch.randn(P, D, device=dev).bfloat16()

# 1. embed: token 100 is out of [0, 100) -> recorded, row 1 reads wte[0] instead
tok = torch.tensor([3, 100, 7], dtype=torch.int32, device=dev)
pos = torch.tensor([0, 1, 2], dtype=torch.int32, device=dev)
x = ops.embed(tok, pos, wte, wpe)
res["embed"] = ops.device_errors()
res["embed_clamped"] = bool(torch.allclose(x[1], wte[0].float() + wpe[1].float()))

# 2. attention: slot 9 of a 4-slot cache
S, H, T = 4, 2, 32
kc = torch.randn(S, H, T, 64, device=dev).bfloat16()
vc = torch.randn(S, H, T, 64, device=dev).bfloat16()
q = torch.randn(2, H * 64, device=dev).bfloat16()
slot = torch.tensor([1, 9], dtype=torch.int32, device=dev)
kvlen = torch.tensor([5, 5], dtype=torch.int32, device=dev)
ops.row_attention(q, kc, vc, slot, kvlen)
res["attention"] = ops.device_errors()

# 3. QKV GEMM epilogue: position 40 >= t_max 32 in the K/V scatter
d = H * 64
a = torch.randn(2, 64, device=dev).bfloat16()
w = torch.randn(3 * d, 64, device=dev).bfloat16()
qo = torch.empty(2, d, device=dev).bfloat16()
ops.gemm(a, w, ops.EPI_QKV, q_out=qo, k_cache=kc, v_cache=vc, row_slot=torch.tensor([0, 1], dtype=torch.int32, device=dev),
         row_pos=torch.tensor([3, 40], dtype=torch.int32, device=dev))
res["qkv"] = ops.device_errors()

# 4. seen_set: row 5 of a 2-row bitmap
seen = torch.zeros(2, 4, dtype=torch.int32, device=dev)
ops.seen_set(seen, torch.tensor([0, 5], dtype=torch.int32, device=dev), torch.tensor([1, 2], dtype=torch.int32, device=dev))
res["seen"] = ops.device_errors()

# 5. a clean end-to-end decode through every kernel: no violations
from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
from distributed_lms_raft_llm_amd.models.config import GPT2Config
from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights
cfg = GPT2Config("tiny", n_layer=2, n_embd=128, n_head=2, n_positions=64, vocab_size=500, eos_token_id=499)
eng = HipGPT2Engine(cfg, init_gpt2_weights(cfg, seed=1), max_batch=4, max_length=24)
out = eng.generate([[1, 2, 3], [4, 5, 6, 7, 8]])
res["engine_lens"] = [len(o) for o in out]
res["engine"] = ops.device_errors()
print("RESULT " + json.dumps(res))
"""


def test_checked_build_records_and_clamps_bad_indices():
    env = dict(os.environ, DLMS_KERNEL_CHECKS="1", PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-c", SCRIPT], env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert len(res["embed"]) == 1 and "embed token id = 100 not in [0, 100)" in res["embed"][0], res["embed"]
    assert res["embed_clamped"]
    assert len(res["attention"]) == 1 and "attention slot = 9 not in [0, 4)" in res["attention"][0], res["attention"]
    assert len(res["qkv"]) == 1 and "QKV scatter position = 40 not in [0, 32)" in res["qkv"][0], res["qkv"]
    assert len(res["seen"]) == 1 and "seen_set row = 5 not in [0, 2)" in res["seen"][0], res["seen"]
    assert res["engine"] == [] and all(5 <= n <= 24 for n in res["engine_lens"][1:]), res


def test_production_build_has_no_check_records():
    import torch

    from distributed_lms_raft_llm_amd import ops

    if ops.checked_mode():
        pytest.skip("session runs the checked build")
    x = ops.embed(torch.tensor([1, 2], dtype=torch.int32, device="cuda"),
                  torch.tensor([0, 1], dtype=torch.int32, device="cuda"),
                  torch.randn(10, 64, device="cuda").bfloat16(), torch.randn(4, 64, device="cuda").bfloat16())
    assert x.shape == (2, 64)
    assert ops.device_errors() == []
