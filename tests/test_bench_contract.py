"""bench.py driver contract on CPU: one JSON line from rank 0 with the required keys, both as a
single process and as 2 data-parallel ranks under torchrun (gloo), where ``value`` is the
whole-job aggregate and the elapsed time is the max over ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}

pytestmark = pytest.mark.timeout(300)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


ARGS = ["--steps", "2", "--warmup", "1", "--prompt-len", "8", "--max-length", "24", "--batch", "2"]


def test_bench_single_process_json_line():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "bench.py", *ARGS], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert KEYS <= set(d), set(KEYS) - set(d)
    assert d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == "dp1" and d["config"]["global_batch"] == 2
    # 2 queries x (24 - 8) new tokens per step
    assert d["new_tokens_per_step"] == 32.0
    assert abs(d["value"] - 32.0 * 1000 / d["ms_per_step"]) / d["value"] < 0.05


def test_bench_two_ranks_under_torchrun():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "bench.py", "--gpus", "2", *ARGS]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = lines[0]
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    assert d["new_tokens_per_step"] == 64.0  # summed over both ranks
    assert abs(d["value"] - 64.0 * 1000 / d["ms_per_step"]) / d["value"] < 0.05


def test_bench_self_launches_ranks_without_torchrun():
    """``bench.py --gpus 2`` with no launcher spawns its two ranks itself (before any GPU call)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS, "--latency-batches", ""], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    assert lines[0]["config"]["parallelism"] == "dp2" and lines[0]["new_tokens_per_step"] == 64.0


def test_bench_rejects_mismatched_world_size():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", WORLD_SIZE="1")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_bench_reports_latency_points():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "bench.py", *ARGS, "--latency-batches", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_lines(p.stdout)[0]
    assert d["p50_query_latency_ms_b1"] > 0 and d["tok_s_b1"] > 0


def test_bench_labels_are_model_correct():
    """Only the BASELINE config (GPT-2-124M, bf16) carries the published metric name's ratio; other
    models report under their own name with vs_baseline null (BASELINE.md has no number for them)."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.metric_for("gpt2") == bench.METRIC
    assert "GPT-2-XL" in bench.metric_for("gpt2-xl") and "124M" not in bench.metric_for("gpt2-xl")
    assert "GPT-2-medium" in bench.metric_for("gpt2-medium")
    assert bench.vs_baseline("gpt2", "bf16", 53.7 * 10) == 10.0
    assert bench.vs_baseline("gpt2-medium", "bf16", 1e5) is None
    assert bench.vs_baseline("gpt2", "fp8", 1e5) is None
    assert "GPT-2-XL" in bench.data_for("gpt2-xl") and "124M" not in bench.data_for("gpt2-xl")
    assert "GPT-2-124M" in bench.data_for("gpt2")
