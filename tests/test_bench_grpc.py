"""The open-loop gRPC serving benchmark (scripts/bench_grpc.py) end to end on
the CPU: client processes spawned first, a tutoring server with front-end processes sharing its
port, the host-only null engine; the JSON line carries exact tokens/s from the server counter."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("target", ["tutoring", "lms"])
def test_bench_grpc_null_engine(tmp_path, target):
    out = tmp_path / "serving.jsonl"
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "bench_grpc.py"), "--engine", "null", "--target", target,
           "--rates", "150", "--duration", "3", "--warmup", "1", "--client-procs", "2", "--frontends", "2",
           "--students", "4", "--gate", "off", "--out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads(out.read_text().strip().splitlines()[-1])
    assert line["target"] == ("Tutoring" if target == "tutoring" else "LMS") + ".GetLLMAnswer"
    assert line["failed"] == 0 and line["ok"] > 100
    assert line["tok_s"] > 0 and line["p50_ms"] > 0 and line["p99_ms"] >= line["p50_ms"]
    # null engine: max_length 150 minus the prompt -- every answer is full length
    assert 100 < line["tokens_per_query"] < 150
