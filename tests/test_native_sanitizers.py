"""The native tokenizer library under host sanitizers: ASan+UBSan round trips
and a ThreadSanitizer run with 8 threads sharing one handle (ctypes drops the GIL, so gRPC worker
threads really do call into it concurrently).  GPU sanitizers are not available on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "distributed_lms_raft_llm_amd", "native", "csrc", "tokenizers.cpp")
HARNESS = os.path.join(ROOT, "tests", "native", "tokenizer_stress.cpp")

pytestmark = [pytest.mark.timeout(300), pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")]


@pytest.mark.parametrize("san,mode", [("address,undefined", "single"), ("thread", "threads")])
def test_tokenizers_clean_under_sanitizer(tmp_path, san, mode):
    exe = tmp_path / f"stress_{mode}"
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
           SRC, HARNESS, "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), mode], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0 and "failures: 0" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
