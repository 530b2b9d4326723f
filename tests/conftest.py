import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The engine serves GPT-2-124M batch-1 decode with the persistent dataflow kernel by default; the
# engine / serving tests pin the launch-per-op latency path they were written for (several compare
# engines token for token, and the two paths sum in different orders).  tests/test_dataflow_gpu.py
# turns the dataflow path on explicitly and checks it against the fp32 oracle and that path, and
# __graft_entry__.smoke() runs it at batch 1.
os.environ.setdefault("DLMS_DATAFLOW", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running (multi-process clusters)")
    config.addinivalue_line("markers", "multigpu(n): needs n GPUs of one node (skipped when fewer are visible)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        ngpu = torch.cuda.device_count()
        for item in items:
            m = item.get_closest_marker("multigpu")
            if m is not None and ngpu < (m.args[0] if m.args else 2):
                item.add_marker(pytest.mark.skip(reason=f"needs {m.args[0] if m.args else 2} GPUs, {ngpu} visible"))
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
