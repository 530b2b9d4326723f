import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The engine's shipped defaults run in every test (batch-1 GPT-2-124M / medium decode on the
# persistent dataflow kernel included); the few tests written for a specific launch-per-op path
# and comparing it token for token pin DLMS_DATAFLOW=0 themselves.


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
