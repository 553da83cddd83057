import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSFORMERS_NO_ADVISORY_WARNINGS", "true")
os.environ.setdefault("HF_HUB_OFFLINE", "1")
os.environ.setdefault("TRANSFORMERS_OFFLINE", "1")
# the tests' small shapes run the fused FFN kernels (in production FFNs of <= 1024 token rows go unfused, ops/routing.py
# ffn_min_rows; tests/test_model_gpu.py::test_small_ffn_runs_unfused_by_default covers that routing)
os.environ.setdefault("DLLM_ROUTE", "ffn_min_rows=0,wgrad_min_rows=0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the built _C extension")
    config.addinivalue_line("markers", "slow: multi-process or long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
