"""Tiny driver for rocprofv3 --pmc passes: one projection GEMM through csrc/gemm_fused.hip (no epilogue) and through
hipBLASLt (torch, shipped TunableOp table), a few launches each.

    python tools/gemm_pmc_driver.py [M K N variant]      (default: t5-base encoder QKV at b=128, ping-pong variant 9)
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.utils import tunableop  # noqa: E402

M, K, N, V = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (131072, 768, 2304, 9)))
tunableop.enable(0)
C = _ext.native()
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
for _ in range(5):
    C.gemm_fused(x, w, False, 0, None, None, None, 0.0, 0, V)
    F.linear(x, w)
torch.cuda.synchronize()
print("ok", M, K, N, V)
