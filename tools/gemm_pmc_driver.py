"""Tiny driver for rocprofv3 --pmc passes: the t5-base encoder wi GEMM (65536 x 768 -> 3072) through
csrc/gemm_fused.hip (no epilogue, variant 4) and through hipBLASLt, a few launches each."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.utils import tunableop  # noqa: E402

tunableop.enable(0)
C = _ext.native()
x = torch.randn(65536, 768, device="cuda").to(torch.bfloat16)
w = (torch.randn(3072, 768, device="cuda") * 768 ** -0.5).to(torch.bfloat16)
for _ in range(5):
    C.gemm_fused(x, w, False, 0, None, None, None, 0.0, 0, 4)
    F.linear(x, w)
torch.cuda.synchronize()
print("ok")
