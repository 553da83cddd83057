"""Tiny driver for rocprofv3 --pmc passes: one projection GEMM through csrc/gemm_fused.hip (no epilogue) and through
hipBLASLt (torch, shipped TunableOp table), a few launches each.

    python tools/gemm_pmc_driver.py [M K N variant]      (default: t5-base encoder QKV at b=128, ping-pong variant 9)

variant "w4": the one-wave-per-SIMD kernel (csrc/gemm_w4.hip), "w4nn": the same with a k-major B (input gradient),
"wg": its weight-gradient mode (c [N, K] fp32 += dy[M, N]^T x[M, K], both operands k-major, split-K), the same FLOPs.
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.utils import tunableop  # noqa: E402

args = sys.argv[1:5] if len(sys.argv) >= 5 else ["131072", "768", "2304", "9"]
M, K, N = (int(v) for v in args[:3])
V = args[3]
tunableop.enable(0)
C = _ext.native()
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
wt = w.t().contiguous()
dy = torch.randn(M, N, device="cuda").to(torch.bfloat16) if V == "wg" else None
c = torch.zeros(N, K, device="cuda") if V == "wg" else None
for _ in range(5):
    if V == "wg":
        C.gemm_wgrad(dy, x, c, True, -1, 0)
    elif V == "w4":
        C.gemm_w4(x, w, False)
        F.linear(x, w)
    elif V == "w4nn":  # x [M, K] . wt [K, N]
        C.gemm_w4(x, wt, True)
        torch.matmul(x, wt)
    else:
        C.gemm_fused(x, w, False, 0, None, None, None, 0.0, 0, int(V))
        F.linear(x, w)
torch.cuda.synchronize()
print("ok", M, K, N, V)
