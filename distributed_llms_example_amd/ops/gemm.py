"""Weight-gradient GEMM ``dW (+)= dYᵀ X`` on the hand-written gfx950 kernel (csrc/gemm.hip).

Both operands are token-major ([tokens, features]), the reduction runs over tokens (10⁴-10⁵), and the
result is accumulated straight into the flat gradient buffer (bf16, or fp32 for fp32 gradient
accumulation).  Shapes the kernel does not cover (N not a multiple of 256, M not of 8, token counts not
multiples of 64, CPU tensors) go to
``torch.addmm`` (hipBLASLt / CPU BLAS).  ``DLLM_NATIVE_WGRAD=0`` forces the library path (A/B runs).
"""
from __future__ import annotations

import os

import torch

from .. import _ext

_VARIANT = int(os.environ.get("DLLM_WGRAD_VARIANT", "-1"))  # -1: pick by K (csrc/gemm.hip)


def _native_ok(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor) -> bool:
    if os.environ.get("DLLM_NATIVE_WGRAD", "1") == "0" or not _ext.use_native(dy2):
        return False
    return bool(_ext.native().gemm_wgrad_supported(dy2, x2, out))


@torch.no_grad()
def wgrad_accumulate(out: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, beta: bool = True) -> torch.Tensor:
    """``out (+)= dy2ᵀ @ x2`` with dy2 = [T, M], x2 = [T, N], out = [M, N]."""
    if _native_ok(dy2, x2, out):
        _ext.native().gemm_wgrad(dy2, x2, out, beta, _VARIANT, 0)
        return out
    if out.dtype != dy2.dtype:  # fp32 gradient buffer, bf16 operands: library GEMM, then one fp32 add
        g = torch.mm(dy2.t(), x2)
        return out.add_(g) if beta else out.copy_(g)
    if beta:
        return out.addmm_(dy2.t(), x2)
    return torch.mm(dy2.t(), x2, out=out)


@torch.no_grad()
def bias_grad_accumulate(out: torch.Tensor, dy2: torch.Tensor) -> torch.Tensor:
    """``out += dy2.sum(0)`` (bias gradient of a linear layer, accumulated in place)."""
    if _ext.use_native(dy2) and dy2.dtype == torch.bfloat16 and dy2.stride(-1) == 1 and dy2.shape[-1] % 2 == 0 \
            and dy2.stride(0) % 2 == 0 and out.is_contiguous():
        _ext.native().colsum_acc(dy2, out)
        return out
    return out.add_(dy2.sum(0).to(out.dtype))
