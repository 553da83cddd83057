"""Fused FFN activation (+ gate) (+ dropout).

* T5 v1.0: ``dropout(relu(wi x))`` (transformers modeling_t5.py:83-94)
* flan-T5 / v1.1: ``dropout(gelu_new(wi_0 x) * (wi_1 x))`` (modeling_t5.py:97-123); here wi_0/wi_1
  are one fused GEMM producing ``[..., 2F]`` and this op consumes both halves in one pass.
* BART: ``dropout_p_act(gelu(fc1 x))`` with exact-erf GELU (modeling_bart.py:297-299).

Kernels: csrc/act.hip.  Dropout masks are regenerated in backward from the seed (ops/rng.py).
"""
from __future__ import annotations

import math

import torch

from .. import _ext
from .rng import keep_mask, rowwise_keep_mask

ACTS = {"relu": 0, "gelu": 1, "gelu_new": 2, "gelu_fast": 2, "silu": 3}


def _act_ref(x, act):
    if act == "relu":
        return torch.relu(x)
    if act == "gelu":
        return torch.nn.functional.gelu(x)
    if act in ("gelu_new", "gelu_fast"):
        return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))
    if act == "silu":
        return torch.nn.functional.silu(x)
    raise ValueError(act)


def _reference(x, act, gated, p, seed):
    xf = x.float()
    if gated:
        f = x.shape[-1] // 2
        y = _act_ref(xf[..., :f], act) * xf[..., f:]
    else:
        y = _act_ref(xf, act)
    if p > 0.0:
        y = y * ffn_keep_mask(act, gated, seed, p, y.shape, y.device).to(y.dtype) * (1.0 / (1.0 - p))
    return y.to(x.dtype)


def ffn_keep_mask(act: str, gated: bool, seed: int, p: float, shape, device) -> torch.Tensor:
    """The FFN activation's dropout decisions, as the kernels draw them: the row-Weyl hash of (token row, output column)
    (ops/rng.py rowwise_keep_mask; csrc/common.h rw_* in csrc/gemm_w4.hip, csrc/gemm_fused.hip, csrc/act.hip) for
    every activation, gated or not (``act`` / ``gated`` kept for call sites that name the FFN)."""
    cols = shape[-1]
    rows = 1
    for s in shape[:-1]:
        rows *= s
    return rowwise_keep_mask(seed, p, rows, cols, device).view(shape)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act_id, gated, p, seed):
        C = _ext.native()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        y = C.act_fwd(x2, int(act_id), bool(gated), float(p), int(seed))
        ctx.save_for_backward(x2)
        ctx.cfg = (act_id, gated, p, seed, shape)
        oshape = (*shape[:-1], shape[-1] // 2) if gated else shape
        return y.view(oshape)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.native()
        (x2,) = ctx.saved_tensors
        act_id, gated, p, seed, shape = ctx.cfg
        dx = C.act_bwd(dy.reshape(x2.shape[0], -1), x2, int(act_id), bool(gated), float(p), int(seed))
        return dx.view(shape), None, None, None, None


def act_dropout(x, act: str, p: float = 0.0, seed: int = 0, gated: bool = False):
    if _ext.use_native(x):
        return _ActFn.apply(x, ACTS[act], gated, p, seed)
    return _reference(x, act, gated, p, seed)


def dropout(x, p: float, seed: int):
    """Standalone dropout with the shared counter-based mask (used where no producer kernel exists)."""
    if p <= 0.0:
        return x
    if _ext.use_native(x):
        return _DropoutFn.apply(x, p, seed)
    return x * keep_mask(seed, p, x.shape, x.device).to(x.dtype) * (1.0 / (1.0 - p))


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.cfg = (p, seed)
        return _ext.native().dropout_fwd(x.contiguous(), float(p), int(seed))

    @staticmethod
    def backward(ctx, dy):
        p, seed = ctx.cfg
        return _ext.native().dropout_fwd(dy.contiguous(), float(p), int(seed)), None, None
