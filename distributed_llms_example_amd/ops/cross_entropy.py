"""Fused (label-smoothed) cross-entropy over the LM-head logits.

Matches ``CrossEntropyLoss(ignore_index=-100)`` used inside T5/BART (transformers
modeling_t5.py:1050-1054, modeling_bart.py:942-946) and the Trainer's LabelSmoother
``(1-eps)*nll + eps*mean_v(-logp_v)`` over non-ignored tokens (trainer_pt_utils.py:437-483).
BART's ``final_logits_bias`` (modeling_bart.py:940) is added inside the kernel instead of
materialising ``logits + bias``.

The forward kernel makes one online-softmax pass per row (fp32 math on bf16 logits) and keeps only
``lse`` per row; the backward kernel writes ``softmax - target`` straight into the logits buffer
(``inplace_grad=True``) so no second ``[N, V]`` tensor is allocated.  Kernels: csrc/ce.hip.
"""
from __future__ import annotations

import torch

from .. import _ext


def _reference(logits, labels, bias, smoothing, ignore_index):
    x = logits.float()
    if bias is not None:
        x = x + bias.float().view(1, -1)
    return torch.nn.functional.cross_entropy(x, labels, ignore_index=ignore_index, label_smoothing=smoothing)


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, bias, smoothing, ignore_index, inplace_grad):
        C = _ext.native()
        loss_rows, lse = C.ce_fwd(logits, labels, bias, float(smoothing), int(ignore_index))
        valid = (labels != ignore_index)
        count = valid.sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, labels, bias, lse, count)
        ctx.cfg = (smoothing, ignore_index, inplace_grad)
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, g):
        C = _ext.native()
        logits, labels, bias, lse, count = ctx.saved_tensors
        smoothing, ignore_index, inplace = ctx.cfg
        scale = (g.float() / count).reshape(1)
        dlogits = C.ce_bwd(scale, logits, labels, lse, bias, float(smoothing), int(ignore_index), bool(inplace))
        return dlogits, None, None, None, None, None


def cross_entropy(logits, labels, *, bias=None, label_smoothing: float = 0.0, ignore_index: int = -100,
                  inplace_grad: bool = False):
    """Mean CE over rows with ``labels != ignore_index``.  logits ``[N, V]``, labels ``[N]``."""
    if _ext.use_native(logits):
        return _CEFn.apply(logits.contiguous(), labels.contiguous(), bias, label_smoothing, ignore_index,
                           inplace_grad)
    return _reference(logits, labels, bias, label_smoothing, ignore_index)
