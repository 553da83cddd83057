"""Embedding lookup whose backward accumulates straight into the flat gradient buffer.

``F.embedding`` forward is a row gather (ATen's vectorized gather kernel is bandwidth-bound already); its
backward is where the work is: ATen scatters into a fresh ``[V, d]`` tensor that AccumulateGrad then adds
into ``p.grad``.  Here the backward sorts the token ids and runs csrc/embed.hip, a deterministic sorted
segment-sum that adds each id's rows, in sorted order, into the parameter's slice of the flat gradient
buffer (bf16 or fp32, parallel/flat.py) — bitwise reproducible, no ``[V, d]`` temporary, and the tied
T5/BART embedding's three contributions (encoder lookup, decoder lookup, LM head) land in one buffer with
the reducer hooks fired once after the last (ops/linear.py ``_use`` / ``_fire``).

Reference: every script builds the model with ``AutoModelForSeq2SeqLM.from_pretrained``
(ref/train-task.py:84, ref/train-accelerator.py:160), whose shared / positional embeddings are
``nn.Embedding`` (BART: ``padding_idx = pad_token_id``, whose row receives no gradient).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext
from .linear import _fire, _fusable, _gbuf, _use


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, padding_idx, params):
        # the Parameter travels inside a tuple: a bare tensor argument would become an autograd input edge
        (param,) = params
        ctx.save_for_backward(ids)
        ctx.param, ctx.padding_idx = param, padding_idx
        _use(param)
        return F.embedding(ids, weight, padding_idx)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        p, pad = ctx.param, ctx.padding_idx
        d = dy.shape[-1]
        dy2 = dy.reshape(-1, d)
        flat_ids = ids.reshape(-1)
        out = _gbuf(p)
        with torch.no_grad():
            if _ext.use_native(dy2) and dy2.dtype == torch.bfloat16 and d % 8 == 0 and d <= 2048:
                if dy2.stride(-1) != 1 or dy2.stride(0) % 8 != 0 or dy2.data_ptr() % 16 != 0:
                    dy2 = dy2.contiguous()
                srt, perm = torch.sort(flat_ids, stable=True)
                _ext.native().embed_bwd(srt, perm, dy2, out, -1 if pad is None else int(pad))
            else:
                g = dy2.to(out.dtype)
                if pad is not None:
                    g = g.masked_fill((flat_ids == pad).unsqueeze(-1), 0)
                out.index_add_(0, flat_ids, g)
        _fire(p)
        return None, None, None, None


def embedding(ids: torch.Tensor, weight: torch.Tensor, padding_idx: int | None = None) -> torch.Tensor:
    """``F.embedding(ids, weight, padding_idx)`` with the gradient accumulated by a native segment-sum."""
    if torch.is_grad_enabled() and _fusable(weight) and weight.requires_grad:
        # a fresh leaf over the weight's storage gives the output a grad_fn (ids carry no gradient) without an
        # edge to the Parameter's AccumulateGrad; its own .grad is never populated (backward returns None)
        return _EmbedFn.apply(ids, weight.detach().requires_grad_(True), padding_idx, (weight,))
    return F.embedding(ids, weight, padding_idx)
