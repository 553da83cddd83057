"""Fused (residual + dropout +) RMSNorm / LayerNorm.

T5 is pre-norm with a weight-only RMSNorm in fp32 (transformers modeling_t5.py:50-72, residual +
dropout at :137-141, :400): the residual stream update ``h = h + dropout(sublayer)`` and the next
sub-layer's norm are one kernel here, returning both the new stream ``s`` and ``norm(s)``.
BART is post-norm with a biased LayerNorm (modeling_bart.py:280-308):
``LN(residual + dropout(sublayer))`` is one kernel.  Backward regenerates the dropout mask from
the counter-based seed (ops/rng.py), so no mask is stored.

Kernels: csrc/norm.hip (``norm_fwd`` / ``norm_bwd``).  On CPU (or with DLLM_REFERENCE_OPS=1)
the functions below run the plain-torch reference, which is also the test oracle.
"""
from __future__ import annotations

import torch

from .. import _ext
from . import streams
from . import gemm
from .gemm import colsum_partials_acc, colsum_record
from .linear import _fire, _fusable, _gbuf, _use
from .rng import keep_mask

RMS, LAYER = 0, 1


def _reference(x, resid, weight, bias, eps, p, seed, kind):
    xf = x.float()
    if p > 0.0:
        xf = xf * keep_mask(seed, p, x.shape, x.device).to(xf.dtype) * (1.0 / (1.0 - p))
    s = xf + resid.float() if resid is not None else xf
    s = s.to(x.dtype)
    sf = s.float()
    if kind == RMS:
        rstd = torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps)
        out = sf * rstd * weight.float()
    else:
        mean = sf.mean(-1, keepdim=True)
        var = (sf - mean).pow(2).mean(-1, keepdim=True)
        out = (sf - mean) * torch.rsqrt(var + eps) * weight.float()
        if bias is not None:
            out = out + bias.float()
    return out.to(x.dtype), s


class _NormFn(torch.autograd.Function):
    """out = norm(s) with s = (resid +) dropout(x); returns (out, s)."""

    @staticmethod
    def forward(ctx, x, resid, weight, bias, eps, p, seed, kind, params=None, colsum=False):
        C = _ext.native()
        ctx.params = params
        ctx.colsum = colsum
        for q in params or ():
            _use(q)
        shape = x.shape
        d = shape[-1]
        x2 = x.reshape(-1, d)
        r2 = resid.reshape(-1, d) if resid is not None else None
        out, s, mean, rstd = C.norm_fwd(x2, r2, weight, bias, float(eps), float(p), int(seed), int(kind), True)
        ctx.save_for_backward(s, weight, bias, mean, rstd)
        ctx.cfg = (p, seed, kind, resid is not None, shape)
        ctx.set_materialize_grads(False)
        return out.view(shape), s.view(shape)

    @staticmethod
    def backward(ctx, dout, ds):
        C = _ext.native()
        s, weight, bias, mean, rstd = ctx.saved_tensors
        p, seed, kind, has_resid, shape = ctx.cfg
        d = shape[-1]
        dout2 = dout.reshape(-1, d) if dout is not None else None
        ds2 = ds.reshape(-1, d) if ds is not None else None
        want_stream = has_resid and p > 0.0
        dfr = gemm.deferring() if ctx.params is not None else None
        dx, dstream, dw, db, dxs = C.norm_bwd(dout2, ds2, s, weight, bias, mean, rstd, float(p), int(seed), int(kind),
                                              want_stream, *_acc_targets(ctx.params), want_colsum=ctx.colsum,
                                              partials_only=dfr is not None)
        if dfr is not None:  # deferred window: the weight / bias gradient partials are reduced once per window
            _defer_partials(dfr, ctx.params, dw, db)
            dw = db = None
        dx = dx.view(shape)
        if ctx.colsum:  # handed to the producing linear layer's backward as its bias gradient (ops/gemm.py)
            # with the tensor's version: autograd may add a second consumer's gradient into dx in place, after which
            # the column sum is stale (ops/gemm.py bias_grad_accumulate checks it)
            colsum_record(dx, dxs)
        # d(resid) == d(s) (pre-dropout gradient); identical to dx when p == 0
        dres = None
        if has_resid:
            dres = dstream.view(shape) if want_stream else dx
        streams.pair_join()  # side-stream weight gradients paired with this memory-bound kernel (ops/streams.py)
        return (dx, dres) + _param_grads(ctx.params, weight, bias, dw, db) + (None, None, None, None, None, None)


class _NormOnlyFn(torch.autograd.Function):
    """out = norm(x) (no residual, no dropout)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, kind, params=None):
        C = _ext.native()
        ctx.params = params
        for q in params or ():
            _use(q)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        out, _, mean, rstd = C.norm_fwd(x2, None, weight, bias, float(eps), 0.0, 0, int(kind), False)
        ctx.save_for_backward(x2, weight, bias, mean, rstd)
        ctx.cfg = (kind, shape)
        return out.view(shape)

    @staticmethod
    def backward(ctx, dout):
        C = _ext.native()
        x2, weight, bias, mean, rstd = ctx.saved_tensors
        kind, shape = ctx.cfg
        dx, _, dw, db, _ = C.norm_bwd(dout.reshape(-1, shape[-1]), None, x2, weight, bias, mean, rstd, 0.0, 0,
                                      int(kind), False, *_acc_targets(ctx.params))
        streams.pair_join()
        return (dx.view(shape),) + _param_grads(ctx.params, weight, bias, dw, db) + (None, None, None)


def _defer_partials(dfr, params, dw_part, db_part):
    """Keep this micro-batch's [G, d] partials (no_sync) or reduce them with the kept ones into the flat gradient (the
    window's last micro-batch): one reduction per parameter per window instead of one per micro-batch."""
    for prm, part in ((params[0], dw_part), (params[1], db_part)):
        if prm is None or part is None:
            continue
        out = _gbuf(prm)
        kept = dfr.partials(out, part)
        if kept is not None:
            colsum_partials_acc(out, torch.cat(kept + [part]) if kept else part)


def _acc_targets(params):
    """Flat-buffer gradient views the kernel accumulates into (ops/linear.py: GEMM-fused accumulation)."""
    if params is None:
        return None, None
    w, b = params
    return _gbuf(w), _gbuf(b)


def _param_grads(params, weight, bias, dw, db):
    if params is not None:  # accumulated in place by the kernel; AccumulateGrad never runs for them
        for q in params:
            if q is not None:
                _fire(q)
        return None, None
    return dw.to(weight.dtype), (db.to(bias.dtype) if db is not None else None)


def _norm(x, resid, weight, bias, eps, p, seed, kind, colsum=False):
    if _ext.use_native(x):
        params = None
        if torch.is_grad_enabled() and _fusable(weight) and _fusable(bias):
            params = (weight, bias)
            weight = weight.detach()
            bias = bias.detach() if bias is not None else None
        if resid is None and p == 0.0:
            return _NormOnlyFn.apply(x, weight, bias, eps, kind, params), x
        return _NormFn.apply(x, resid, weight, bias, eps, p, seed, kind, params, colsum and x.requires_grad)
    return _reference(x, resid, weight, bias, eps, p, seed, kind)


def rms_norm(x, weight, eps=1e-6):
    return _norm(x, None, weight, None, eps, 0.0, 0, RMS)[0]


def layer_norm(x, weight, bias, eps=1e-5):
    return _norm(x, None, weight, bias, eps, 0.0, 0, LAYER)[0]


def dropout_rms_norm(x, weight, eps, p, seed):
    """(rms(s)*w, s) with s = dropout(x): T5 embedding dropout fused with block 0's first norm."""
    return _norm(x, None, weight, None, eps, p, seed, RMS)


def add_dropout_rms_norm(resid, x, weight, eps, p, seed):
    """(rms(s)*w, s) with s = resid + dropout(x): T5 residual update fused with the next norm."""
    return _norm(x, resid, weight, None, eps, p, seed, RMS)


def add_dropout_layer_norm(resid, x, weight, bias, eps, p, seed, x_bias_grad=False):
    """LN(resid + dropout(x)): BART post-norm residual block.  ``x_bias_grad``: x is a biased linear layer's output
    (out_proj / fc2); the backward kernel then also sums its gradient over tokens and hands that bias gradient to the
    layer's backward with the gradient tensor (no separate column-sum pass, ops/gemm.py bias_grad_accumulate)."""
    return _norm(x, resid, weight, bias, eps, p, seed, LAYER, x_bias_grad)[0]


def dropout_layer_norm(x, weight, bias, eps, p, seed):
    return _norm(x, None, weight, bias, eps, p, seed, LAYER)[0]


def add_dropout_layer_norm_pre(resid, x, weight, bias, eps, p, seed, x_bias_grad=False):
    """(LN(s), s) with s = resid + dropout(x): a pre-LN residual update fused with the next sub-layer's LayerNorm
    (mBART / Pegasus layers, transformers modeling_mbart.py / modeling_pegasus.py).  ``x_bias_grad`` as in
    ``add_dropout_layer_norm``."""
    return _norm(x, resid, weight, bias, eps, p, seed, LAYER, x_bias_grad)


def dropout_layer_norm_pre(x, weight, bias, eps, p, seed):
    """(LN(s), s) with s = dropout(x): a pre-LN stack's embedding dropout fused with its first LayerNorm."""
    return _norm(x, None, weight, bias, eps, p, seed, LAYER)
